#!/usr/bin/env python3
"""Device assembly of every translation unit of the library (the build's own
flags, --cuda-device-only -S) with comments and path/ident lines stripped, one
file per unit, for checking that a source cleanup leaves the generated code
unchanged:

    python tools/isa_snapshot.py /tmp/isa_before
    ... edit ...
    python tools/isa_snapshot.py /tmp/isa_after && diff -r /tmp/isa_before /tmp/isa_after
"""
import concurrent.futures
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gymothelloenv_amd import build as B  # noqa: E402


def units():
    u = [("capi.hip", "capi", []), ("masked.hip", "masked", [])]
    u += [("kernels_n.hip", "kernels_n%d" % n, ["-DOTH_N=%d" % n]) for n in B.SIZES]
    u += [("play_rand_n.hip", "play_rand_n%d" % n, ["-DOTH_N=%d" % n] + B.play_flags()) for n in B.PLAY_SIZES]
    return u


def clean(text):
    out = []
    for line in text.splitlines():
        s = line.split(";", 1)[0].rstrip() if not line.lstrip().startswith(".") else line.rstrip()
        if not s or s.lstrip().startswith((".ident", ".file", ".amdgpu_hsa", "//")):
            continue
        if "oth-src-sha256" in s or "__hip_cuid" in s:
            continue
        out.append(s)
    return "\n".join(out) + "\n"


def one(u, outdir):
    src, name, defs = u
    tmp = os.path.join(outdir, name + ".raw.s")
    cmd = [B.HIPCC, "--offload-arch=%s" % B.ARCH] + B.BASE_FLAGS + ["-I", os.path.join(ROOT, "include")] + defs + \
        ['-DOTH_SRC_HASH="0"', "--cuda-device-only", "-S", "-o", tmp, os.path.join(B.CSRC, src)]
    subprocess.run(cmd, check=True, cwd=ROOT)
    txt = open(tmp).read()
    os.remove(tmp)
    with open(os.path.join(outdir, name + ".s"), "w") as f:
        f.write(clean(txt))
    return name


def main():
    outdir = sys.argv[1]
    os.makedirs(outdir, exist_ok=True)
    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        for name in ex.map(lambda u: one(u, outdir), units()):
            print(name, flush=True)


if __name__ == "__main__":
    main()
