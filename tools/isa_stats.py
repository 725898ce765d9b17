#!/usr/bin/env python3
"""Static instruction mix of kernels in the gfx950 device assembly of one
translation unit (hipcc --cuda-device-only -S), for quick A/B of code shapes
before a GPU run.

    python tools/isa_stats.py [--src kernels_n.hip] [--n 8] [--match k_ply] [-D FLAG=1 ...] [--dump DIR]
"""
import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def assemble(src, n, defs, extra=()):
    out = "/tmp/oth_isa_%s_%d.s" % (os.path.basename(src).split(".")[0], n)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
           "-DOTH_N=%d" % n, "--cuda-device-only", "-S", os.path.join(ROOT, "gymothelloenv_amd", "csrc", src),
           "-o", out] + ["-D" + d for d in defs] + list(extra)
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


def kernels(asm):
    res = {}
    meta = {}
    for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n){0,40}?\s+\.sgpr_count:\s+(\d+)\n(?:.*\n){0,12}?\s+\.vgpr_count:\s+(\d+)",
                         asm):
        meta[m.group(1)] = (int(m.group(2)), int(m.group(3)))
    for m in re.finditer(r"^(_Z\S+):\s*;.*$", asm, re.M):
        name = m.group(1)
        end = asm.find(".Lfunc_end", m.end())  # the whole body: block placement may put an s_endpgm mid-function
        body = asm[m.end():end]
        ins = re.findall(r"^\s+([a-z_][a-z0-9_]*)", body, re.M)
        res[name] = (ins, body, meta.get(name))
    return res


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
        return dict(zip(names, out))
    except OSError:
        return {n: n for n in names}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="kernels_n.hip")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--match", default="k_ply")
    ap.add_argument("-D", dest="defs", action="append", default=[])
    ap.add_argument("--top", type=int, default=0)
    ap.add_argument("--dump")
    ap.add_argument("--extra", action="append", default=[])
    a = ap.parse_args()
    ks = kernels(assemble(a.src, a.n, a.defs, a.extra))
    dm = demangle(list(ks))
    for name, (ins, body, meta) in ks.items():
        pretty = dm.get(name, name)
        if a.match not in pretty:
            continue
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith("s_waitcnt"))
        vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_")))
        lds = sum(v for k, v in c.items() if k.startswith("ds_"))
        print("%s  sgpr/vgpr %s  VALU %d  SALU %d  VMEM %d  LDS %d  waitcnt %d  branches %d" % (
            pretty[:90], meta, valu, salu, vmem, lds, c["s_waitcnt"],
            sum(v for k, v in c.items() if k.startswith("s_cbranch"))))
        if a.top:
            for k, v in c.most_common(a.top):
                print("   %5d %s" % (v, k))
        if a.dump:
            os.makedirs(a.dump, exist_ok=True)
            open(os.path.join(a.dump, re.sub(r"[^A-Za-z0-9_]", "_", pretty)[:80] + ".s"), "w").write(body)


if __name__ == "__main__":
    sys.exit(main())
