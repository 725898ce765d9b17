"""Build liboth_mi355x.so in-tree with hipcc for gfx950 (no JIT cache: the .so
travels with the repo snapshot to the GPU box)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", "othello_kernels.hip")]
DEPS = SRC + [os.path.join(HERE, "csrc", "bitboard.hpp"), os.path.join(ROOT, "include", "othello_mi355x.h")]
OUT = os.path.join(HERE, "liboth_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OTH_OFFLOAD_ARCH", "gfx950")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in DEPS)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC, "--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-I", os.path.join(ROOT, "include"), "-o", OUT + ".tmp"] + SRC
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
