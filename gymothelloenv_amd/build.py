"""Build liboth_mi355x.so in-tree with hipcc for gfx950 (no JIT cache: the .so
travels with the repo snapshot to the GPU box).

The kernels are templates over the board size N; csrc/kernels_n.hip is
compiled once per N (-DOTH_N=4..16) in parallel, csrc/capi.hip holds the C
ABI, and the objects are linked into one shared library."""
import concurrent.futures
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SIZES = list(range(4, 17))
DEPS = [os.path.join(CSRC, f) for f in ("capi.hip", "kernels_n.hip", "masked.hip", "device.hpp", "launch.hpp", "bitboard.hpp")] + \
    [os.path.join(ROOT, "include", "othello_mi355x.h")]
OUT = os.path.join(HERE, "liboth_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OTH_OFFLOAD_ARCH", "gfx950")


def needs_build(out=OUT):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in DEPS)


def _jobs():
    n = os.cpu_count() or 4
    cap = int(os.environ.get("MAX_JOBS", "16"))
    return max(1, min(n, cap, len(SIZES) + 2))


def build(force=False, verbose=True, extra_flags=(), out=OUT, jobs=None):
    if not force and not needs_build(out):
        return out
    objdir = tempfile.mkdtemp(prefix="oth_objs_")
    base = [HIPCC, "--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-pass-failed", "-I", os.path.join(ROOT, "include")] + list(extra_flags)
    units = [(os.path.join(CSRC, "capi.hip"), os.path.join(objdir, "capi.o"), []),
             (os.path.join(CSRC, "masked.hip"), os.path.join(objdir, "masked.o"), [])]
    units += [(os.path.join(CSRC, "kernels_n.hip"), os.path.join(objdir, "kernels_n%d.o" % n), ["-DOTH_N=%d" % n])
              for n in SIZES]

    def compile_one(u):
        src, obj, defs = u
        cmd = base + defs + ["-c", "-o", obj, src]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed: %s\n%s" % (" ".join(cmd), r.stdout))
        return obj

    if verbose:
        print("hipcc %s -> %s (%d units, %s)" % (" ".join(base[1:]), out, len(units), objdir), flush=True)
    try:
        with concurrent.futures.ThreadPoolExecutor(jobs or _jobs()) as ex:
            objs = list(ex.map(compile_one, units))
        subprocess.check_call([HIPCC, "--offload-arch=%s" % ARCH, "-shared", "-o", out + ".tmp"] + objs)
        os.replace(out + ".tmp", out)
    finally:
        shutil.rmtree(objdir, ignore_errors=True)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
