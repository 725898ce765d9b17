"""Build liboth_mi355x.so in-tree with hipcc for gfx950 (no JIT cache: the .so
travels with the repo snapshot to the GPU box).

The kernels are templates over the board size N; csrc/kernels_n.hip is
compiled once per N (-DOTH_N=4..16) in parallel, csrc/play_rand_n.hip (the
fused random-play kernels, its own scheduler flags) once per N = 4..11, csrc/capi.hip holds
the C ABI, and the objects are linked into one shared library.

Reproducibility: objects go to a fixed directory (`_objs/`, git-ignored) so the
compiler's per-TU ids (derived from the input path and options) are the same on
every build, and the library embeds the SHA-256 of its sources and flags
(`oth_version()` reports it, `embedded_hash()` reads it from the file).  The
loader refuses a library whose embedded hash is not the hash of the sources in
the tree, so a binary that ran on the GPU box is provably built from HEAD."""
import concurrent.futures
import hashlib
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SIZES = list(range(4, 17))
SOURCES = ("capi.hip", "kernels_n.hip", "play_rand_n.hip", "masked.hip", "device.hpp", "launch.hpp", "bitboard.hpp",
           "masked.hpp", "ply.hpp", "sample_step.hpp", "maximin_wave.hpp")
PLAY_SIZES = list(range(4, 12))  # k_play_rand (one-word boards) and k_play_rand_w (two-word boards)
# play_rand_n.hip: the max-ILP machine scheduler (one wave per SIMD: latency hidden by the schedule
# counts, occupancy does not); the rest of the library keeps the default scheduler
PLAY_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
DEPS = [os.path.join(CSRC, f) for f in SOURCES] + [os.path.join(ROOT, "include", "othello_mi355x.h")]
OUT = os.path.join(HERE, "liboth_mi355x.so")
OBJDIR = os.path.join(HERE, "_objs")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OTH_OFFLOAD_ARCH", "gfx950")
BASE_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-pass-failed"]
_HASH_RE = re.compile(rb"oth-src-sha256:([0-9a-f]{64})")


def play_flags(out=OUT):
    """play_rand_n.hip's scheduler flags: PLAY_FLAGS for the shipped library;
    OTH_PLAY_FLAGS replaces them for the tools' A/B variants (out != OUT) only."""
    if out != OUT and os.environ.get("OTH_PLAY_FLAGS") is not None:
        return os.environ["OTH_PLAY_FLAGS"].split()
    return list(PLAY_FLAGS)


def source_hash(extra_flags=(), out=OUT):
    """SHA-256 over the library's sources (name + bytes) and its build flags."""
    h = hashlib.sha256()
    for p in DEPS:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(" ".join([ARCH] + BASE_FLAGS + play_flags(out) + list(extra_flags)).encode())
    return h.hexdigest()


def embedded_hash(path=OUT):
    """The source hash a built library carries (None if absent or unreadable)."""
    try:
        with open(path, "rb") as f:
            m = _HASH_RE.search(f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def needs_build(out=OUT, extra_flags=()):
    return embedded_hash(out) != source_hash(extra_flags, out)


def _jobs():
    n = os.cpu_count() or 4
    cap = int(os.environ.get("MAX_JOBS", "16"))
    return max(1, min(n, cap, len(SIZES) + 2))


def build(force=False, verbose=True, extra_flags=(), out=OUT, jobs=None, only_sizes=None):
    """only_sizes (A/B variants of the tools, never the shipped library): compile the
    per-N units of these board sizes only and link the other sizes' objects of the
    main build (which must exist) -- a variant of one size in a fraction of the time."""
    if not force and not needs_build(out, extra_flags):
        return out
    assert only_sizes is None or out != OUT, "the shipped library is always built whole"
    digest = source_hash(extra_flags, out)
    objdir = OBJDIR if out == OUT else os.path.join(OBJDIR, os.path.splitext(os.path.basename(out))[0])
    shutil.rmtree(objdir, ignore_errors=True)
    os.makedirs(objdir)
    base = [HIPCC, "--offload-arch=%s" % ARCH] + BASE_FLAGS + ["-I", os.path.join(ROOT, "include")] + list(extra_flags)
    units = [(os.path.join(CSRC, "capi.hip"), os.path.join(objdir, "capi.o"), ['-DOTH_SRC_HASH="%s"' % digest]),
             (os.path.join(CSRC, "masked.hip"), os.path.join(objdir, "masked.o"), [])]
    units += [(os.path.join(CSRC, "kernels_n.hip"), os.path.join(objdir, "kernels_n%d.o" % n), ["-DOTH_N=%d" % n])
              for n in SIZES]
    units += [(os.path.join(CSRC, "play_rand_n.hip"), os.path.join(objdir, "play_rand_n%d.o" % n),
               ["-DOTH_N=%d" % n] + play_flags(out)) for n in PLAY_SIZES]

    def compile_one(u):
        src, obj, defs = u
        cmd = base + defs + ["-c", "-o", obj, src]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, cwd=ROOT)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed: %s\n%s" % (" ".join(cmd), r.stdout))
        return obj

    if verbose:
        print("hipcc %s -> %s (%d units, src %s)" % (" ".join(base[1:]), out, len(units), digest[:16]), flush=True)
    reuse = []
    if only_sizes is not None:
        keep = {"capi.o", "masked.o"} | {"kernels_n%d.o" % n for n in only_sizes} | {"play_rand_n%d.o" % n
                                                                                   for n in only_sizes}
        reuse = [os.path.join(OBJDIR, os.path.basename(u[1])) for u in units if os.path.basename(u[1]) not in keep]
        units = [u for u in units if os.path.basename(u[1]) in keep]
        missing = [o for o in reuse if not os.path.exists(o)]
        if missing:
            raise RuntimeError("only_sizes needs the main build's objects: %s" % missing[:3])
        if embedded_hash(OUT) != source_hash():  # the reused objects must come from these sources
            raise RuntimeError("only_sizes reuses the main build's objects: rebuild %s from the current sources "
                               "first" % OUT)
    with concurrent.futures.ThreadPoolExecutor(jobs or _jobs()) as ex:
        objs = list(ex.map(compile_one, units)) + reuse
    subprocess.check_call([HIPCC, "--offload-arch=%s" % ARCH, "-shared", "-o", out + ".tmp"] + objs, cwd=ROOT)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
