#!/usr/bin/env python3
"""Interleaved A/B of compile-time variants of the observation encoders
(k_observe_w) in ONE process: int64 BOARD and f32 MAKE_STATE into preallocated
tensors, each variant's launches captured in a HIP graph and replayed; every
variant must write the same values (checked first).

    python tools/ab_variants.py --build old=-DOTH_OBS_SMALL_E=0 new=       # here (CPU, hipcc)
    python tools/ab_observe.py old new [--envs 65536,1048576 --launches 50 --rounds 6]   # GPU box

("head" is the shipped library; torch_fill, torch's fill_ of the same tensor, is
timed beside them; --no-check times probes that write other values.)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "gymothelloenv_amd", "variants")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+")
    ap.add_argument("--envs", default="65536,1048576")
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--no-check", action="store_true", help="time variants that write other values (probes)")
    ap.add_argument("--layouts", default="board,make_state")
    ap.add_argument("--dtype", help="one element type for every layout (default: board int64, make_state float32)")
    a = ap.parse_args()
    import torch

    import bench
    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    dev = torch.device("cuda", 0)
    libs = {nm: L.load() if nm == "head" else L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm)) for nm in a.names}
    n = a.board_size
    for E in [int(x) for x in a.envs.split(",")]:
        envs = {nm: VecOthelloEnv(E, board_size=n, auto_reset=True, seed=3, device=dev, lib=lib)
                for nm, lib in libs.items()}
        for env in envs.values():
            env.step_policy("random", n_plies=25, record=False)
        forms = {"board": torch.int64, "make_state": torch.float32}
        for layout in a.layouts.split(","):
            dt = getattr(torch, a.dtype) if a.dtype else forms.get(layout, torch.int8)
            esize = torch.empty(0, dtype=dt).element_size()
            shape = (E, n, n) if layout in ("board", "legal", "absolute") else \
                ((E, 2, n, n) if layout == "board_legal" else (E, 4, n, n))
            bufs = {nm: torch.empty(shape, dtype=dt, device=dev) for nm in a.names}
            ref = None
            for nm, env in envs.items():
                env.observe(layout, dt, out=bufs[nm])
                if ref is None:
                    ref = bufs[nm].clone()
                assert a.no_check or torch.equal(bufs[nm], ref), "variant %s writes other values" % nm
            graphs = {"torch_fill": None}
            for nm, env in envs.items():
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(a.launches):
                        env.observe(layout, dt, out=bufs[nm])
                graphs[nm] = g
            g = torch.cuda.CUDAGraph()  # the store floor: torch's fill_ of the same tensor
            with torch.cuda.graph(g):
                for _ in range(a.launches):
                    bufs[a.names[0]].fill_(1)
            graphs["torch_fill"] = g
            times = {nm: [] for nm in graphs}
            for r in range(a.rounds + 1):
                for nm in graphs:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record()
                    graphs[nm].replay()
                    e1.record()
                    torch.cuda.synchronize()
                    if r:
                        times[nm].append(e0.elapsed_time(e1) * 1e3 / a.launches)
            b = bench.observe_bytes(n, E, layout, esize)
            res = {nm: {"us": statistics.median(t), "GBps": b / (statistics.median(t) * 1e-6) / 1e9}
                   for nm, t in times.items()}
            print(json.dumps({"E": E, "layout": layout, "dtype": str(dt), "bytes": b, "results": res}), flush=True)
            del graphs, bufs


if __name__ == "__main__":
    main()
