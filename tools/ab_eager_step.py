#!/usr/bin/env python3
"""Interleaved A/B of the eager VecOthelloEnv.step host path across compile-time
variants of the library (the host side of oth_step), one process: K eager
calls back to back on 65,536 8x8 boards, wall time per call (the host launch
path bounds it), median of rounds.

    python tools/ab_variants.py --build ggl= direct=-DOTH_STEP_DIRECT=1 --sizes 8   # here
    python tools/ab_eager_step.py ggl direct                                        # GPU box
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "gymothelloenv_amd", "variants")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--calls", type=int, default=3000)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    dev = torch.device("cuda", 0)
    envs = {nm: VecOthelloEnv(a.envs, auto_reset=True, seed=3, device=dev,
                              lib=L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm))) for nm in a.names}
    act = torch.full((a.envs,), 19, dtype=torch.int32, device=dev)  # legal from the start, then the invalid path
    r = torch.empty(a.envs, dtype=torch.int32, device=dev)
    d = torch.empty(a.envs, dtype=torch.uint8, device=dev)
    times = {nm: [] for nm in a.names}
    for rnd in range(a.rounds + 1):
        for nm, env in envs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.calls):
                env.step(act, rewards=r, dones=d, observe=False)
            torch.cuda.synchronize()
            if rnd:
                times[nm].append((time.perf_counter() - t0) / a.calls * 1e6)
    print(json.dumps({"E": a.envs, "calls": a.calls, "results": {nm: {"us_per_call_median": statistics.median(t),
                                                                      "us_per_call_min": min(t)}
                                                                 for nm, t in times.items()}}))


if __name__ == "__main__":
    main()
