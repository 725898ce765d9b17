#!/usr/bin/env python3
"""Floor of the observation writes at small launches: oth_observe (k_observe_w)
against torch's own fill_ and copy_ of a tensor of the same shape and dtype, each
as a HIP graph of `--launches` launches (median of 5 replays), so the figure a
write of this many bytes reaches on this box is beside ours.

    python tools/probe_obs.py [--envs 65536,262144] [--launches 50]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def graphed_us(torch, fn, launches):
    for _ in range(3):
        fn()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(launches):
            fn()
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / launches)
    del g
    return statistics.median(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", default="65536,262144")
    ap.add_argument("--launches", type=int, default=50)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    dev = torch.device("cuda", 0)
    n = 8
    for E in [int(x) for x in a.envs.split(",")]:
        env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=3, device=dev)
        env.step_policy("random", n_plies=25, record=False)
        for layout, dt, planes in (("board", torch.int64, 1), ("make_state", torch.float32, 4)):
            shape = (E, n, n) if planes == 1 else (E, planes, n, n)
            buf = torch.empty(shape, dtype=dt, device=dev)
            src = torch.ones(shape, dtype=dt, device=dev)
            nbytes = buf.numel() * buf.element_size()
            rows = {"observe": lambda: env.observe(layout, dt, out=buf), "torch_fill": lambda: buf.fill_(1),
                    "torch_copy": lambda: buf.copy_(src)}
            for name, fn in rows.items():
                torch.cuda.synchronize()
                us = graphed_us(torch, fn, a.launches)
                moved = nbytes * (2 if name == "torch_copy" else 1)
                print(json.dumps({"E": E, "layout": layout, "dtype": str(dt), "op": name, "us": us,
                                  "bytes_written": nbytes, "GBs_written": nbytes / us / 1e3,
                                  "GBs_moved": moved / us / 1e3}), flush=True)
            del buf, src
        env.close()


if __name__ == "__main__":
    main()
