#!/usr/bin/env python3
"""Where the north-star step() time goes at 65,536 8x8 boards (GPU box):

  graph_step      oth_step (k_ply_step) replayed from a HIP graph of P launches
  graph_copy      torch copies moving the same bytes per ply (30 B read + 31 B
                  written per board, two tensors) in a graph: the memory floor
  graph_tiny      a one-element torch add per launch in a graph: the launch floor
  eager_step      VecOthelloEnv.step(..., observe=False) in a Python loop
  eager_ctypes    the bare ctypes oth_step call in a Python loop
  eager_tiny      a one-element torch add in a Python loop (torch's own launch path)

    python tools/probe_step.py [--envs 65536 --plies 64]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--plies", type=int, default=64)
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    dev = torch.device("cuda", 0)
    E, P = a.envs, a.plies
    env = VecOthelloEnv(E, board_size=8, auto_reset=True, seed=7, device=dev)
    env.step_policy("random", n_plies=30, record=False)
    b0, m0, l0 = [t.clone() for t in env.get_state()]
    acts = torch.empty(P, E, dtype=torch.int32, device=dev)
    env.step_policy("random", n_plies=P, actions=acts, rewards=torch.empty_like(acts),
                    dones=torch.empty(P, E, dtype=torch.uint8, device=dev))
    rew = torch.empty(E, dtype=torch.int32, device=dev)
    don = torch.empty(E, dtype=torch.uint8, device=dev)
    src = torch.empty(E * 30 // 4, dtype=torch.int32, device=dev)
    dst = torch.empty(E * 31 // 4, dtype=torch.int32, device=dev)
    tiny = torch.zeros(1, device=dev)
    stream = torch.cuda.current_stream(dev)

    def timed(fn, per):
        out = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) * 1e3 / per)
        return statistics.median(out)

    def graph(body):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(P):
                body(i)
        return g
    res = {}
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), env.graph_region():
        for i in range(P):
            env.step(acts[i], rewards=rew, dones=don, observe=False)

    def rep_step():
        env.set_state(b0, m0, l0)
        torch.cuda.synchronize()
        return timed(g.replay, P)
    res["graph_step"] = statistics.median([rep_step() for _ in range(3)])
    gc = graph(lambda i: dst[:src.numel()].copy_(src))
    res["graph_copy"] = timed(gc.replay, P)
    gt = graph(lambda i: tiny.add_(1.0))
    res["graph_tiny"] = timed(gt.replay, P)
    env.set_state(b0, m0, l0)

    def eager_step():
        for i in range(P):
            env.step(acts[i], rewards=rew, dones=don, observe=False)
    eager_step()
    env.set_state(b0, m0, l0)
    res["eager_step"] = timed(eager_step, P)
    fn, h = env._step_fn, env._hv
    ptrs = [(acts[i].data_ptr(), rew.data_ptr(), don.data_ptr()) for i in range(P)]
    raw = torch._C._cuda_getCurrentRawStream

    def eager_ctypes():
        for pa, pr, pd in ptrs:
            fn(h, pa, pr, pd, raw(0))
    env.set_state(b0, m0, l0)
    res["eager_ctypes"] = timed(eager_ctypes, P)

    def eager_tiny():
        for _ in range(P):
            tiny.add_(1.0)
    res["eager_tiny"] = timed(eager_tiny, P)
    print(json.dumps({"E": E, "plies": P, "us_per_launch": res}), flush=True)


if __name__ == "__main__":
    main()
