#!/usr/bin/env python3
"""Interleaved A/B of compile-time variants on the single-ply external-action
path (oth_policy_actions greedy -> oth_step, both Solo-engine kernels), one
process, HIP events; every variant must produce identical actions first.

    python tools/ab_variants.py --build a= b=-DOTH_SOLO_U32=0     # here
    python tools/ab_step.py a b [--envs 65536 --iters 200 --rounds 6]   # GPU box
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
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import _lib as L
    from gymothelloenv_amd.vec_env import VecOthelloEnv
    envs = {}
    for nm in a.names:
        lib = L.load_path(os.path.join(VDIR, "liboth_%s.so" % nm))
        envs[nm] = VecOthelloEnv(a.envs, board_size=a.board_size, auto_reset=True, seed=0, device="cuda:0", lib=lib,
                                 initial_rand_steps=10)
        envs[nm].reset()
    rew = torch.empty(a.envs, dtype=torch.int32, device="cuda:0")
    don = torch.empty(a.envs, dtype=torch.uint8, device="cuda:0")

    def one(env):
        act = env.policy_actions("greedy")
        env.step(act, rewards=rew, dones=don, observe=False)
        return act

    ref = None
    for nm, env in envs.items():  # identical trajectories
        acts = torch.stack([one(env) for _ in range(50)])
        if ref is None:
            ref = acts
        assert torch.equal(acts, ref), "variant %s differs" % nm
    times = {nm: [] for nm in envs}
    for _ in range(a.rounds):
        for nm, env in envs.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                one(env)
            e1.record()
            torch.cuda.synchronize()
            times[nm].append(e0.elapsed_time(e1) * 1e3 / a.iters)
    print(json.dumps({"path": "policy_actions greedy + step", "E": a.envs, "N": a.board_size,
                      "results": {nm: {"us_per_ply_median": statistics.median(t), "us_per_ply_min": min(t)}
                                  for nm, t in times.items()}}))


if __name__ == "__main__":
    main()
