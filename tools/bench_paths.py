#!/usr/bin/env python3
"""Side measurements of every batched entry point at 65,536 boards (8x8 by
default): per call average over back-to-back calls on one stream (HIP events),
algorithmic HBM bytes per call and the implied GB/s.  Run under rocprofv3
--kernel-trace --stats to split launch overhead from kernel time.

    python tools/bench_paths.py [--envs 65536] [--board-size 8] [--iters 200]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    from gymothelloenv_amd.vec_env import nwords
    E, n = args.envs, args.board_size
    W = nwords(n)
    state = 2 * (16 * W + 2 + 8 * W)  # boards + meta + legal, read and written
    dev = torch.device("cuda", 0)
    env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=0, device=dev)
    env.reset()
    env.step_policy("random", n_plies=20, record=False)
    g = torch.Generator(device=dev).manual_seed(0)
    acts = torch.empty(E, dtype=torch.int32, device=dev)
    rew = torch.empty(E, dtype=torch.int32, device=dev)
    don = torch.empty(E, dtype=torch.uint8, device=dev)
    prot = torch.ones(E, dtype=torch.int8, device=dev)
    logits = torch.randn(E, n * n, device=dev, generator=g)
    obs8 = torch.empty(E, 4, n, n, dtype=torch.float32, device=dev)
    legal = torch.empty(E, W, dtype=torch.int64, device=dev)

    def sampled(step):
        def fn():
            a, _, _ = env.sample_actions(logits, log_probs=False, entropy=False)
            step(a)
        return fn

    cases = [
        ("step_policy random, 1 ply/launch", lambda: env.step_policy("random", n_plies=1, actions=acts[None],
                                                                        rewards=rew[None], dones=don[None]),
         state + 9),
        ("sample_actions (masked categorical)", lambda: env.sample_actions(logits), 4 * n * n + 8 * W + 12),
        ("sample_actions + step", sampled(lambda a: env.step(a, rewards=rew, dones=don, observe=False)),
         4 * n * n + 8 * W + 4 + state + 4 + 5),
        ("sample_actions + step_vs random opponent",
         sampled(lambda a: env.step_vs(a, opponent="random", protagonist=prot, observe=False)),
         4 * n * n + 8 * W + 4 + state + 4 + 1 + 9 + 4),
        ("sample_actions + step_vs greedy opponent",
         sampled(lambda a: env.step_vs(a, opponent="greedy", protagonist=prot, observe=False)),
         4 * n * n + 8 * W + 4 + state + 4 + 1 + 9 + 4),
        ("observe make_state f32", lambda: env.observe("make_state", torch.float32, out=obs8),
         16 * W + 2 + 8 * W + 4 * 4 * n * n),
        ("legal_mask", lambda: env._lib.oth_legal(env._h, ctypes.c_void_p(legal.data_ptr()), env._stream()),
         16 * W),
        ("policy_actions greedy", lambda: env.policy_actions("greedy"), 16 * W + 2 + 8 * W + 4),
    ]
    for name, fn, bytes_per_board in cases:
        if "step_vs" in name:
            env.reset_vs(opponent="random", protagonist=prot)
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        print(json.dumps({"path": name, "E": E, "board_size": n, "us_per_call": us, "boards_per_s": E / (us * 1e-6),
                          "algorithmic_bytes_per_board": bytes_per_board,
                          "achieved_GBs": E * bytes_per_board / (us * 1e-6) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
