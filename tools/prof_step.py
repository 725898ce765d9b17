#!/usr/bin/env python3
"""The single-ply paths one launch per ply (run under rocprofv3 for kernel
traces and counter passes; prints one JSON line per case with HIP-event times).

  step_ext    oth_step (OthelloBaseEnv.step, othello.py:412-462) with external
              device actions: P plies of recorded random play replayed one
              launch per ply from the recording's start state (every action
              legal, auto-reset; the replay must end in the recording's state)
  play1       oth_step_policy(random, 1 ply) -- k_play_rand, one ply per launch
  sample_step oth_sample_step (Policy.act + step in one launch), random logits

    python tools/prof_step.py [--envs 65536,1048576] [--plies 64] [--cases step_ext,play1,sample_step]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", default="65536,1048576")
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--plies", type=int, default=64)
    ap.add_argument("--cases", default="step_ext,play1,sample_step")
    args = ap.parse_args()
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    dev = torch.device("cuda", 0)
    n, P = args.board_size, args.plies
    W = (n * n + 63) // 64
    cases = args.cases.split(",")
    for E in [int(x) for x in args.envs.split(",")]:
        env = VecOthelloEnv(E, board_size=n, auto_reset=True, seed=7, device=dev)
        env.step_policy("random", n_plies=30, record=False)  # mid-game mix of boards
        rew = torch.empty(E, dtype=torch.int32, device=dev)
        don = torch.empty(E, dtype=torch.uint8, device=dev)
        acts1 = torch.empty(1, E, dtype=torch.int32, device=dev)

        def timed(name, fn, iters, bytes_per_board, extra=None):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(iters):
                fn(i)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / iters
            rec = {"case": name, "E": E, "board_size": n, "us_per_ply": us, "env_steps_per_s": E / (us * 1e-6),
                   "algorithmic_bytes_per_board": bytes_per_board,
                   "achieved_GBs": E * bytes_per_board / (us * 1e-6) / 1e9}
            rec.update(extra or {})
            print(json.dumps(rec), flush=True)

        if "step_ext" in cases:
            b0, m0, l0 = env.get_state()
            ply0 = env.ply_counter
            rec_a = torch.empty(P, E, dtype=torch.int32, device=dev)
            rec_r = torch.empty(P, E, dtype=torch.int32, device=dev)
            rec_d = torch.empty(P, E, dtype=torch.uint8, device=dev)
            env.step_policy("random", n_plies=P, actions=rec_a, rewards=rec_r, dones=rec_d)
            b1, m1, l1 = env.get_state()
            for rep in range(3):  # first replay warms up; the last is checked
                env.set_state(b0, m0, l0)
                env.ply_counter = ply0
                timed("step_ext", lambda i: env.step(rec_a[i], rewards=rew, dones=don, observe=False), P,
                      40 * W + 11, {"rep": rep})
            b2, m2, l2 = env.get_state()
            same = bool(torch.equal(b1, b2) and torch.equal(m1, m2) and torch.equal(l1, l2) and
                        torch.equal(rew, rec_r[-1]) and torch.equal(don, rec_d[-1]))
            print(json.dumps({"case": "step_ext_check", "E": E, "replay_equals_recording": same}), flush=True)
            if not same:
                raise SystemExit("step_ext replay differs from the recorded play")
        if "play1" in cases:
            for rep in range(2):
                timed("play1", lambda i: env.step_policy("random", n_plies=1, actions=acts1, rewards=rew[None],
                                                         dones=don[None]), P, 40 * W + 11, {"rep": rep})
        if "sample_step" in cases:
            g = torch.Generator(device=dev).manual_seed(0)
            logits = torch.randn(E, n * n, device=dev, generator=g)
            a = torch.empty(E, dtype=torch.int32, device=dev)
            for rep in range(2):
                timed("sample_step", lambda i: env.sample_step(logits, log_probs=False, entropy=False, actions=a,
                                                               rewards=rew, dones=don), P,
                      4 * n * n + 40 * W + 11, {"rep": rep})
        del env
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
