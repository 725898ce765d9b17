#!/usr/bin/env python3
"""The single-ply paths, one launch per ply (run under rocprofv3 for kernel
traces and counter passes; prints one JSON line per case).  Each case is
captured into a HIP graph of P launches and replayed, so the kernels run back
to back as in a training loop (an eager Python loop leaves the GPU idle
between launches); the per-ply time is HIP events around the replay / P.

  step_ext    oth_step (OthelloBaseEnv.step, othello.py:412-462) with external
              device actions: P plies of recorded random play replayed from the
              recording's start state (every action legal, auto-reset; the
              replay must end in the recording's state)
  play1       oth_step_policy(random, 1 ply) (k_ply_rand)
  sample_step oth_sample_step (Policy.act + step in one launch), random logits
  step_obs    oth_step_observe: step_ext with the int64 get_observation from the
              same launch (k_ply_step_obs)
  step_obs_ms the same with f32 make_state
  ss_obs      oth_sample_step_observe: sample_step with the next make_state f32

    python tools/prof_step.py [--envs 65536,1048576] [--plies 32] [--cases step_ext,play1,sample_step]
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
    ap.add_argument("--plies", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
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
        b0, m0, l0 = [t.clone() for t in env.get_state()]
        rew = torch.empty(E, dtype=torch.int32, device=dev)
        don = torch.empty(E, dtype=torch.uint8, device=dev)

        def graphed(name, body, bytes_per_board, reset_state=True, check=None):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), env.graph_region():
                for i in range(P):
                    body(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for rep in range(args.reps):
                if reset_state:
                    env.set_state(b0, m0, l0)
                torch.cuda.synchronize()
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / P
                rec = {"case": name, "E": E, "board_size": n, "rep": rep, "us_per_ply": us,
                       "env_steps_per_s": E / (us * 1e-6), "algorithmic_bytes_per_board": bytes_per_board,
                       "achieved_GBs": E * bytes_per_board / (us * 1e-6) / 1e9, "timing": "graph of %d launches" % P}
                if check is not None and rep == args.reps - 1:
                    rec["check"] = check()
                print(json.dumps(rec), flush=True)
            del g

        if "step_ext" in cases:
            rec_a = torch.empty(P, E, dtype=torch.int32, device=dev)
            rec_r = torch.empty(P, E, dtype=torch.int32, device=dev)
            rec_d = torch.empty(P, E, dtype=torch.uint8, device=dev)
            env.set_state(b0, m0, l0)
            env.step_policy("random", n_plies=P, actions=rec_a, rewards=rec_r, dones=rec_d)
            want = [t.clone() for t in env.get_state()]

            def same():
                ok = all(torch.equal(x, y) for x, y in zip(env.get_state(), want))
                ok = ok and torch.equal(rew, rec_r[-1]) and torch.equal(don, rec_d[-1])
                if not ok:
                    raise SystemExit("step_ext replay differs from the recorded play")
                return "replay_equals_recording"
            graphed("step_ext", lambda i: env.step(rec_a[i], rewards=rew, dones=don, observe=False), 40 * W + 11,
                    check=same)
        if "step_obs" in cases or "step_obs_ms" in cases:
            rec_a = torch.empty(P, E, dtype=torch.int32, device=dev)
            env.set_state(b0, m0, l0)
            env.step_policy("random", n_plies=P, actions=rec_a, record=True)
            for case, lay, dt, per in (("step_obs", "board", torch.int64, 8 * n * n),
                                       ("step_obs_ms", "make_state", torch.float32, 16 * n * n)):
                if case not in cases:
                    continue
                ob = torch.empty((E, n, n) if lay == "board" else (E, 4, n, n), dtype=dt, device=dev)
                graphed(case, lambda i, ob=ob, lay=lay: env.step(rec_a[i], rewards=rew, dones=don, obs=ob,
                                                                 obs_layout=lay), 40 * W + 11 + per)
                del ob
        if "ss_obs" in cases:
            g = torch.Generator(device=dev).manual_seed(0)
            logits = torch.randn(E, n * n, device=dev, generator=g)
            a = torch.empty(E, dtype=torch.int32, device=dev)
            ms = torch.empty(E, 4, n, n, dtype=torch.float32, device=dev)
            graphed("ss_obs", lambda i: env.sample_step(logits, log_probs=False, entropy=False, actions=a,
                                                       rewards=rew, dones=don, observe="make_state", obs=ms),
                    4 * n * n + 40 * W + 11 + 16 * n * n)
            del ms
        if "play1" in cases:
            a1 = torch.empty(1, E, dtype=torch.int32, device=dev)
            graphed("play1", lambda i: env.step_policy("random", n_plies=1, actions=a1, rewards=rew[None],
                                                      dones=don[None]), 40 * W + 11)
        if "sample_step" in cases:
            g = torch.Generator(device=dev).manual_seed(0)
            logits = torch.randn(E, n * n, device=dev, generator=g)
            a = torch.empty(E, dtype=torch.int32, device=dev)
            graphed("sample_step", lambda i: env.sample_step(logits, log_probs=False, entropy=False, actions=a,
                                                            rewards=rew, dones=don), 4 * n * n + 40 * W + 11)
        if "sample_only" in cases or "sample_then_step" in cases:
            g = torch.Generator(device=dev).manual_seed(0)
            logits = torch.randn(E, n * n, device=dev, generator=g)
            if "sample_only" in cases:
                graphed("sample_only", lambda i: env.sample_actions(logits, log_probs=False, entropy=False),
                        4 * n * n + 8 * W + 4, reset_state=False)
            if "sample_then_step" in cases:
                def two(i):
                    a, _, _ = env.sample_actions(logits, log_probs=False, entropy=False)
                    env.step(a, rewards=rew, dones=don, observe=False)
                graphed("sample_then_step", two, 4 * n * n + 40 * W + 11 + 8)
        del env
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
