#!/usr/bin/env python3
"""MaxiMinPolicy(d).get_action for every board (oth_policy_actions) on E
mid-game 8x8 boards (25 plies of random play), `--launches` launches per depth:
the runner for the kernel traces and counter passes of k_maximin_wave (depth >=
3) and the one-lane MaxiMin-2 kernel.  Prints one JSON line per depth.

    rocprofv3 --kernel-trace --stats --output-format csv -d D -o run -- python3 tools/prof_maximin.py
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--board-size", type=int, default=8)
    ap.add_argument("--depths", type=int, nargs="+", default=[2, 3, 4])
    ap.add_argument("--launches", type=int, default=3)
    a = ap.parse_args()
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    dev = torch.device("cuda", 0)
    env = VecOthelloEnv(a.envs, board_size=a.board_size, auto_reset=True, seed=5, device=dev)
    env.step_policy("random", n_plies=25, record=False)
    for d in a.depths:
        pol = "maximin%d" % d
        env.policy_actions(pol)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.launches):
            env.policy_actions(pol)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"policy": pol, "boards": a.envs, "board_size": a.board_size,
                          "us_per_call": e0.elapsed_time(e1) * 1e3 / a.launches}), flush=True)


if __name__ == "__main__":
    main()
