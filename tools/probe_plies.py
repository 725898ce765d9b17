#!/usr/bin/env python3
"""The per-launch fixed cost of the play kernels: k_play_rand launches of P
plies for P = 1 .. 100 at 65,536 boards (greedy with 0-10-ply openings, config
3; random, config 2), 10 launches per (policy, P) in a fixed order, so that a
rocprofv3 kernel trace of this script gives each group's kernel durations:

    rocprofv3 --kernel-trace --stats -d gpurun_out/x -o plies -- python tools/probe_plies.py
    python tools/probe_plies.py --trace 'gpurun_out/x/**/plies_results.db'

The launch duration against P is a line: its slope the steady ply, its
intercept the fixed cost of a launch (loads, LDS tables, first scan, stores)."""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PLIES = (1, 2, 4, 10, 20, 50, 100)
CASES = (("greedy", 10), ("random", 0))
LAUNCHES = 10


def run(E):
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    for policy, init in CASES:
        env = VecOthelloEnv(E, board_size=8, auto_reset=True, seed=0, device="cuda:0", initial_rand_steps=init)
        env.reset()
        env.step_policy(policy, n_plies=30, record=False)  # mid-game
        for P in PLIES:
            a = torch.empty(P, E, dtype=torch.int32, device="cuda:0")
            r = torch.empty(P, E, dtype=torch.int32, device="cuda:0")
            d = torch.empty(P, E, dtype=torch.uint8, device="cuda:0")
            torch.cuda.synchronize()
            for _ in range(LAUNCHES):
                env.step_policy(policy, n_plies=P, actions=a, rewards=r, dones=d)
            torch.cuda.synchronize()
        env.close()
    print("probe_plies done", flush=True)


def parse(path):
    """Each policy's k_play_rand dispatches in launch order, LAUNCHES per P (a
    one-ply random launch runs k_ply_rand instead and is skipped; the 30-ply
    warm-up runs k_play)."""
    rows = []
    for f in glob.glob(path, recursive=True):
        if f.endswith(".db"):  # rocprofv3's default (rocpd SQLite) output
            import sqlite3
            con = sqlite3.connect(f)
            rows += [(s, n, e - s) for n, s, e in con.execute("select name, start, end from kernels")]
            continue
        with open(f) as fh:
            for row in csv.DictReader(fh):
                s0, e0 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                rows.append((s0, row["Kernel_Name"], e0 - s0))
    rows.sort()
    res = {}
    for policy, tag in (("greedy", "k_play_rand<8, 1>"), ("random", "k_play_rand<8, 0>")):
        durs = [d for _, n, d in rows if tag in n]
        plies = [P for P in PLIES if not (policy == "random" and P == 1)]
        m = {}
        for j, P in enumerate(plies):
            g = sorted(durs[j * LAUNCHES:(j + 1) * LAUNCHES])
            m[P] = g[len(g) // 2] / 1e3
        xs, ys = list(m), [m[p] for p in m]
        n = len(xs)
        mx, my = sum(xs) / n, sum(ys) / n
        slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        res[policy] = {"median_launch_us_by_plies": m, "fit_us_per_ply": slope, "fit_fixed_us": my - slope * mx}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=65536)
    ap.add_argument("--trace")
    a = ap.parse_args()
    if a.trace:
        parse(a.trace)
    else:
        run(a.boards)
