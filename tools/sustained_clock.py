#!/usr/bin/env python3
"""The headline kernel (k_play_rand<8, random>, 65,536 boards, every per-ply
output stored) launched back to back for `--seconds`, for the bench's
`sustained` line and its effective clock:

    python tools/sustained_clock.py [--plies 100 --seconds 3]
    rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d D -o run -- \
        python3 tools/sustained_clock.py --plies 1000 --seconds 3
    python tools/sustained_clock.py --summarize D --plies 1000     # -> effective clock (GHz)

The effective clock is GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) over the
dispatch's duration (MI355X_MICROARCH.md, 'DVFS give-back'), averaged over the
dispatches of the second half of the run; the quotient reads high on dispatches
shorter than about 0.3 ms, hence 1,000-ply launches (~0.7 ms) for the clock."""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(plies, seconds, E):
    import torch

    from gymothelloenv_amd import VecOthelloEnv
    dev = torch.device("cuda", 0)
    env = VecOthelloEnv(E, board_size=8, auto_reset=True, seed=0, device=dev)
    env.reset()
    a = torch.empty(plies, E, dtype=torch.int32, device=dev)
    r = torch.empty(plies, E, dtype=torch.int32, device=dev)
    d = torch.empty(plies, E, dtype=torch.uint8, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    env.step_policy("random", n_plies=plies, actions=a, rewards=r, dones=d)
    torch.cuda.synchronize()
    e0.record()
    env.step_policy("random", n_plies=plies, actions=a, rewards=r, dones=d)
    e1.record()
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) * 1e-3
    k = max(10, int(seconds / per))
    e0.record()
    for _ in range(k):
        env.step_policy("random", n_plies=plies, actions=a, rewards=r, dones=d)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / k
    print(json.dumps({"plies": plies, "boards": E, "launches": k, "seconds": k * us * 1e-6, "avg_launch_us": us,
                      "us_per_ply": us / plies, "env_steps_per_s": E * plies / (us * 1e-6)}))


def summarize(d, kernel="k_play_rand"):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel in row["Kernel_Name"]:
                rows.append(row)
    by = {}
    for row in rows:
        key = row.get("Dispatch_Id") or row.get("Correlation_Id")
        rec = by.setdefault(key, {"dur": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
        rec[row["Counter_Name"]] = rec.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    ds = [by[k] for k in sorted(by, key=lambda x: int(x))]
    ds = ds[len(ds) // 2:]  # the second half: the chip under sustained load
    clocks = [r["GRBM_GUI_ACTIVE"] / 8 / (r["dur"] * 1e-9) / 1e9 for r in ds if "GRBM_GUI_ACTIVE" in r and r["dur"]]
    return {"dispatches": len(ds), "effective_clock_ghz": statistics.median(clocks) if clocks else None,
            "effective_clock_ghz_min": min(clocks) if clocks else None,
            "avg_dispatch_us": statistics.mean(r["dur"] for r in ds) * 1e-3 if ds else None,
            "source": os.path.relpath(d, ROOT)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plies", type=int, default=100)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--summarize")
    a = ap.parse_args()
    if a.summarize:
        print(json.dumps(summarize(a.summarize)))
    else:
        run(a.plies, a.seconds, a.envs)


if __name__ == "__main__":
    main()
