#!/usr/bin/env python3
"""Summarise tools/pmc_profile.sh output into profiles/pmc_traffic.json.

    python tools/pmc_summarize.py gpurun_out/pmc1 random-play-8x8-E65536-P100
    python tools/pmc_summarize.py DIR WORKLOAD --kernel "k_play_rand<8, 1>" --out pmc_configs.json

Per dispatch of the bench kernel (k_play): FETCH_SIZE / WRITE_SIZE (KiB, from
separate passes) -> HBM bytes, with the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of wide coalesced
streaming reads, so the read side is doubled; WRITE_SIZE is exact for
streaming stores.  Also VALU / SALU instructions and wave cycles per dispatch.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, kernel="k_play"):
    vals = collections.defaultdict(list)
    durs = []
    for f in glob.glob(os.path.join(path, "pmc*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, (sum(durs) / len(durs) if durs else None)


def trace_avg(path, kernel="k_play"):
    f = os.path.join(path, "trace", "run_kernel_stats.csv")
    if not os.path.exists(f):
        return None
    for r in csv.DictReader(open(f)):
        if kernel in r["Name"]:
            return {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                    "max_ns": float(r["MaxNs"]), "name": r["Name"]}
    return None


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("workload")
    ap.add_argument("--kernel", default="k_play", help="substring of the kernel name (first match)")
    ap.add_argument("--out", default="pmc_traffic.json", help="file under profiles/")
    a = ap.parse_args()
    path, workload = a.path, a.workload
    c, dur = per_dispatch(path, a.kernel)
    fetch = c.get("FETCH_SIZE", 0.0) * 1024
    write = c.get("WRITE_SIZE", 0.0) * 1024
    rec = {
        "hbm_bytes_per_launch": 2 * fetch + write,
        "fetch_size_bytes_raw": fetch,
        "fetch_bytes_corrected_x2": 2 * fetch,
        "write_bytes": write,
        "valu_insts_per_launch": c.get("SQ_INSTS_VALU"),
        "salu_insts_per_launch": c.get("SQ_INSTS_SALU"),
        "lds_insts_per_launch": c.get("SQ_INSTS_LDS"),
        "waves_per_launch": c.get("SQ_WAVES"),
        "wave_cycles_quad": c.get("SQ_WAVE_CYCLES"),
        "wait_any_quad": c.get("SQ_WAIT_ANY"),
        "active_inst_any_quad": c.get("SQ_ACTIVE_INST_ANY"),
        "grbm_gui_active": c.get("GRBM_GUI_ACTIVE"),
        "profiled_dispatch_avg_ns": dur,
        "kernel_trace": trace_avg(path, a.kernel),
        "source": os.path.relpath(path, ROOT),
    }
    out = os.path.join(ROOT, "profiles", a.out)
    d = json.load(open(out)) if os.path.exists(out) else {}
    d[workload] = rec
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
