#!/usr/bin/env python3
"""Per (kernel, grid) summary of a tools/gpu_prof_step.sh (or pmc_profile.sh)
output directory: average kernel-trace duration, and the counters of every
pmc* pass averaged per dispatch, with derived per-board figures.

    python tools/kstats.py <dir> [--match k_step,k_play_rand,k_sample_step] [--json out.json]

HBM bytes: FETCH_SIZE x 2 (gfx950 counts half the bytes of wide coalesced reads,
MI355X_MICROARCH.md section HBM) + WRITE_SIZE, both in KiB per dispatch.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name):
    m = re.match(r"(?:void )?(?:[\w:]+::)?(\w+<[^()]*>|\w+)", name)
    return m.group(1) if m else name[:60]


def summarize(d, match):
    pats = match.split(",") if match else None
    keep = (lambda n: any(p in n for p in pats)) if pats else (lambda n: True)
    out = collections.OrderedDict()
    tr = os.path.join(d, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        for r in csv.DictReader(open(tr)):
            if not keep(r["Kernel_Name"]):
                continue
            k = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]))
            rec = out.setdefault(k, {"kernel": k[0], "grid": k[1], "durs": [], "ctr": collections.defaultdict(list),
                                     "vgpr": int(r["VGPR_Count"]), "lds": int(r["LDS_Block_Size"])})
            rec["durs"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if not keep(r["Kernel_Name"]):
                continue
            k = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            rec = out.setdefault(k, {"kernel": k[0], "grid": k[1], "durs": [], "ctr": collections.defaultdict(list),
                                     "vgpr": int(r["VGPR_Count"]), "lds": int(r["LDS_Block_Size"])})
            rec["ctr"][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = []
    for rec in out.values():
        c = {k: sum(v) / len(v) for k, v in rec["ctr"].items()}
        durs = sorted(rec["durs"])
        row = {"kernel": rec["kernel"], "grid": rec["grid"], "vgpr": rec["vgpr"], "lds": rec["lds"],
               "calls": len(durs), "avg_ns": sum(durs) / len(durs) if durs else None,
               "median_ns": durs[len(durs) // 2] if durs else None}
        row.update({k: round(v, 1) for k, v in c.items()})
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            row["hbm_bytes"] = 2 * 1024 * c.get("FETCH_SIZE", 0.0) + 1024 * c.get("WRITE_SIZE", 0.0)
        if "SQ_WAVES" in c and "SQ_INSTS_VALU" in c and c["SQ_WAVES"]:
            row["valu_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        if "SQ_WAVE_CYCLES" in c and c.get("SQ_WAVE_CYCLES"):
            row["wait_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
            row["active_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_BUSY_CYCLES"):
            row["avg_waves_resident_per_se"] = c.get("SQ_WAVE_CYCLES", 0) / c["SQ_BUSY_CYCLES"]
        res.append(row)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="oth_dev")
    ap.add_argument("--json")
    a = ap.parse_args()
    res = summarize(a.dir, a.match)
    for r in res:
        print(json.dumps(r))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
