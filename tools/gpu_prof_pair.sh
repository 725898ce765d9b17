set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/ab_sample_step.py p0 p1 --rounds 2 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r02v/tr/run_kernel_stats.csv")):
    print(r["Name"][:70], r["Calls"], r["AverageNs"], r["MinNs"])
PY
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS --output-format csv -d $O/pmc -o run -- python3 tools/ab_sample_step.py p0 p1 --rounds 1 --reps 1 --plies 8 > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/r02v/pmc/run_counter_collection.csv")):
    if "k_sample_step" in r["Kernel_Name"]:
        v[(r["Kernel_Name"][:34], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, x in sorted(v.items()):
    print(k, sum(x) / len(x), len(x))
PY
