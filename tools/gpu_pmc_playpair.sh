set -o pipefail
O=gpurun_out/r02za; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --output-format csv -d $O/pmc -o run -- python3 tools/ab_variants.py --run pp0 pp1 --plies 100 --launches 2 --rounds 1 > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/r02za/pmc/run_counter_collection.csv")):
    if "k_play_rand" in r["Kernel_Name"]:
        v[(r["Kernel_Name"][:30], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, x in sorted(v.items()):
    print(k, sum(x) / len(x), len(x))
PY
