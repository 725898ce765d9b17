set -o pipefail
O=${1:-gpurun_out/r02g}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tf -o run -- python3 tools/bench_graph.py --fused --reps 5 > $O/tf.log 2>&1 || { tail $O/tf.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ts -o run -- python3 tools/bench_graph.py --reps 5 > $O/ts.log 2>&1 || { tail $O/ts.log; exit 1; }
cut -d, -f1-8 $O/tf/run_kernel_stats.csv | cut -c1-250
cut -d, -f1-8 $O/ts/run_kernel_stats.csv | cut -c1-250
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM --output-format csv -d $O/pmc -o run -- python3 tools/bench_graph.py --fused --reps 2 --plies 8 > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/r02g/pmc/run_counter_collection.csv")):
    if "k_sample_step" in r["Kernel_Name"] or "k_masked" in r["Kernel_Name"] or "k_step" in r["Kernel_Name"]:
        v[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, x in sorted(v.items()):
    print(k, sum(x) / len(x), len(x))
PY
