set -o pipefail
O=${1:-gpurun_out/r02j}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM --output-format csv -d $O/pmc1 -o run -- python3 tools/bench_graph.py --fused --reps 2 --plies 8 > $O/pmc1.log 2>&1 || { tail $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS --output-format csv -d $O/pmc2 -o run -- python3 tools/bench_graph.py --fused --reps 2 --plies 8 > $O/pmc2.log 2>&1 || { tail $O/pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM --output-format csv -d $O/pmc3 -o run -- python3 tools/bench_graph.py --reps 2 --plies 8 > $O/pmc3.log 2>&1 || { tail $O/pmc3.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob
for d in ("pmc1", "pmc2", "pmc3"):
    v = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/r02j/%s/run_counter_collection.csv" % d):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if any(k in n for k in ("k_sample_step", "k_masked", "k_step")):
                v[(n[:32], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, x in sorted(v.items()):
        print(d, k, round(sum(x) / len(x)), len(x))
PY
