set -o pipefail
O=gpurun_out/r02w; mkdir -p $O
run() { local out=$1; shift; timeout -k 10 240 python tools/ab_sample_step.py "$@" > $O/$out.json 2> $O/$out.err || { tail -20 $O/$out.err; exit 1; }; echo "$out"; cat $O/$out.json; }
run stage_n8 p0 s0 s1
run stage_n8_lp p0 s0 s1 --lp
run stage_n8_odd p0 s0 s1 --lp --envs 3001
timeout -k 10 600 python -u -m pytest tests/test_gpu_masked.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/ab_sample_step.py p0 s1 --rounds 2 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r02w/tr/run_kernel_stats.csv")):
    if "oth" in r["Name"]: print(r["Name"][:70], r["Calls"], r["AverageNs"], r["MinNs"])
PY
