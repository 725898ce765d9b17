# tests + bench + kernel trace + fused-path benches (one GPU call)
set -o pipefail
O=${1:-gpurun_out/r02e}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench_default.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side > $O/bench_driver.json 2>> $O/bench.err || exit 1
for f in "" "--fused" "--device-draws" "--fused --device-draws"; do
  timeout -k 10 200 python tools/bench_graph.py $f >> $O/bench_graph.jsonl 2>> $O/bench.err || exit 1
done
cat $O/bench_graph.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-side > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
grep -h "k_play" $O/trace/run_kernel_stats.csv | cut -c1-200
