set -o pipefail
O=${1:-gpurun_out/r02f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_masked.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for f in "" "--fused" "--fused --device-draws" "--fused --board-size 6" "--fused --board-size 10"; do
  timeout -k 10 200 python tools/bench_graph.py $f >> $O/bench_graph.jsonl 2>> $O/bench.err || exit 1
done
cat $O/bench_graph.jsonl
