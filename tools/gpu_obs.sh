# k_observe_w: observation parity tests, then every batched path at 65,536 and 1,048,576 boards with a kernel trace
set -o pipefail
O=${1:-gpurun_out/r02obs}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread -k "observ or make_state or obs" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for E in 65536 1048576; do
timeout -k 10 300 python tools/bench_paths.py --envs $E --iters 50 > $O/paths_$E.jsonl 2> $O/paths.err || { tail $O/paths.err; exit 1; }
grep observe $O/paths_$E.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_paths.py --envs 1048576 --iters 20 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
grep observe $O/trace/run_kernel_stats.csv | cut -c1-160
