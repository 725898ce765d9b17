set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
run() { local out=$1; shift; timeout -k 10 240 python tools/ab_sample_step.py "$@" > $O/$out.json 2> $O/$out.err || { tail -20 $O/$out.err; exit 1; }; echo "$out"; cat $O/$out.json; }
for E in 3001 8192 16384 65536; do
run quad_n8_E$E q0 q1 --lp --envs $E
run quad_n6_E$E q0 q1 --lp --envs $E --board-size 6
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_masked.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/bench_graph.py --fused > $O/bg.json && timeout -k 10 200 python tools/bench_graph.py --fused --device-draws >> $O/bg.json && cat $O/bg.json
