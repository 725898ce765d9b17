set -o pipefail
O=gpurun_out/r02u; mkdir -p $O
run() { local out=$1; shift; timeout -k 10 240 python tools/ab_sample_step.py "$@" > $O/$out.json 2> $O/$out.err || { tail -20 $O/$out.err; exit 1; }; echo "$out"; cat $O/$out.json; }
run pair_n8 p0 p1
run pair_n8_lp p0 p1 --lp
run pair_n6 p0 p1 --board-size 6
run pair_n6_lp p0 p1 --board-size 6 --lp
run pair_n7_lp p0 p1 --board-size 7 --lp --envs 3001
timeout -k 10 600 python -u -m pytest tests/test_gpu_masked.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
