set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 300 python tools/ab_variants.py --run old new --plies 100 --launches 20 --rounds 8 > $O/ab_fast.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_fast.json
timeout -k 10 300 python tools/ab_variants.py --run old new --plies 100 --launches 20 --rounds 5 --board-size 6 > $O/ab_fast6.json 2>> $O/ab.err || exit 1
cat $O/ab_fast6.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.json 2>/dev/null && cut -c1-400 $O/bench_driver.json
