set -o pipefail
O=gpurun_out/r02r; mkdir -p $O
for n in 10 9 12 16; do
timeout -k 10 300 python tools/ab_variants.py --run fw0 fw1 --plies 100 --launches 10 --rounds 6 --board-size $n > $O/ab_n$n.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_n$n.json
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
