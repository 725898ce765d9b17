set -o pipefail
O=gpurun_out/r02o; mkdir -p $O
for n in 8 6; do
timeout -k 10 300 python tools/ab_variants.py --run pipe0 pipe1 --plies 100 --launches 20 --rounds 8 --board-size $n > $O/ab_n$n.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_n$n.json
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "random or config or terminated" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
