set -o pipefail
O=gpurun_out/r02s; mkdir -p $O
for n in 8 6; do
timeout -k 10 300 python tools/ab_variants.py --run gr0 gr1 --plies 10 --launches 20 --rounds 6 --policy greedy --init-rand 10 --board-size $n > $O/ab_greedy_n$n.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_greedy_n$n.json
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "greedy or config or fills or terminated or vs" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
