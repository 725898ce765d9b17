set -o pipefail
O=gpurun_out/r02zd; mkdir -p $O
for spec in "random 0 10 100" "random 0 9 100" "random 0 11 100" "greedy 10 10 10" "random 0 12 50"; do
set -- $spec
timeout -k 10 300 python tools/ab_variants.py --run q40 q41 --plies $4 --launches 10 --rounds 6 --policy $1 --init-rand $2 --board-size $3 > $O/ab_$1_$2_$3.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec"; cat $O/ab_$1_$2_$3.json
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
