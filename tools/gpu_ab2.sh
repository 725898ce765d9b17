set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
for n in 8 6; do
timeout -k 10 300 python tools/ab_variants.py --run base carry both --plies 100 --launches 20 --rounds 8 --board-size $n > $O/ab_n$n.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_n$n.json
done
timeout -k 10 300 python tools/ab_variants.py --run base both --plies 10 --launches 20 --rounds 6 --policy greedy --init-rand 10 > $O/ab_greedy.json 2>> $O/ab.err || exit 1
cat $O/ab_greedy.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
