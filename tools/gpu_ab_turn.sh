set -o pipefail
O=gpurun_out/r02p; mkdir -p $O
for n in 8 6; do
timeout -k 10 300 python tools/ab_variants.py --run t0 t2 --plies 100 --launches 20 --rounds 8 --board-size $n > $O/ab_n$n.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_n$n.json
done
timeout -k 10 300 python tools/ab_variants.py --run t0 t2 --plies 10 --launches 20 --rounds 6 --policy greedy --init-rand 10 > $O/ab_greedy.json 2>> $O/ab.err || exit 1
cat $O/ab_greedy.json
