# k_play_rand scheduler variants: i0 max-ilp (default), i2 + schedule-metric-bias=0, i3 + set-wave-priority
set -o pipefail
O=${1:-gpurun_out/r03k}; mkdir -p $O
export TMPDIR=/tmp
for spec0 in "random 0 8 100 65536" "random 0 8 100 131072" "greedy 10 8 10 65536"; do
set -- $spec0
timeout -k 10 300 python tools/ab_variants.py --run i0 i2 i3 --plies $4 --launches 10 --rounds 10 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec0"; cat $O/ab_$1_$3_$5.json
done
# multi-word random play: x0 = HEAD (k_play_rand_w in kernels_n.hip, Philox at each group's start),
# x1 = k_play_rand_w in the max-ILP unit with the next Philox block inside the group's first ply
for n in 10 12; do
timeout -k 10 300 python tools/ab_variants.py --run x0 x1 --plies 100 --launches 10 --rounds 8 --policy random --board-size $n --envs 65536 > $O/ab_random_${n}_65536.json 2> $O/abx.err || { tail -20 $O/abx.err; exit 1; }
cat $O/ab_random_${n}_65536.json
done
