# A/B: k_play_rand's next Philox block inside the first ply's region (OTH_RAND_FILL) and the
# max-ilp machine scheduler (-mllvm -amdgpu-sched-strategy=max-ilp), alone and together
set -o pipefail
O=${1:-gpurun_out/r02fi}; mkdir -p $O
for spec in "random 0 8 100 65536" "random 0 6 100 65536" "greedy 10 8 10 65536" "random 0 10 100 65536" "random 0 8 100 131072"; do
set -- $spec
timeout -k 10 300 python tools/ab_variants.py --run f0 f1 i0 i1 --plies $4 --launches 10 --rounds 8 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec"; cat $O/ab_$1_$3_$5.json
done
for n in 8 10; do
timeout -k 10 300 python tools/ab_sample_step.py f0 i0 --board-size $n > $O/ss_n$n.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ss_n$n.json
done
