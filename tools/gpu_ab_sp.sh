# A/B: k_play_rand with the next Philox block's rounds spread over the four plies of the group (OTH_RAND_SPREAD)
set -o pipefail
O=${1:-gpurun_out/r02sp}; mkdir -p $O
for spec in "random 0 8 100 65536" "random 0 6 100 65536" "random 0 8 100 131072" "random 0 8 100 16384"; do
set -- $spec
timeout -k 10 300 python tools/ab_variants.py --run sp0 sp1 --plies $4 --launches 10 --rounds 8 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec"; cat $O/ab_$1_$3_$5.json
done
