# placement probe: k_play_rand with 80 KiB of unused dynamic LDS per block (at most one block per CU) vs none
set -o pipefail
O=${1:-gpurun_out/r02pad}; mkdir -p $O
for spec in "random 0 8 100 65536" "random 0 6 100 65536" "random 0 8 100 32768"; do
set -- $spec
timeout -k 10 300 python tools/ab_variants.py --run pad0 pad1 --plies $4 --launches 10 --rounds 8 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec"; cat $O/ab_$1_$3_$5.json
done
