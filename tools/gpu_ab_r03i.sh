# k_play_rand per-ply output stores: base (last commit: selects per ply, global stores) against
# alternating word roles with m0 global stores, m1 a buffer descriptor per row, m2 one per 4-row group
set -o pipefail
O=${1:-gpurun_out/r03i}; mkdir -p $O
export TMPDIR=/tmp
for spec0 in "random 0 8 100 65536 base t0 t1 t2" "random 0 8 100 131072 base t0 t1 t2" "random 0 6 100 65536 t0 t1 t2" "greedy 10 8 10 65536 base t0 t1 t2"; do
set -- $spec0
timeout -k 10 300 python tools/ab_variants.py --run ${@:6} --plies $4 --launches 10 --rounds 10 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec0"; cat $O/ab_$1_$3_$5.json
done
