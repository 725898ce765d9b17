# A/B: U2 shifts as one v_lshl*_b64 (u1, the A/B build macro OTH_U2_SH64=1; now the only form) against v_lshlrev_b32 + v_alignbit_b32 (u0),
# on every engine that runs OneWord's scan: k_play_rand (random, greedy), the single-ply kernels,
# the fused sample + step
set -o pipefail
O=${1:-gpurun_out/r03sh64}; shift; V="${*:-u0 u1}"; mkdir -p $O
for spec0 in "random 0 8 100 65536" "random 0 6 100 65536" "greedy 10 8 10 65536" "random 0 8 100 131072" "random 0 7 100 65536"; do
set -- $spec0
timeout -k 10 300 python tools/ab_variants.py --run $V --plies $4 --launches 10 --rounds 8 --policy $1 --init-rand $2 --board-size $3 --envs $5 > $O/ab_$1_$3_$5.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
echo "$spec0"; cat $O/ab_$1_$3_$5.json
done
timeout -k 10 300 python tools/ab_ply.py $V --envs 65536,1048576 --rounds 6 > $O/ab_ply.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab_ply.jsonl
timeout -k 10 300 python tools/ab_sample_step.py $V --board-size 8 > $O/ss_n8.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ss_n8.json
