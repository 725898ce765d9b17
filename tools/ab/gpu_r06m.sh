# round 6, batch m: a & ~b in the one-word flips and horizontal scan as v_bitop3_b32
# on VGPRs (andn, OTH_BITOP3_ANDN 1) against v_bfi_b32 with an inline 0 (head), random
# play at 65,536 boards (one wave per SIMD) and 131,072 (config 4's shard: two)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06m
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head andn --plies 100 > $O/rand8.json 2> $O/rand8.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head andn --plies 100 --envs 131072 > $O/rand8_131072.json 2> $O/rand8_131072.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head andn --policy greedy --plies 100 --init-rand 10 --envs 131072 > $O/greedy100_131072.json 2> $O/greedy100_131072.err || exit 1
echo batch-m-done
