# round 6, batch u: batch t's arms again with twice the rounds (random 8x8: head /
# pe0 = rays first, old; greedy 100-ply: all four)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06u
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run pe0 old head --plies 100 --rounds 20 > $O/rand8.json 2> $O/rand8.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run old pe0 rf0 head --policy greedy --plies 100 --init-rand 10 --rounds 20 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run old pe0 --board-size 6 --plies 100 --rounds 20 > $O/rand6.json 2> $O/rand6.err || exit 1
echo batch-u-done
