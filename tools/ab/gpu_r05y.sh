# round 5, batch y: the play kernels (k_play_rand random / greedy) under the
# default (sdef) and max-occupancy (socc) machine schedulers against max-ILP (head)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05y
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head sdef socc --policy greedy --plies 100 --init-rand 10 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head sdef socc --policy greedy --plies 10 --init-rand 10 > $O/greedy10.json 2> $O/greedy10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head sdef socc --policy random --plies 100 > $O/random100.json 2> $O/random100.err || exit 1
echo batch-y-done
