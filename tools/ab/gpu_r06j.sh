# round 6, batch j: greedy play with random openings in 4-ply groups (head,
# OTH_GREEDY_GROUPS 1: the group's Philox block at its start, words taken
# statically) against the per-ply block test and word choice (gg0), config 3 at
# 65,536 boards; the random-play headline as a control.  Built here:
#   python tools/ab_variants.py --build gg0=-DOTH_GREEDY_GROUPS=0 --sizes 8
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${BATCH:-r06j}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head gg0 --policy greedy --plies 100 --init-rand 10 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head gg0 --policy greedy --plies 10 --init-rand 10 > $O/greedy10.json 2> $O/greedy10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head gg0 --plies 100 > $O/rand8.json 2> $O/rand8.err || exit 1
echo batch-j-done
