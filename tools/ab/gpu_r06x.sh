# round 6, batch x: greedy play's opening-pick table load before the greedy move with
# the ray loads first already in (head): a scheduling barrier after the load (pe1),
# after the move (pe2), both (pe3).  Config 3 at 65,536 boards, 100- and 10-ply
# launches, twice.  Built here:
#   python tools/ab_variants.py --build pe1=-DOTH_PICK_EARLY=1 pe2=-DOTH_PICK_EARLY=2 pe3=-DOTH_PICK_EARLY=3 --sizes 8
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06x
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head pe1 pe2 pe3 --policy greedy --plies 100 --init-rand 10 --rounds 15 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run pe3 pe2 pe1 head --policy greedy --plies 100 --init-rand 10 --rounds 15 > $O/greedy100b.json 2> $O/greedy100b.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head pe1 pe2 pe3 --policy greedy --plies 10 --init-rand 10 --rounds 15 > $O/greedy10.json 2> $O/greedy10.err || exit 1
echo batch-x-done
