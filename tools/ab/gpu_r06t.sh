# round 6, batch t: LDS round trips on the ply's chain -- the eight ray loads of the
# one-word flips issued together before the runs (OTH_RAYS_FIRST) and greedy play's
# opening-pick table load before the greedy move, its use after (OTH_PICK_EARLY);
# head = both, pe0 / rf0 = one off, old = both off.  Configs 2, 3 and 5 (6x6) at
# 65,536 boards.  Built here:
#   python tools/ab_variants.py --build pe0=-DOTH_PICK_EARLY=0 rf0=-DOTH_RAYS_FIRST=0 old="-DOTH_PICK_EARLY=0 -DOTH_RAYS_FIRST=0" --sizes 6,8
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06t
mkdir -p $O
cd $R
V="head pe0 rf0 old"
timeout -k 10 300 python -u tools/ab_variants.py --run $V --policy greedy --plies 100 --init-rand 10 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run $V --policy greedy --plies 10 --init-rand 10 > $O/greedy10.json 2> $O/greedy10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run $V --plies 100 > $O/rand8.json 2> $O/rand8.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run $V --board-size 6 --plies 100 > $O/rand6.json 2> $O/rand6.err || exit 1
echo batch-t-done
