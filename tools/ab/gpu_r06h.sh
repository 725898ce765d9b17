# round 6, batch h: the 64-bit shifts' amount as an SGPR set by s_mov_b32 (head,
# OTH_SH_MODE 1) or a VGPR (sh2) instead of inline-asm shifts by a literal (sh0,
# round 5's code), which the backend follows with an s_nop whenever the next
# instruction reads the result; configs 2, 3 and 5 at 65,536 boards.  Built here:
#   python tools/ab_variants.py --build sh0=-DOTH_SH_MODE=0 sh2=-DOTH_SH_MODE=2 --sizes 6,8,10
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06h
mkdir -p $O
cd $R
V="head sh0 sh2"
timeout -k 10 300 python -u tools/ab_variants.py --run $V --plies 100 > $O/rand8.json 2> $O/rand8.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run $V --policy greedy --plies 100 --init-rand 10 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run $V --policy greedy --plies 10 --init-rand 10 > $O/greedy10.json 2> $O/greedy10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run $V --board-size 6 --plies 100 > $O/rand6.json 2> $O/rand6.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run $V --board-size 10 --plies 100 > $O/rand10.json 2> $O/rand10.err || exit 1
echo batch-h-done
