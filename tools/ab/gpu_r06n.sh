# round 6, batch n: multi-word random play without openings compiled apart (head,
# OTH_W_OPEN_SPLIT 1: no opening bookkeeping, no scalar branch on init_rand in the
# terminal block) against one loop for both (wo0); the terminal reward by a mask
# in both.  Config 5 at 10x10, 65,536 boards.  Built here:
#   python tools/ab_variants.py --build wo0=-DOTH_W_OPEN_SPLIT=0 --sizes 10
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06n
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head wo0 --board-size 10 --plies 100 > $O/rand10.json 2> $O/rand10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head wo0 --board-size 10 --plies 100 --init-rand 10 > $O/rand10_open.json 2> $O/rand10_open.err || exit 1
echo batch-n-done
