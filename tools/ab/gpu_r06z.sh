# round 6, batch z: k_play_rand's first scan (the fills' prime) before the LDS tables'
# stores and barrier, while the table loads land (head, OTH_PRIME_EARLY 1), against
# after the barrier (pr0).  Config 3 at 10- and 100-ply launches, config 2, 6x6.
#   python tools/ab_variants.py --build pr0=-DOTH_PRIME_EARLY=0 --sizes 6,8
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06z
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head pr0 --policy greedy --plies 10 --init-rand 10 --rounds 20 > $O/greedy10.json 2> $O/greedy10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run pr0 head --policy greedy --plies 10 --init-rand 10 --rounds 20 > $O/greedy10b.json 2> $O/greedy10b.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head pr0 --policy greedy --plies 100 --init-rand 10 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head pr0 --plies 100 --rounds 20 > $O/rand8.json 2> $O/rand8.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head pr0 --board-size 6 --plies 100 > $O/rand6.json 2> $O/rand6.err || exit 1
echo batch-z-done
