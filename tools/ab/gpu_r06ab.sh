# round 6, batch ab: the opening-length draw by murmur3's finaliser (head) against
# Philox4x32-10 (phx, round 5's spec; outputs differ, --no-check); config 3 at
# 65,536 boards, 100- and 10-ply launches, and 10x10 random with openings.  Then the
# GPU suites that pin openings against the oracle.
#   python tools/ab_variants.py --build phx=-DOTH_OPENING_PHILOX=1 --sizes 8,10
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ab
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head phx --policy greedy --plies 100 --init-rand 10 --no-check --rounds 15 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run phx head --policy greedy --plies 100 --init-rand 10 --no-check --rounds 15 > $O/greedy100b.json 2> $O/greedy100b.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head phx --policy greedy --plies 10 --init-rand 10 --no-check --rounds 15 > $O/greedy10.json 2> $O/greedy10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head phx --plies 100 --rounds 15 > $O/rand8.json 2> $O/rand8.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_play_groups.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo batch-ab-done
