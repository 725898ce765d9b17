# round 6, batch aa (probe): what the opening-length Philox draw in greedy play's
# terminal block costs -- head against a wrong, cheap draw (cheap; outputs differ,
# --no-check).  Config 3 at 65,536 boards.
#   python tools/ab_variants.py --build cheap=-DOTH_PROBE_CHEAP_OPENING=1 --sizes 8
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06aa
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head cheap --policy greedy --plies 100 --init-rand 10 --no-check --rounds 15 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run cheap head --policy greedy --plies 100 --init-rand 10 --no-check --rounds 15 > $O/greedy100b.json 2> $O/greedy100b.err || exit 1
echo batch-aa-done
