# round 6, batch ac: the opening hash with its (seed, purpose) key loop-invariant
# (head) against Philox (phx; outputs differ, --no-check), config 3; then the whole
# GPU suite, smoke() and the default bench on the head build.
#   python tools/ab_variants.py --build phx=-DOTH_OPENING_PHILOX=1 --sizes 8
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ac
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head phx --policy greedy --plies 100 --init-rand 10 --no-check --rounds 15 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run phx head --policy greedy --plies 100 --init-rand 10 --no-check --rounds 15 > $O/greedy100b.json 2> $O/greedy100b.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head phx --policy greedy --plies 10 --init-rand 10 --no-check --rounds 15 > $O/greedy10.json 2> $O/greedy10.err || exit 1
bash tools/gpu_val.sh $O/val || exit 1
echo batch-ac-done
