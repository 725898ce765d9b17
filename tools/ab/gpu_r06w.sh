# round 6, batch w: the multi-word flips' eight ray loads issued together before the
# runs (head, OTH_W_RAYS_FIRST 1) against interleaved with them (wrf0); config 5 at
# 10x10, 65,536 boards, twice.  Built here:
#   python tools/ab_variants.py --build wrf0=-DOTH_W_RAYS_FIRST=0 --sizes 10
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06w
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head wrf0 --board-size 10 --plies 100 --rounds 20 > $O/rand10.json 2> $O/rand10.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run wrf0 head --board-size 10 --plies 100 --rounds 20 > $O/rand10b.json 2> $O/rand10b.err || exit 1
echo batch-w-done
