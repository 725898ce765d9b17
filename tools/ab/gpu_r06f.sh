# round 6, batch f: greedy play's opening pick and greedy move both computed then
# selected (gbf) against the exec-masked branches (head), config 3 at 65,536 boards;
# then kernel traces + counters of configs 3 and 5 on the current build
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06f
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_variants.py --run head gbf --policy greedy --plies 100 --init-rand 10 > $O/greedy100.json 2> $O/greedy100.err || exit 1
timeout -k 10 300 python -u tools/ab_variants.py --run head gbf --policy greedy --plies 10 --init-rand 10 > $O/greedy10.json 2> $O/greedy10.err || exit 1
bash tools/gpu_prof_configs.sh $O/cfg greedy10 greedy100 rand6,rand10 > $O/prof.log 2>&1 || exit 1
echo batch-f-done
