# Round-3 validation of the built tree: GPU suite, smoke, default bench, the bench kernel's
# PMC passes, the single-ply / fused-ply kernel traces and counters (65,536 and 1,048,576 boards).
set -o pipefail
O=${1:-gpurun_out/r03fin}; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_val.sh $O || exit 1
bash tools/pmc_profile.sh $O/pmc || { echo PMC_FAIL; exit 1; }
bash tools/gpu_prof_step.sh $O/step || { echo STEP_FAIL; exit 1; }
