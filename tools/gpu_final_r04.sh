# Round-4 validation of the built tree: the whole GPU suite, smoke(), the default
# bench, the headline kernel's counter passes, configs 3 / 5 and the observation
# encoders' traces and counters, and the single-ply / fused-ply kernels' traces and
# counters (65,536 and 1,048,576 boards).
set -o pipefail
O=${1:-gpurun_out/r04fin}; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_val.sh $O || exit 1
bash tools/pmc_profile.sh $O/pmc || { echo PMC_FAIL; exit 1; }
bash tools/gpu_prof_configs.sh $O/cfg || { echo CFG_FAIL; exit 1; }
bash tools/gpu_prof_step.sh $O/step || { echo STEP_FAIL; exit 1; }
