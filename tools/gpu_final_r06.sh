# Round-6 validation of the built tree: the whole GPU suite, smoke(), the default
# bench, the headline kernel's trace and counter passes, the single-ply and fused
# step / observation paths' traces and counters (65,536 and 1,048,576 boards), and
# the sustained clock; configs 3 and 5's traces and counters.
set -o pipefail
O=${1:-gpurun_out/r06fin}; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_val.sh $O || exit 1
bash tools/pmc_profile.sh $O/pmc || { echo PMC_FAIL; exit 1; }
bash tools/gpu_prof_step.sh $O/step --plies 32 --cases step_ext,step_obs,step_obs_ms,sample_step,ss_obs || { echo STEP_FAIL; exit 1; }
bash tools/gpu_prof_configs.sh $O/cfg greedy10 greedy100 rand6,rand10 > $O/cfg.log 2>&1 || { echo CFG_FAIL; exit 1; }
python3 tools/kstats.py $O/step --json $O/step/kstats.json > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/clk -o run -- python3 tools/sustained_clock.py --plies 1000 --seconds 3 > $O/clk.log 2>&1 || exit 1
python3 tools/sustained_clock.py --summarize $O/clk > $O/clk.json || exit 1
echo final-done
