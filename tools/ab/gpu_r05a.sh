# round 5, batch a: the fused step + observation (oth_step_observe,
# oth_sample_step_observe), the single-board record path (oth_step_sync), the
# config-4 shard and count_disks pins, MaxiMin on a wave per board -- their GPU tests, smoke, the lane-layout
# A/B of k_ply_step_obs, greedy play on lane pairs (k_play_greedy2, variant gp1)
# against k_play_rand<8, GREEDY>, the bench and a kernel trace of the headline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05a
mkdir -p $O
timeout -k 10 560 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step_observe.py tests/test_gpu_dropin.py "tests/test_gpu_parity.py::test_config4_shard_replays_on_oracle" "tests/test_gpu_parity.py::test_count_disks_batched_matches_oracle" "tests/test_gpu_parity.py::test_maximin_wave_matches_oracle" "tests/test_gpu_parity.py::test_maximin_leaf_budget_refuses_before_launch" "tests/test_gpu_parity.py::test_maximin_actions_match_reference" > $O/pytest_new.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_step_obs.py --variants so1x64 so2x32 > $O/ab_step_obs.json 2> $O/ab_step_obs.err && \
timeout -k 10 200 python -u tools/ab_variants.py --run head gp1 --policy greedy --init-rand 10 --plies 100 --launches 10 > $O/ab_greedy_pair100.json 2> $O/ab_greedy_pair.err && \
timeout -k 10 200 python -u tools/ab_variants.py --run head gp1 --policy greedy --init-rand 10 --plies 10 --launches 50 > $O/ab_greedy_pair10.json 2>> $O/ab_greedy_pair.err && \
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-side --no-cpu-baseline --steps 20 --warmup 5 > $O/prof.log 2>&1
