# round 5, batch n: the learners' fused ply with its make_state, two chunks of
# 32 boards per wave (ssc2: the first chunk's stores in flight while the second
# is sampled and stepped) against one; the sample-step tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05n
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_observe.py tests/test_gpu_masked.py tests/test_gpu_hazards.py -k "sample" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssc2 --envs 65536 > $O/ab_ss_obs_65k.json 2> $O/ab_ss_obs_65k.err || exit 1
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssc2 --envs 131072 > $O/ab_ss_obs_131k.json 2> $O/ab_ss_obs_131k.err || exit 1
timeout -k 10 300 python -u tools/ab_ss_obs.py head ssc2 --envs 1048576 --plies 8 --rounds 4 > $O/ab_ss_obs_1m.json 2> $O/ab_ss_obs_1m.err || exit 1
echo batch-n-done
