# round 5, batch h: more lane layouts of the fused step (lane pairs or single
# lanes with 16 or 32 boards a wave), and MaxiMin's balanced pair walks (depth
# >= 4) against the static pair rounds (variant mmstatic), with the MaxiMin
# parity tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05h
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_parity.py::test_maximin_wave_matches_oracle" "tests/test_gpu_parity.py::test_maximin_actions_match_reference" "tests/test_gpu_dropin.py::test_maximin_policy_dropin" "tests/test_gpu_parity.py::test_maximin_leaf_budget_refuses_before_launch" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_step_obs.py --variants so2x16 so1x32 so1x16 > $O/ab_step_obs.json 2> $O/ab_step_obs.err || exit 1
timeout -k 10 400 python -u tools/ab_maximin.py mmstatic --depths 3 4 5 6 > $O/ab_maximin_bal.jsonl 2> $O/ab_maximin_bal.err || exit 1
echo batch-h-done
