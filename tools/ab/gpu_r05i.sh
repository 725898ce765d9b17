# round 5, batch i: MaxiMin's pair subtrees by compile-time recursion
# (maximin_node, registers) against the explicit-stack walk (variant mmflat),
# with the MaxiMin parity tests; the fused step against torch fill_ of its
# observation (the store floor) and with 8-byte observations by pairs (pair8)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05i
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_parity.py::test_maximin_wave_matches_oracle" "tests/test_gpu_parity.py::test_maximin_actions_match_reference" "tests/test_gpu_dropin.py::test_maximin_policy_dropin" "tests/test_gpu_parity.py::test_maximin_leaf_budget_refuses_before_launch" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_maximin.py mmflat --depths 3 4 5 6 > $O/ab_maximin_nested.jsonl 2> $O/ab_maximin_nested.err || exit 1
timeout -k 10 300 python -u tools/ab_step_obs.py --variants pair8 > $O/ab_step_obs.json 2> $O/ab_step_obs.err || exit 1
echo batch-i-done
