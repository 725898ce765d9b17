# round 5, batch e: the fused-observation tests (step_vs with its observation,
# the large-launch shape from 262,144 boards), the fused paths' times at 65,536
# and 1,048,576 boards, smoke and the bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_observe.py "tests/test_gpu_parity.py::test_maximin_leaf_budget_refuses_before_launch" tests/test_gpu_dropin.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/prof_step.py --plies 32 --cases step_ext,step_obs,step_obs_ms,ss_obs > $O/times.jsonl 2> $O/times.err || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo batch-e-done
