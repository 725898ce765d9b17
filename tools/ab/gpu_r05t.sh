# round 5, batch t: oth_step_observe in one launch for boards of two or more
# words (k_step_obs) against the two launches (somulti0), 10x10 at 65,536 boards;
# the step-observe tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05t
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_observe.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_step_obs.py --variants somulti0 --board-size 10 > $O/ab_step_obs_10.json 2> $O/ab_step_obs_10.err || exit 1
echo batch-t-done
