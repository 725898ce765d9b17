# round 5, batch m: large launches -- oth_observe with about 4 KiB of output per
# wave (head) against 64 KiB (the shipped shape before), 2 and 8 KiB; the fused
# step and sample-step with their observations as two launches from 262,144
# boards (head) against one (sofused); the observation tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_observe.py tests/test_gpu_parity.py -k "observ" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_observe.py head reg64k reg2k reg8k --envs 1048576 --launches 20 --rounds 4 > $O/ab_obs_region.jsonl 2> $O/ab_obs_region.err || exit 1
timeout -k 10 300 python -u tools/ab_step_obs.py --variants sofused --envs 1048576 --plies 8 --rounds 4 > $O/ab_step_obs_1m.json 2> $O/ab_step_obs_1m.err || exit 1
timeout -k 10 300 python -u tools/ab_ss_obs.py head sofused --envs 1048576 --plies 8 --rounds 4 > $O/ab_ss_obs_1m.json 2> $O/ab_ss_obs_1m.err || exit 1
echo batch-m-done
