# Round 4, batch d: observation kernels' parity and the A/B of streaming stores,
# the host cost of one launch without Python (tools/launch_cost), and the step
# floors at 1,048,576 boards.
set -o pipefail
O=${1:-gpurun_out/r04d}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "observation" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/ab_observe.py new nt --envs 65536,1048576 > $O/ab_obs_nt.jsonl 2> $O/ab_obs.err || { tail $O/ab_obs.err; exit 1; }
cat $O/ab_obs_nt.jsonl
timeout -k 10 120 tools/launch_cost gymothelloenv_amd/liboth_mi355x.so > $O/launch_cost.jsonl 2>&1 || { tail $O/launch_cost.jsonl; exit 1; }
cat $O/launch_cost.jsonl
timeout -k 10 300 python tools/probe_step.py > $O/probe_step_65536.json 2> $O/probe.err || { tail $O/probe.err; exit 1; }
cat $O/probe_step_65536.json
timeout -k 10 300 python tools/probe_step.py --envs 1048576 --plies 32 > $O/probe_step_1m.json 2>> $O/probe.err || { tail $O/probe.err; exit 1; }
cat $O/probe_step_1m.json
timeout -k 10 300 python tools/ab_ply.py new dnt0 --envs 1048576 > $O/ab_dones.jsonl 2> $O/ab_dones.err || { tail $O/ab_dones.err; exit 1; }
cat $O/ab_dones.jsonl
