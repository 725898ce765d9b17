# Round 4, batch a: parity of the changed kernels, A/B of lane-pair single-ply
# kernels / pair-split scan / 16-boards-per-wave observations against the
# round-3 shapes (variants old / new), the bench with its new side lines, and
# counter passes of configs 3 / 5 and the observation encoders.
set -o pipefail
O=${1:-gpurun_out/r04a}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hazards.py tests/test_gpu_masked.py -m gpu -q -x --timeout 300 --timeout-method thread -k "single_ply or observation or external or step or live or sample" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/ab_ply.py old new --envs 65536,1048576 > $O/ab_ply.jsonl 2> $O/ab_ply.err || { tail $O/ab_ply.err; exit 1; }
cat $O/ab_ply.jsonl
timeout -k 10 300 python tools/ab_sample_step.py old new --envs 65536 > $O/ab_ss.jsonl 2> $O/ab_ss.err || { tail $O/ab_ss.err; exit 1; }
cat $O/ab_ss.jsonl
timeout -k 10 300 python tools/ab_observe.py old new > $O/ab_obs.jsonl 2> $O/ab_obs.err || { tail $O/ab_obs.err; exit 1; }
cat $O/ab_obs.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
bash tools/gpu_prof_configs.sh $O/cfg || exit 1
