# Round 4, batch b: parity of the changed play / observe kernels, A/B of the
# greedy changes (axis sums, one Philox block per 4 opening plies) and of the
# handle's LDS tables against round 3's kernels, observation waves of 16 / 8 / 4
# boards, and where the step() time goes (tools/probe_step.py).
set -o pipefail
O=${1:-gpurun_out/r04b}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hazards.py -m gpu -q -x --timeout 300 --timeout-method thread -k "greedy or random or rollout or observation or single_ply or live or u2 or fills or config" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/ab_variants.py --run new r3 tab0 --policy greedy --plies 10 --init-rand 10 > $O/ab_greedy10.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab_greedy10.json
timeout -k 10 300 python tools/ab_variants.py --run new r3 tab0 --policy greedy --plies 100 --launches 5 --init-rand 10 > $O/ab_greedy100.json 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab_greedy100.json
timeout -k 10 300 python tools/ab_variants.py --run new r3 tab0 --policy random --plies 100 > $O/ab_random8.json 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab_random8.json
timeout -k 10 300 python tools/ab_observe.py new bpw8 bpw4 --envs 65536 > $O/ab_obs.jsonl 2> $O/ab_obs.err || { tail $O/ab_obs.err; exit 1; }
cat $O/ab_obs.jsonl
timeout -k 10 300 python tools/probe_step.py > $O/probe_step.json 2> $O/probe.err || { tail $O/probe.err; exit 1; }
cat $O/probe_step.json
