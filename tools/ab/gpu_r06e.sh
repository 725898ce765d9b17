# round 6, batch e: int8 / bf16 observations 16 bytes a lane (put_narrow; n0 =
# round 5's quads) -- the observation suites, the learners' fused ply with int8 /
# bf16 make_state, k_observe_w int8 / bf16; 10x10 random play with the
# branch-free two-word pick (head) against the per-word branches (s0)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06e
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_observe.py tests/test_gpu_parity.py tests/test_gpu_masked.py -k "observ or step_observe or legal or sample" > $O/pytest.log 2>&1 || exit 1
for dt in int8 bfloat16 float32; do
  timeout -k 10 300 python -u tools/ab_ss_obs.py head n0 --dtype $dt > $O/ss_obs_$dt.json 2> $O/ss_obs_$dt.err || exit 1
done
timeout -k 10 300 python -u tools/ab_observe.py head n0 --envs 65536,1048576 --layouts make_state,board,legal --dtype int8 > $O/obs_int8.jsonl 2> $O/obs_int8.err || exit 1
timeout -k 10 300 python -u tools/ab_observe.py head n0 --envs 65536,1048576 --layouts make_state,board --dtype bfloat16 > $O/obs_bf16.jsonl 2> $O/obs_bf16.err || exit 1
timeout -k 10 400 python -u tools/ab_variants.py --run head s0 --board-size 10 --plies 100 > $O/rand10.json 2> $O/rand10.err || exit 1
timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda', 0)
print(json.dumps(bench.step_observe_lines(65536, 8, dev, torch.cuda.current_stream(dev))), flush=True)
" > $O/step_observe.jsonl 2> $O/step_observe.err || exit 1
echo batch-e-done
