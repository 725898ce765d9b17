# round 6, batch d: the whole GPU suite on the build with bf16 observations, the
# multi-word carry axis and dword flips; the learners' ply with int8 / bf16
# make_state; 10x10 random play A/B: head (carry axis + dword flips) against
# c0 (Kogge-Stone horizontal axis), f0 (flips_fills) and c0f0 (both, round 5's code)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda', 0)
for r in range(2):
    print(json.dumps(bench.step_observe_lines(65536, 8, dev, torch.cuda.current_stream(dev))), flush=True)
" > $O/step_observe.jsonl 2> $O/step_observe.err || exit 1
timeout -k 10 400 python -u tools/ab_variants.py --run head c0 f0 c0f0 --board-size 10 --plies 100 > $O/rand10.json 2> $O/rand10.err || exit 1
echo batch-d-done
