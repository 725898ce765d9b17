# round 6, batch c: bfloat16 observations (OTH_BF16) and the learners' ply with
# make_state in int8 / bf16 (bench step_observe_lines) at 65,536 8x8 boards
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06c
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_step_observe.py tests/test_gpu_parity.py -k "observ or step_observe" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda', 0)
for r in range(2):
    print(json.dumps(bench.step_observe_lines(65536, 8, dev, torch.cuda.current_stream(dev))), flush=True)
" > $O/step_observe.jsonl 2> $O/step_observe.err || exit 1
echo batch-c-done
