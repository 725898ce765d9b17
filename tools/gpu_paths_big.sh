# every batched entry point at 1,048,576 8x8 boards (kernel trace), beside torch's own write / copy rates
set -o pipefail
O=${1:-gpurun_out/r02big}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_paths.py --envs 1048576 --iters 50 > $O/paths.jsonl 2> $O/paths.err || { tail $O/paths.err; exit 1; }
cat $O/paths.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_paths.py --envs 1048576 --iters 20 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
timeout -k 10 120 python - > $O/torch_bw.json <<'PY'
import json, torch
dev = torch.device("cuda", 0)
x = torch.empty(1048576 * 256, dtype=torch.float32, device=dev)  # 1 GiB, make_state f32 of 1,048,576 boards
y = torch.empty_like(x)
for _ in range(3):
    x.fill_(1.0); y.copy_(x)
torch.cuda.synchronize()
res = {}
for name, fn, nbytes in (("fill", lambda: x.fill_(2.0), x.numel() * 4), ("copy", lambda: y.copy_(x), 2 * x.numel() * 4)):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 100.0
    res[name] = {"us": us, "GBs": nbytes / us / 1e3}
print(json.dumps(res))
PY
cat $O/torch_bw.json
