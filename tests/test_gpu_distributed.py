"""The multi-GPU path on the real collective: a process group on the "nccl"
backend (RCCL on ROCm) with the product's ShardedVecOthelloEnv and the W/D/L
all-gather (distributed.gather_wdl, ppo_run_self_play.py:432-441's tally).
One GPU allows one rank per communicator (RCCL refuses two ranks on one
device), so this runs world size 1 in a child process; the N-rank sharding
itself is covered on CPU (test_distributed_cpu.py, test_bench_cpu.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path.insert(0, %(root)r)
import torch, torch.distributed as dist
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
torch.cuda.set_device(0)
from gymothelloenv_amd.distributed import ShardedVecOthelloEnv, gather_wdl
env = ShardedVecOthelloEnv(65536, board_size=8, auto_reset=True, seed=3, device="cuda:0")
env.reset()
env.step_policy("random", n_plies=130)
local = env.counts()
g = gather_wdl(local)
tot = env.global_counts()
t = torch.tensor([1.5], dtype=torch.float64, device="cuda:0")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
print(json.dumps({"backend": dist.get_backend(), "local": local.cpu().tolist(), "gathered": g.cpu().tolist(),
                  "total": tot.cpu().tolist(), "max": float(t.item())}), flush=True)
dist.destroy_process_group()
"""


def test_rccl_wdl_all_gather_single_rank():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["backend"] == "nccl"
    assert d["gathered"] == [d["local"]] and d["total"] == d["local"]
    assert sum(d["local"]) >= 65536 and d["max"] == 1.5
