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


CHILD2 = r"""
import hashlib, json, os, sys
sys.path.insert(0, %(root)r)
import torch, torch.distributed as dist
dist.init_process_group("gloo")
from gymothelloenv_amd.distributed import ShardedVecOthelloEnv
env = ShardedVecOthelloEnv(%(G)d, board_size=8, auto_reset=True, seed=11, initial_rand_steps=4, device="cuda:0")
env.reset()
acts, _, _ = env.step_policy("random", n_plies=%(P)d)
b, m, lg = env.get_state()
torch.cuda.synchronize()
print(json.dumps({"rank": env.rank, "base": env.env_id_base, "n": env.num_envs,
                  "acts": hashlib.sha256(acts.cpu().numpy().tobytes()).hexdigest(),
                  "boards": hashlib.sha256(b.cpu().numpy().tobytes()).hexdigest(),
                  "local": env.counts().cpu().tolist(), "total": env.global_counts().cpu().tolist()}), flush=True)
dist.destroy_process_group()
"""


def test_two_ranks_on_one_gpu_equal_one_process():
    """The product's multi-rank path with two ranks (gloo: RCCL takes one rank
    per device) sharing cuda:0: each rank's ShardedVecOthelloEnv shard plays
    exactly the boards [base, base + n) of a one-process run at the same
    global E (actions, final boards), and the all-gathered W/D/L equals the
    one-process tally (ppo_run_self_play.py:432-441)."""
    import hashlib
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gymothelloenv_amd import VecOthelloEnv
    G, P = 9001, 90  # ragged: the first rank takes one board more
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", CHILD2 % {"root": ROOT, "G": G, "P": P}], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        so, se = p.communicate(timeout=100)
        assert p.returncode == 0, se[-3000:]
        outs.append(json.loads(so.strip().splitlines()[-1]))
    ref = VecOthelloEnv(G, board_size=8, auto_reset=True, seed=11, initial_rand_steps=4, device="cuda:0")
    ref.reset()
    acts, _, _ = ref.step_policy("random", n_plies=P)
    b, _, _ = ref.get_state()
    acts, b = acts.cpu().numpy(), b.cpu().numpy()
    for d in sorted(outs, key=lambda d: d["rank"]):
        lo, hi = d["base"], d["base"] + d["n"]
        assert hashlib.sha256(acts[:, lo:hi].copy().tobytes()).hexdigest() == d["acts"], d["rank"]
        assert hashlib.sha256(b[lo:hi].copy().tobytes()).hexdigest() == d["boards"], d["rank"]
        assert d["total"] == ref.counts().cpu().tolist()
    assert [o["n"] for o in sorted(outs, key=lambda d: d["rank"])] == [4501, 4500]
    assert [sum(x) for x in zip(*(o["local"] for o in outs))] == ref.counts().cpu().tolist()


def _bench(args, extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_bench_two_ranks_on_one_gpu_equal_one_rank():
    """bench.py's multi-rank path end to end (the driver's 8-GPU run, rehearsed
    with 2 ranks sharing cuda:0 over gloo): the launcher, the shards, the timed
    region, the max-over-ranks reduction and the W/D/L all-gather give a line
    whose W/D/L equals a one-rank run at the same 262,144 global boards
    (ppo_run_self_play.py:432-441's tally), with the scaling reading aids
    filled in.  No scaling number is claimed from it (one GPU, shared)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    common = ["--global-envs", "262144", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-side"]
    one = _bench(["--gpus", "1"] + common)
    two = _bench(["--gpus", "2"] + common, {"OTH_BENCH_BACKEND": "gloo", "OTH_BENCH_DEVICE": "0"})
    assert one["config"]["global_boards"] == two["config"]["global_boards"] == 262144
    assert two["ranks"] == 2 and two["shared_device"] is True and two["n_gpus"] == 1
    assert two["config"]["boards_per_gpu"] == 131072 and one["config"]["boards_per_gpu"] == 262144
    assert two["per_gpu_value"] > 0 and abs(two["per_gpu_value"] * 2 - two["value"]) < 1e-6 * two["value"]
    solo = two["single_gpu_same_shard"]
    assert solo["boards"] == 131072 and solo["value"] > 0 and solo["unit"] == "env-steps/s"
    assert two["wdl"] == one["wdl"] and sum(one["wdl"].values()) > 262144
    assert two["steps"] == one["steps"] == 3 and two["value"] > 0 and one["value"] > 0
