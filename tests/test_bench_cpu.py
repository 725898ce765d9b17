"""bench.py's launcher and bookkeeping on CPU (no GPU call): the N-rank spawn
path with a gloo process group up to the shard plan, the WORLD_SIZE / --gpus
check, the §8(d) byte model and the default board counts per config."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)


def test_step_bytes_follow_survey_8d():
    assert bench.step_bytes(1) == 51  # 6x6 and 8x8
    assert bench.step_bytes(2) == 91  # 10x10
    assert bench.step_bytes(4) == 171  # 16x16


def test_plan_defaults_per_config():
    a = bench.parse_args([])
    assert (a.steps, a.warmup) == (50, 10)
    assert bench.plan(a, 1, 0) == (65536, 0, 65536, 100)  # config 2
    a8 = bench.parse_args(["--gpus", "8"])
    G, base, E, P = bench.plan(a8, 8, 7)
    assert (G, base, E) == (1048576, 7 * 131072, 131072)  # config 4
    g = bench.parse_args(["--global-envs", "1000", "--gpus", "3"])
    assert [bench.plan(g, 3, r)[1:3] for r in range(3)] == [(0, 334), (334, 333), (667, 333)]
    assert bench.plan(bench.parse_args(["--policy", "greedy"]), 1, 0)[3] == 10
    with pytest.raises(SystemExit):
        bench.plan(bench.parse_args(["--envs", "5", "--global-envs", "10"]), 1, 0)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_spawned_ranks_cover_the_global_boards(world):
    """--gpus N without WORLD_SIZE: bench.py starts N ranks (RANK/LOCAL_RANK/
    WORLD_SIZE set), they form a gloo group and all-gather their shard plans."""
    r = _run(["--gpus", str(world), "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout  # rank 0 prints exactly one JSON line
    d = json.loads(line[0])
    assert d["world"] == world and d["global_envs"] == world * 131072
    shards = sorted(d["shards"])
    assert [s[0] for s in shards] == list(range(world))
    nxt = 0
    for rank, base, n in shards:  # contiguous global env ids, no gap or overlap
        assert base == nxt and n == 131072
        nxt += n
    assert nxt == d["global_envs"]
    # the record's keys at N > 1 (numbers are null in a dry run): the scaling reading aids
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline", "config",
              "per_gpu_value", "single_gpu_same_shard", "ranks", "shared_device"):
        assert k in d, k
    assert d["n_gpus"] == world and d["ranks"] == world and d["shared_device"] is False
    assert d["config"]["boards_per_gpu"] == 131072 and d["roofline"]["bound"] == "valu-issue"


def test_driver_torchrun_launch_of_eight_ranks():
    """The driver's own N = 8 command (torch.distributed.run, one rank per GPU,
    127.0.0.1 rendezvous) as a dry run on CPU ranks: the launch, the WORLD_SIZE
    check, the shard plan of config 4 and rank 0's single JSON line."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run"],
                       env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    d = json.loads(line[0])
    assert d["world"] == 8 and d["n_gpus"] == 8 and d["global_envs"] == 1048576
    assert sorted(d["shards"]) == [[k, k * 131072, 131072] for k in range(8)]
    assert d["config"]["boards_per_gpu"] == 131072 and d["scaling"] == "weak"


def test_shared_device_rehearsal_is_labelled():
    """Ranks pinned to one device (OTH_BENCH_DEVICE) report one distinct GPU."""
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"OTH_BENCH_DEVICE": "0"})
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["shared_device"] is True and d["n_gpus"] == 1 and d["ranks"] == 2


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_single_rank_dry_run():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["shards"] == [[0, 0, 65536]] and d["plies_per_step"] == 100


def test_fused_path_pmc_records_are_committed():
    """The bench's step_observe entries name committed PMC records (traffic per
    launch within a few percent of the algorithmic bytes: no re-reads)."""
    import bench
    for key in ("step-observe-board-int64-8x8-E65536", "sample-step-make-state-f32-8x8-E65536"):
        rec = bench.load_pmc(key)
        assert rec and rec["source"].startswith("profiles/")
        assert 0.95 < rec["hbm_bytes_per_launch"] / rec["algorithmic_bytes_per_launch"] < 1.1
        assert bench.pmc_ref(key)["hbm_bytes_per_launch"] > 0
