"""Multi-process path on CPU (gloo, world_size 2 and 4): sharding by global env
id plus the W/D/L all-gather reproduce a single-process run exactly.  The
per-shard play is the CPU oracle here (no GPU); on the GPU box the same code
runs the HIP engine over RCCL (bench.py, tests/test_gpu_parity.py
::test_sharding_is_invisible)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gymothelloenv_amd.distributed import gather_wdl, shard, total_wdl

GLOBAL_E, PLIES, SEED = 1000, 130, 17


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, q):
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        base, n = shard(GLOBAL_E, world, rank)
        s = oracle.reset(8, n)
        acts, _, _, wdl = oracle.rollout(s, oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET, 0, PLIES,
                                         seed=SEED, id_base=base)
        per_rank = gather_wdl(torch.from_numpy(wdl))
        tot = total_wdl(torch.from_numpy(wdl))
        acts_all = [torch.empty(PLIES * (GLOBAL_E // world + 1), dtype=torch.int32) for _ in range(world)]
        pad = torch.full((PLIES, GLOBAL_E // world + 1), -9, dtype=torch.int32)
        pad[:, :n] = torch.from_numpy(acts)
        dist.all_gather(acts_all, pad.reshape(-1))
        if rank == 0:
            q.put((per_rank.numpy(), tot.numpy(), [a.numpy() for a in acts_all]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_rollout_equals_single_process(world):
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    per_rank, tot, acts_all = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = oracle.reset(8, GLOBAL_E)
    acts, _, _, wdl = oracle.rollout(s, oracle.F_SUDDEN_DEATH | oracle.F_AUTO_RESET, 0, PLIES, seed=SEED)
    np.testing.assert_array_equal(tot, wdl)
    assert per_rank.shape == (world, 3) and (per_rank.sum(0) == wdl).all()
    cols = []
    for r in range(world):
        _, n = shard(GLOBAL_E, world, r)
        cols.append(acts_all[r].reshape(PLIES, -1)[:, :n])
    np.testing.assert_array_equal(np.concatenate(cols, axis=1), acts)


def test_shard_partition():
    for total in (1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            ranges = [shard(total, world, r) for r in range(world)]
            assert sum(n for _, n in ranges) == total
            pos = 0
            for base, n in ranges:
                assert base == pos
                pos += n
            assert max(n for _, n in ranges) - min(n for _, n in ranges) <= 1
    assert shard(1 << 20, 8, 3) == (3 * 131072, 131072)  # config 4: 131,072 boards per GPU
    with pytest.raises(ValueError):
        shard(10, 2, 2)
