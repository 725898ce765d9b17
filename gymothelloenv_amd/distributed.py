"""Multi-GPU: one process per GPU, boards sharded by contiguous global env id.

Boards are independent, so a step has no data-path
collective: every rank steps its own shard.  The only exchange is the
win/draw/loss tally (the harnesses' W/D/L counting, run.py:100-130,
ppo_run_self_play.py:432-441): one all-gather of int64[3] per reporting window
-- RCCL over xGMI with the "nccl" backend on MI355X, gloo on CPU.  Because the
Philox key is (seed, global env id, ply), results do not depend on the number
of ranks.
"""
import torch
import torch.distributed as dist


def shard(global_envs, world, rank):
    """Contiguous range of global env ids for `rank`: (env_id_base, n_local).
    The first (global_envs % world) ranks take one extra board."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world %d" % (rank, world))
    q, r = divmod(int(global_envs), int(world))
    n_local = q + (1 if rank < r else 0)
    base = rank * q + min(rank, r)
    return base, n_local


def gather_wdl(counts, group=None):
    """All-gather every rank's {black wins, draws, white wins} -> (world, 3) int64."""
    world = dist.get_world_size(group)
    counts = counts.reshape(3).to(torch.int64).contiguous()
    if dist.get_backend(group) == "nccl":
        out = torch.empty(world * 3, dtype=torch.int64, device=counts.device)
        dist.all_gather_into_tensor(out, counts, group=group)
        return out.view(world, 3)
    host = counts.cpu()  # gloo: host tensors
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host, group=group)
    return torch.stack(parts).to(counts.device)


def total_wdl(counts, group=None):
    return gather_wdl(counts, group).sum(0)


class ShardedVecOthelloEnv(object):
    """This rank's shard of a global batch of boards (one process per GPU)."""

    def __init__(self, global_envs, rank=None, world=None, device=None, **kw):
        from .vec_env import VecOthelloEnv
        rank = dist.get_rank() if rank is None else rank
        world = dist.get_world_size() if world is None else world
        self.rank, self.world, self.global_envs = rank, world, global_envs
        self.env_id_base, self.num_envs = shard(global_envs, world, rank)
        self.env = VecOthelloEnv(self.num_envs, env_id_base=self.env_id_base, device=device, **kw)

    def __getattr__(self, name):
        return getattr(self.env, name)

    def global_counts(self, reset=False, group=None):
        """W/D/L summed over every rank (one all-gather)."""
        return total_wdl(self.env.counts(reset=reset), group)
