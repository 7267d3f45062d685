"""Multi-GPU layout: one process per GPU, env instances sharded contiguously.

Rank r of W owns global env ids [r * n, (r + 1) * n); env id i is seeded
base_seed + i, so the union of the shards is the same batch a single process
with W * n envs would run.  Instances are independent,
so stepping needs no collective; the only exchange is the optional gather of
the observation batch to every rank (RCCL all-gather over xGMI when the
process group is "nccl", gloo on CPU tensors in the tests).
"""
import torch
import torch.distributed as dist


def shard_range(envs_per_rank, rank):
    return rank * envs_per_rank, (rank + 1) * envs_per_rank


def shard_seeds(envs_per_rank, rank, base_seed=1000):
    lo, hi = shard_range(envs_per_rank, rank)
    return [base_seed + i for i in range(lo, hi)]


def all_gather_batch(tensors, group=None):
    """Gather a dict of per-rank [n, ...] tensors into [W * n, ...] on every rank,
    global env order (rank-major).  One collective per key, written straight
    into the output buffer (all_gather_into_tensor)."""
    world = dist.get_world_size(group)
    out = {}
    for k, t in tensors.items():
        t = t.contiguous()
        full = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(full, t, group=group)
        out[k] = full
    return out


class ShardedVecEnv:
    """This rank's shard of a node-wide batch of envs (VecMagicalEnv underneath)."""

    def __init__(self, env_name, envs_per_rank, rank=None, device=None, base_seed=1000, gather=False):
        from .envs import VecMagicalEnv
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.envs_per_rank = envs_per_rank
        self.gather = gather
        self.vec = VecMagicalEnv(env_name, envs_per_rank, device=device or f"cuda:{torch.cuda.current_device()}",
                                 seeds=shard_seeds(envs_per_rank, self.rank, base_seed))

    def _out(self, obs):
        return all_gather_batch(obs) if self.gather and self.world > 1 else obs

    def reset(self):
        return self._out(self.vec.reset())

    def step(self, actions):
        obs, rew, done, info = self.vec.step(actions)
        return self._out(obs), rew, done, info

    def close(self):
        self.vec.close()
