"""Multi-GPU layout: one process per GPU, env instances sharded contiguously.

Rank r of W owns global env ids [r * n, (r + 1) * n); env id i is seeded
base_seed + i, so the union of the shards is the same batch a single process
with W * n envs would run.  Instances are independent,
so stepping needs no collective.  The north star's exchange -- every rank gets
the whole node's step results -- is one all-gather per step:

* each rank's step outputs (observations, reward, done, eval_score[, target])
  live in ONE packed u8 buffer (PackedLayout): the simulator writes straight
  into its key views (VecMagicalEnv.bind_outputs), so there is no pack copy;
* one ``all_gather_into_tensor`` of that buffer (RCCL over xGMI with the
  "nccl" process group, gloo for CPU tensors in the tests) yields [W, bytes];
  PackedLayout.unpack turns it into per-key [W, n, ...] views, again without
  a copy (global env id = r * n + i);
* two such buffers alternate between steps and the collective runs on its own
  HIP stream, so the gather of step t overlaps the compute of step t + 1
  (ShardedVecEnv.step_async).  A step's gathered views stay valid until the
  step after next.
"""
import collections

import numpy as np
import torch
import torch.distributed as dist

_ALIGN = 256  # byte alignment of every key inside the packed buffer (the simulator needs 16)


def shard_range(envs_per_rank, rank):
    return rank * envs_per_rank, (rank + 1) * envs_per_rank


def shard_seeds(envs_per_rank, rank, base_seed=1000):
    lo, hi = shard_range(envs_per_rank, rank)
    return [base_seed + i for i in range(lo, hi)]


def all_gather_batch(tensors, group=None):
    """Gather a dict of per-rank [n, ...] tensors into [W * n, ...] on every rank,
    global env order (rank-major).  One collective per key (the unpacked form;
    ShardedVecEnv uses one packed collective per step instead)."""
    world = dist.get_world_size(group)
    out = {}
    for k, t in tensors.items():
        t = t.contiguous()
        full = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(full, t, group=group)
        out[k] = full
    return out


class PackedLayout:
    """Byte layout of one rank's step outputs in a single u8 buffer: per key a contiguous [n, ...]
    block at a 256-byte aligned offset, in the order of `fields` (name, per-env shape, dtype)."""

    def __init__(self, n, fields):
        self.n = int(n)
        self.fields = []
        off = 0
        for name, shape, dtype in fields:
            shape = tuple(shape)
            nb = self.n * int(np.prod(shape, dtype=np.int64)) * torch.empty((), dtype=dtype).element_size()
            self.fields.append((name, shape, dtype, off, nb))
            off = (off + nb + _ALIGN - 1) // _ALIGN * _ALIGN
        self.nbytes = off

    @classmethod
    def for_spec(cls, spec, n):
        """The fields VecMagicalEnv.output_buffers() binds for a registry spec (raw HWC observations)."""
        from . import registry
        from .envs import _obs_shapes
        if spec.preproc is None:
            raise ValueError("packed gather: the unwrapped 384^2 view is rendered on demand, not bound")
        chw = registry.PREPROCESSORS[spec.preproc].get("channels_first", False)
        fields = []
        for k, s in _obs_shapes(spec).items():
            fields.append((k, (s[1], s[2], s[0]) if chw else s, torch.uint8))   # buffers are HWC
        fields += [("reward", (), torch.float32), ("done", (), torch.bool), ("eval_score", (), torch.float64)]
        if spec.task == "PickAndPlace":
            fields.append(("target", (4,), torch.float64))
        lay = cls(n, fields)
        lay.chw = chw
        return lay

    def views(self, buf):
        """Per-key [n, ...] views into one rank's packed buffer (u8, nbytes)."""
        assert buf.dtype == torch.uint8 and buf.numel() == self.nbytes and buf.is_contiguous()
        out = collections.OrderedDict()
        for name, shape, dtype, off, nb in self.fields:
            out[name] = buf[off:off + nb].view(dtype).view((self.n,) + shape)
        return out

    def unpack(self, gathered):
        """Per-key [W, n, ...] views into the gathered buffer (u8, W * nbytes, rank-major)."""
        world = gathered.numel() // self.nbytes
        g = gathered.view(world, self.nbytes)
        out = collections.OrderedDict()
        for name, shape, dtype, off, nb in self.fields:
            out[name] = g[:, off:off + nb].view(dtype).view((world, self.n) + shape)
        return out


class GatheredStep:
    """Handle of one step's packed all-gather: wait() orders the caller's current stream after it."""

    def __init__(self, layout, recv, work):
        self.layout, self.recv, self.work = layout, recv, work

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
        return self

    def results(self):
        """(obs dict of [W, n, ...] observation views, reward, done, info={'eval_score'[, 'target']}), all [W, n...]"""
        self.wait()
        v = self.layout.unpack(self.recv)
        if getattr(self.layout, "chw", False):   # as VecMagicalEnv returns them: channels-first views
            for k in [k for k in v if v[k].dim() == 5]:
                v[k] = v[k].permute(0, 1, 4, 2, 3)
        info = {"eval_score": v.pop("eval_score")}
        if "target" in v:
            info["target"] = v.pop("target")
        rew, done = v.pop("reward"), v.pop("done")
        return v, rew, done, info


class ShardedVecEnv:
    """This rank's shard of a node-wide batch of envs (VecMagicalEnv underneath).

    gather=True: every step's results of all ranks are all-gathered to every rank through one packed
    buffer (see the module docstring); step() returns the gathered [W, n, ...] views, step_async() the
    handle without waiting, so the collective of step t overlaps step t + 1."""

    def __init__(self, env_name, envs_per_rank, rank=None, device=None, base_seed=1000, gather=False, vec=None):
        from . import registry
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.envs_per_rank = envs_per_rank
        self.gather = gather
        if vec is None:
            from .envs import VecMagicalEnv
            vec = VecMagicalEnv(env_name, envs_per_rank, device=device or f"cuda:{torch.cuda.current_device()}",
                                seeds=shard_seeds(envs_per_rank, self.rank, base_seed))
        self.vec = vec
        if gather:
            self.layout = PackedLayout.for_spec(registry.lookup(env_name), envs_per_rank)
            dev = torch.device(device) if device is not None else getattr(vec, "device", torch.device("cpu"))
            self.device = dev
            self.send = [torch.empty(self.layout.nbytes, dtype=torch.uint8, device=dev) for _ in range(2)]
            self.recv = [torch.empty(self.world * self.layout.nbytes, dtype=torch.uint8, device=dev) for _ in range(2)]
            self.pending = [None, None]
            self.comm_stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
            self.t = 0

    # -- packed gather pipeline ---------------------------------------------------------------------------
    def _begin(self):
        """Buffer of this step: the gather that last read it (two steps ago) must be done first."""
        b = self.t % 2
        if self.pending[b] is not None:
            self.pending[b].wait()
            self.pending[b] = None
        self.vec.bind_outputs(self.layout.views(self.send[b]))
        return b

    def _launch(self, b):
        send, recv = self.send[b], self.recv[b]
        if self.comm_stream is not None:
            ev = torch.cuda.current_stream(self.device).record_event()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                work = dist.all_gather_into_tensor(recv, send, async_op=True)
                send.record_stream(self.comm_stream)
                recv.record_stream(self.comm_stream)
        else:
            work = dist.all_gather_into_tensor(recv, send, async_op=True)
        h = GatheredStep(self.layout, recv, work)
        self.pending[b] = h
        self.t += 1
        return h

    def reset_async(self):
        b = self._begin()
        self.vec.reset()
        return self._launch(b)

    def step_async(self, actions):
        b = self._begin()
        self.vec.step(actions)
        return self._launch(b)

    # -- gym-style ------------------------------------------------------------------------------------------
    def reset(self):
        if self.gather:
            return self.reset_async().results()[0]
        return self.vec.reset()

    def step(self, actions):
        if self.gather:
            return self.step_async(actions).results()
        return self.vec.step(actions)

    def close(self):
        for h in getattr(self, "pending", []):
            if h is not None:
                h.wait()
        self.vec.close()
