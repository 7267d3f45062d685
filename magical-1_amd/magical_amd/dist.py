"""Multi-GPU layout: one process per GPU, env instances sharded contiguously.

Rank r of W owns global env ids [r * n, (r + 1) * n); env id i is seeded
base_seed + i, so the union of the shards is the same batch a single process
with W * n envs would run.  Instances are independent,
so stepping needs no collective.  The north star's exchange -- every rank gets
the whole node's step results -- is one all-gather per step:

* each rank's step outputs live in ONE packed u8 buffer (PackedLayout): the
  simulator writes straight into its key views (VecMagicalEnv.bind_outputs),
  so there is no pack copy;
* one ``all_gather_into_tensor`` of that buffer (RCCL over xGMI with the
  "nccl" process group, gloo for CPU tensors in the tests) yields [W, bytes];
  PackedLayout.unpack turns it into per-key [W, n, ...] views without a copy
  (global env id = r * n + i);
* gather_mode "frames" (default): the packed buffer holds only the CURRENT
  LoRes frame of each view plus reward / done / eval_score[, target] -- 55 312
  B per env instead of 165 904 (LoRes4E) or 221 200 (LoResStack) -- because 3
  of every 4 stacked frames already reached every rank in earlier steps.  Each
  receiver keeps the frame stacks of all W * n envs as a window ring
  (WindowRestacker, mg_restack_window, round 5): every received frame is
  written once, channel-planar, into a ring of K + 3 slots per env, and the
  stack of step t is a strided view of 4 consecutive slots -- 1 frame read and
  ~1.4 written per env and stacked view instead of materialising the stack (9
  frame passes; NativeRestacker, mg_restack, still used for LoRes3EA, whose
  stack is not one ring's window).  The reset frame fills every slot as in
  benchmarks/__init__.py:75-82,139-147, and an env whose done flag is set
  restarts its stacks (its frame is the next episode's first).  The simulator
  binds its outputs in frames-only mode, so it writes no stacks of its own.
  gather_mode "stacked" gathers the preprocessor's whole outputs instead;
* `nbuf` buffer sets (default 3) rotate between steps; the collective runs on its
  own HIP stream and the restack on a third (in step order), so the exchange of
  step t overlaps the compute of steps t + 1 .. t + nbuf - 1 and the restack of
  step t (HBM-bound) overlaps the all-gather of step t + 1 (xGMI-bound)
  (ShardedVecEnv.step_async).  A step's gathered frames, rewards, done flags and
  scores stay valid for the next nbuf - 1 steps; its stacked views (window
  ring) until the next step_async() / reset_async() -- work the caller queued
  on its stream before that call is ordered before the ring is rewritten (as a
  VecMagicalEnv's outputs are valid until its next step).
* the env underneath may be a magical_amd.pipeline.PipelinedVecEnv (chunks > 1):
  the collective then waits for every chunk's stream of the step, so the chunks
  keep overlapping one another's kernels under the exchange.
"""
import collections

import numpy as np
import torch
import torch.distributed as dist

_ALIGN = 256  # byte alignment of every key inside the packed buffer (the simulator needs 16)
LOFR = 96 * 96 * 3  # bytes of one LoRes RGB frame


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


# mg_restack / mg_bind_outputs preprocessor ids (include/magical_sim.h)
GPU_PREPROC = {"LoRes4E": 1, "LoResCHW4E": 1, "LoResCHW4A": 1, "LoResStack": 2, "LoRes3EA": 3, "LoRes4A": 4}


def stacked_keys(preproc):
    """Keys whose values are 4-frame stacks (rebuilt on the receivers in gather_mode 'frames')."""
    return ("allo", "ego") if preproc == "LoResStack" else ("past_obs",)


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
        self.chw = False
        self.frames_only = False

    @classmethod
    def for_spec(cls, spec, n, frames_only=False):
        """The fields VecMagicalEnv.output_buffers() binds for a registry spec (raw HWC observations);
        frames_only: the current frame of each view instead of the preprocessor's stacks."""
        from . import registry
        from .envs import _obs_shapes
        if spec.preproc is None:
            raise ValueError("packed gather: the unwrapped 384^2 view is rendered on demand, not bound")
        chw = registry.PREPROCESSORS[spec.preproc].get("channels_first", False)
        fields = []
        if frames_only:
            fields += [("allo", (96, 96, 3), torch.uint8), ("ego", (96, 96, 3), torch.uint8)]
        else:
            for k, s in _obs_shapes(spec).items():
                fields.append((k, (s[1], s[2], s[0]) if chw else s, torch.uint8))   # buffers are HWC
        fields += [("reward", (), torch.float32), ("done", (), torch.bool), ("eval_score", (), torch.float64)]
        if spec.task == "PickAndPlace":
            fields.append(("target", (4,), torch.float64))
        lay = cls(n, fields)
        lay.chw = chw
        lay.frames_only = frames_only
        lay.preproc = spec.preproc
        return lay

    def offset(self, name):
        return next(f[3] for f in self.fields if f[0] == name)

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


def restack_ring_bytes(preproc, world, n):
    """Bytes of mg_restack's receive ring: the last 4 frames of every stacked output's view for all W * n envs,
    u8[stacks][4][W * n][96 * 96 * 3] (LoResStack: 2 stacks, allo and ego; else 1)."""
    return len(stacked_keys(preproc)) * 4 * world * n * LOFR


WINDOW_K = 8   # window ring period: K + 3 slots per env and stack, 3 / K extra frame writes per step


def window_ring_bytes(preproc, world, n, K=WINDOW_K):
    """Bytes of mg_restack_window's ring: u8[stacks][W * n][K + 3][3][96][96]."""
    return len(stacked_keys(preproc)) * world * n * (K + 3) * LOFR


def uses_window(preproc):
    """The stacks of these preprocessors are windows of one ring (LoRes3EA's is not: allo frame + 3 ego)."""
    return preproc != "LoRes3EA"


def frames_mode_bytes(preproc, world, n, nbuf=3):
    """Receiver-side device memory of gather_mode 'frames' per rank: the window ring (LoRes3EA: mg_restack's
    ring plus nbuf sets of rebuilt stacks, u8[W * n][96][96][12] per set)."""
    if uses_window(preproc):
        return window_ring_bytes(preproc, world, n)
    return restack_ring_bytes(preproc, world, n) + nbuf * len(stacked_keys(preproc)) * world * n * 4 * LOFR


def window_view(ring, k, wn, s0, K=WINDOW_K):
    """Stack k's [wn, 96, 96, 12] view of the window ring at window start slot s0 (include/magical_sim.h
    mg_restack_window): channel c = plane c % 3 of slot s0 + c // 3."""
    plane = 96 * 96
    return ring.as_strided((wn, 96, 96, 12), ((K + 3) * LOFR, 96, 1, plane),
                           ring.storage_offset() + (k * wn * (K + 3) + s0) * LOFR)


_HIP = None


def _emulate_all_gather(recv, send, world, stream):
    """bench.py --emulate-world: the receive-side HBM writes of an all-gather of `world` ranks, without peers --
    `send` copied into each of the `world` blocks of `recv` by the DMA engines (hipMemcpyAsync
    hipMemcpyDeviceToDeviceNoCU), as xGMI peer writes land in HBM without this GPU's compute units; falls back
    to a copy kernel if the runtime refuses.  Returns which was used."""
    global _HIP
    import ctypes
    nb = send.numel()
    if _HIP is None:
        try:
            _HIP = ctypes.CDLL("libamdhip64.so")
            _HIP.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_void_p]
        except OSError:
            _HIP = False
    if _HIP:
        rc = 0
        for r in range(world):
            rc = rc or _HIP.hipMemcpyAsync(recv.data_ptr() + r * nb, send.data_ptr(), nb, 1024, stream.cuda_stream)
        if rc == 0:
            return "sdma"
    recv.view(world, -1).copy_(send.unsqueeze(0).expand(world, -1))
    return "kernel"


class NativeRestacker:
    """Receiver-side frame stacks of the frames-only gather on the GPU (mg_restack): keeps a ring of the
    last 4 frames of each stacked output's view for all W * n envs (restack_ring_bytes) and writes every
    step's stacks into `outs` (materialised: 9 frame passes per env and stack; LoRes3EA, and the contiguous
    reference the window ring is tested against)."""

    materialized = True

    def __init__(self, layout, world, device):
        from . import native
        self.lib, self.native = native.load(), native
        self.layout, self.world = layout, world
        self.preproc = GPU_PREPROC[layout.preproc]
        self.ring = torch.empty(restack_ring_bytes(layout.preproc, world, layout.n), dtype=torch.uint8,
                                device=device)
        self.off = (layout.offset("allo"), layout.offset("ego"), layout.offset("done"))

    def __call__(self, recv, outs, step, all_fresh):
        import ctypes
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        st = ctypes.c_void_p(torch.cuda.current_stream(recv.device).cuda_stream)
        self.native.check(self.lib.mg_restack(
            p(recv), self.world, self.layout.n, self.layout.nbytes, self.off[0], self.off[1], self.off[2],
            self.preproc, int(step), 1 if all_fresh else 0, p(self.ring), p(outs.get("allo")), p(outs.get("ego")),
            p(outs.get("past_obs")), st))


class WindowRestacker:
    """Receiver-side frame stacks of the frames-only gather as a window ring on the GPU (mg_restack_window):
    __call__ returns the step's stacks as strided views of the ring (valid until the next call is ordered
    after their readers); nothing is materialised."""

    materialized = False

    def __init__(self, layout, world, device, K=WINDOW_K):
        from . import native
        if not uses_window(layout.preproc):
            raise ValueError(f"{layout.preproc}: the stack is not a window of one ring (use NativeRestacker)")
        self.lib, self.native = native.load(), native
        self.layout, self.world, self.K = layout, world, int(K)
        self.preproc = GPU_PREPROC[layout.preproc]
        self.keys = stacked_keys(layout.preproc)
        self.wn = world * layout.n
        self.ring = torch.empty(window_ring_bytes(layout.preproc, world, layout.n, self.K), dtype=torch.uint8,
                                device=device)
        self.off = (layout.offset("allo"), layout.offset("ego"), layout.offset("done"))

    def __call__(self, recv, outs, step, all_fresh):
        import ctypes
        st = ctypes.c_void_p(torch.cuda.current_stream(recv.device).cuda_stream)
        self.native.check(self.lib.mg_restack_window(
            ctypes.c_void_p(recv.data_ptr()), self.world, self.layout.n, self.layout.nbytes, self.off[0], self.off[1],
            self.off[2], self.preproc, int(step), 1 if all_fresh else 0, self.K, ctypes.c_void_p(self.ring.data_ptr()),
            st))
        s0 = (int(step) + self.K - 3) % self.K
        return collections.OrderedDict((k, window_view(self.ring, j, self.wn, s0, self.K))
                                       for j, k in enumerate(self.keys))


class GatheredStep:
    """Handle of one step's exchange: wait() orders the caller's current stream after it (the all-gather
    and, in gather_mode 'frames', the receiver-side restack)."""

    def __init__(self, layout, recv, stacks, work=None, event=None, owner=None, step=None, windowed=False):
        self.layout, self.recv, self.stacks, self.work, self.event = layout, recv, stacks, work, event
        # window-ring stacks (WindowRestacker) are views of one ring that the next exchange rewrites: remember
        # which shard step made them so that a late results() raises instead of returning the next frames
        self.owner, self.step, self.windowed = owner, step, windowed

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
        if self.event is not None:
            torch.cuda.current_stream(self.recv.device).wait_event(self.event)
        return self

    def results(self):
        """(obs dict of [W, n, ...] observation views, reward, done, info={'eval_score'[, 'target']}), all [W, n...]:
        observation keys and order as VecMagicalEnv returns them (PickAndPlace: allo, ego, target_type,
        target_colour, target_position[, past_obs])."""
        if self.windowed and self.owner is not None and self.owner.t > self.step + 1:
            raise RuntimeError(f"GatheredStep.results(): the stacked views of shard step {self.step} are window-ring "
                               f"views, valid only until the next step_async() / reset_async() (the shard is at "
                               f"step {self.owner.t}); read results() before issuing the next step, or build the "
                               "ShardedVecEnv with window=False for stacks that stay valid for nbuf - 1 steps")
        self.wait()
        v = self.layout.unpack(self.recv)
        world, n = v["reward"].shape
        for k, t in (self.stacks or {}).items():   # rebuilt frame stacks replace / add their keys
            v[k] = t.view(world, n, 96, 96, 12)
        if self.layout.chw:   # as VecMagicalEnv returns them: channels-first views
            for k in [k for k in v if v[k].dim() == 5]:
                v[k] = v[k].permute(0, 1, 4, 2, 3)
        info = {"eval_score": v.pop("eval_score")}
        rew, done = v.pop("reward"), v.pop("done")
        obs = collections.OrderedDict([("allo", v.pop("allo")), ("ego", v.pop("ego"))])
        if "target" in v:
            t = info["target"] = v.pop("target")
            t32 = t.to(torch.float32)
            obs["target_type"], obs["target_colour"], obs["target_position"] = t32[..., 0:1], t32[..., 1:2], t32[..., 2:4]
        if "past_obs" in v:
            obs["past_obs"] = v.pop("past_obs")
        return obs, rew, done, info


class ShardedVecEnv:
    """This rank's shard of a node-wide batch of envs (VecMagicalEnv underneath).

    gather=True: every step's results of all ranks reach every rank (see the module docstring); step()
    returns the gathered [W, n, ...] views, step_async() the handle without waiting, so the exchange of
    step t overlaps step t + 1.  gather_mode 'frames' (default on GPU tensors) all-gathers only the current
    frames and rebuilds the stacks on each receiver (`restacker`: NativeRestacker on the GPU; CPU tensors need
    one passed in -- the gloo tests use the oracle's); 'stacked' (default on CPU tensors) all-gathers the
    whole observations.  In 'frames' mode the receivers' rings are valid only from reset_async() on:
    step_async() raises before the shard's first reset_async() and after the VecMagicalEnv underneath was
    reset directly (vec.reset()), since the other ranks' rings would then hold stale frames of its envs."""

    def __init__(self, env_name, envs_per_rank, rank=None, device=None, base_seed=1000, gather=False, vec=None,
                 gather_mode=None, restacker=None, max_episode_steps=None, emulate_world=None, nbuf=3, window=True,
                 chunks=1):
        from . import registry
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        # measurement only (bench.py --emulate-world W): one process stands in for rank 0 of a W-rank node --
        # the all-gather is replaced by a device copy of this rank's buffer into all W receive blocks (the
        # HBM writes a real all-gather makes on the receiver), and the restack rebuilds W * n envs' stacks
        self.emulate_world = None
        if emulate_world and emulate_world > 1:
            if self.world != 1:
                raise ValueError("emulate_world is a single-process measurement mode")
            self.emulate_world = self.world = int(emulate_world)
        self.envs_per_rank = envs_per_rank
        self.gather = gather
        spec = registry.lookup(env_name)
        if vec is None:
            dev_name = device or f"cuda:{torch.cuda.current_device()}"
            seeds = shard_seeds(envs_per_rank, self.rank, base_seed)
            if chunks > 1:   # the pipelined env pool (magical_amd.pipeline): chunks overlap under the exchange
                # (PickAndPlace: the pool copies its target into the packed view on each chunk's stream)
                from .pipeline import PipelinedVecEnv
                vec = PipelinedVecEnv(env_name, envs_per_rank, chunks=chunks, device=dev_name, seeds=seeds,
                                      max_episode_steps=max_episode_steps, window=False)
            else:
                from .envs import VecMagicalEnv
                # the shard's outputs are bound into the packed buffers (frames: current frames only; stacked:
                # materialised stacks), so no window rings on the simulator
                vec = VecMagicalEnv(env_name, envs_per_rank, device=dev_name, seeds=seeds,
                                    max_episode_steps=max_episode_steps, window=False)
        self.vec = vec
        if gather:
            dev = torch.device(device) if device is not None else getattr(vec, "device", torch.device("cpu"))
            if gather_mode is None:
                gather_mode = "frames" if dev.type == "cuda" or restacker is not None else "stacked"
            if gather_mode not in ("frames", "stacked"):
                raise ValueError(f"gather_mode must be 'frames' or 'stacked', not {gather_mode!r}")
            self.gather_mode = gather_mode
            frames = gather_mode == "frames"
            self.layout = PackedLayout.for_spec(spec, envs_per_rank, frames_only=frames)
            self.stacked_nbytes = PackedLayout.for_spec(spec, envs_per_rank).nbytes
            self.device = dev
            # nbuf buffer sets: the compute of step t + nbuf - 1 may start before the exchange of step t is done
            # (measured with 8 emulated ranks, round 4: the exchange of a step takes longer than its compute)
            self.nbuf = nb = int(nbuf)
            if nb < 2:
                raise ValueError("nbuf must be >= 2")
            self.send = [torch.empty(self.layout.nbytes, dtype=torch.uint8, device=dev) for _ in range(nb)]
            self.recv = [torch.empty(self.world * self.layout.nbytes, dtype=torch.uint8, device=dev) for _ in range(nb)]
            self.stacks = [None] * nb
            if frames:
                if restacker is None:
                    if dev.type != "cuda":
                        raise ValueError("gather_mode 'frames' on CPU tensors needs a restacker")
                    restacker = (WindowRestacker(self.layout, self.world, dev) if uses_window(spec.preproc) and
                                 window else NativeRestacker(self.layout, self.world, dev))
                wn = self.world * envs_per_rank
                # materialised stacks (mg_restack, the oracle's restacker): one set per buffer set; the window
                # ring's views need none
                self.stacks = [collections.OrderedDict((k, torch.empty((wn, 96, 96, 12), dtype=torch.uint8, device=dev))
                                                       for k in stacked_keys(spec.preproc))
                               if getattr(restacker, "materialized", True) else {} for _ in range(nb)]
            self.restacker = restacker
            self.pending = [None] * nb
            self.comm_stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
            # the restack has its own stream: restack(t) (HBM-bound) overlaps gather(t + 1) (xGMI-bound)
            self.restack_stream = torch.cuda.Stream(dev) if dev.type == "cuda" and frames else None
            self.restacked = [None] * nb    # per buffer set: event after the restack that last read recv[b]
            self.t = 0
            self._ring_resets = None        # vec.reset_count at the last reset_async (frames mode: ring valid)
            self.restack_timing = False
            self.emulated_copy = None
            self._restack_ev = []

    def enable_restack_timing(self):
        """time every following exchange (on the comm stream) and restack (on the restack stream) with HIP
        events (bench.py)"""
        self.restack_timing = self.restack_stream is not None
        self._restack_ev = []
        self._comm_ev = []

    @staticmethod
    def _total_ms(pairs):
        tot = 0.0
        for a, b in pairs:
            b.synchronize()
            tot += a.elapsed_time(b)
        return tot

    def restack_ms(self):
        """total ms of the restacks timed since enable_restack_timing (synchronises on the last one)"""
        return self._total_ms(self._restack_ev)

    def exchange_ms(self):
        """total ms of the all-gathers (or their --emulate-world copies) on the comm stream, from the collective's
        first operation to its last (the wait for the step's compute is not counted)"""
        return self._total_ms(getattr(self, "_comm_ev", []))

    # -- packed gather pipeline ---------------------------------------------------------------------------
    def _begin(self):
        """Buffer set of this step: the exchange that last used it (two steps ago) must be done first."""
        b = self.t % self.nbuf
        if self.pending[b] is not None:
            self.pending[b].wait()
            self.pending[b] = None
        self.vec.bind_outputs(self.layout.views(self.send[b]), frames_only=self.layout.frames_only)
        return b

    def _finish_outputs(self, b):
        # PickAndPlace's target is written by the simulator only at reset: copy the env's persistent
        # buffer into this step's packed views (never gather a stale or unwritten target)
        # (a pipelined pool copies its target into the bound "target" view itself, on each chunk's stream right
        # after the chunk's step: PipelinedVecEnv.bind_outputs)
        if self.layout.fields[-1][0] == "target" and not self._pooled():
            self.layout.views(self.send[b])["target"].copy_(self.vec.target)

    def _pooled(self):
        return self.comm_stream is not None and hasattr(self.vec, "step_events")

    def _launch(self, b, all_fresh):
        send, recv, stacks = self.send[b], self.recv[b], self.stacks[b]
        step = self.t
        if self.comm_stream is not None:
            ev = torch.cuda.current_stream(self.device).record_event()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                for cev in getattr(self.vec, "step_events", lambda: [])():   # a pipelined pool's chunk streams
                    self.comm_stream.wait_event(cev)
                if self.restacked[b] is not None:   # the restack of step t - 2 has read recv[b]
                    self.comm_stream.wait_event(self.restacked[b])
                if self.restack_timing:
                    c0 = torch.cuda.Event(enable_timing=True)
                    c0.record(self.comm_stream)
                if self.emulate_world:
                    self.emulated_copy = _emulate_all_gather(recv, send, self.world, self.comm_stream)
                else:
                    work = dist.all_gather_into_tensor(recv, send, async_op=True)
                    work.wait()   # the side stream (not the host) waits for the collective
                if self.restack_timing:
                    c1 = torch.cuda.Event(enable_timing=True)
                    c1.record(self.comm_stream)
                    self._comm_ev.append((c0, c1))
                done_ev = self.comm_stream.record_event()
            if stacks is not None:
                # in step order on its own stream (the receive ring carries state from step to step)
                with torch.cuda.stream(self.restack_stream):
                    self.restack_stream.wait_event(done_ev)
                    if self.restack_timing:
                        t0 = torch.cuda.Event(enable_timing=True)
                        t0.record(self.restack_stream)
                    stacks = self.restacker(recv, stacks, step, all_fresh) or stacks
                    if self.restack_timing:
                        t1 = torch.cuda.Event(enable_timing=True)
                        t1.record(self.restack_stream)
                        self._restack_ev.append((t0, t1))
                    done_ev = self.restacked[b] = self.restack_stream.record_event()
            h = GatheredStep(self.layout, recv, stacks, event=done_ev, owner=self, step=step,
                             windowed=stacks is not None and not getattr(self.restacker, "materialized", True))
        else:
            work = dist.all_gather_into_tensor(recv, send, async_op=True)
            work.wait()
            if stacks is not None:
                stacks = self.restacker(recv, stacks, step, all_fresh) or stacks
            h = GatheredStep(self.layout, recv, stacks, owner=self, step=step,
                             windowed=stacks is not None and not getattr(self.restacker, "materialized", True))
        self.pending[b] = h
        self.t += 1
        return h

    def reset_async(self):
        b = self._begin()
        self.vec.reset()
        self._ring_resets = getattr(self.vec, "reset_count", None)
        self._finish_outputs(b)
        return self._launch(b, all_fresh=True)

    def step_async(self, actions):
        if self.layout.frames_only:   # never restack from an unfilled or stale ring
            if self._ring_resets is None and self.t == 0:
                raise RuntimeError("ShardedVecEnv(gather_mode='frames'): call reset() / reset_async() before the "
                                   "first step (the receivers' frame rings are filled by it)")
            if getattr(self.vec, "reset_count", None) != self._ring_resets:
                raise RuntimeError("ShardedVecEnv(gather_mode='frames'): the VecMagicalEnv was reset directly; "
                                   "reset through reset() / reset_async() so every rank's frame ring restarts")
        b = self._begin()
        self.vec.step(actions)
        self._finish_outputs(b)
        return self._launch(b, all_fresh=False)

    # -- gym-style ------------------------------------------------------------------------------------------
    def reset(self):
        if self.gather:
            return self.reset_async().results()[0]
        return self.vec.reset()

    def step(self, actions):
        if self.gather:
            return self.step_async(actions).results()
        return self.vec.step(actions)

    def wait_all(self):
        for h in getattr(self, "pending", []):
            if h is not None:
                h.wait()

    def close(self):
        self.wait_all()
        self.vec.close()
