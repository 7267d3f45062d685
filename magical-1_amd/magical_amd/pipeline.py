"""Pipelined env pool: one batch of envs as C simulators on C HIP streams.

Why: the robot scenes' step kernel holds a whole CU's LDS per workgroup (16 envs x ~9.8 KB) and runs one
wavefront per CU for ~0.54 ms whatever the env count, and the render kernel fills the CUs with 16 KB
workgroups after it; in one stream the two alternate and neither fills the chip.  Split into C chunks, each
with its own stream, chunk k's render runs beside chunk k+1's step kernel and the next step of chunk 0
starts as soon as chunk 0's own render is done (round 4, `tools/overlap_ab.py`: MoveToRegion 4096 envs
2.54 M -> 2.79 M env-steps/s at C = 2, MoveToCorner 1.94 -> 2.08 M; the cooperative many-block scenes are
slower chunked, ClusterColour 1.48 -> 1.23 M, and keep C = 1).

Semantics: every env is exactly the env of the unchunked `VecMagicalEnv` with the same seed (env i of the
pool is env i mod m of chunk i // m, seeded as global env i), stepped with its own action in the same order,
so observations are bit-identical (`tests/test_gpu_parity.py::test_pipelined_pool_matches_batch`).  Chunks
are equal shares of the envs rounded to the step kernel's 16-env workgroups; at most 3, since a process has
4 hardware queues (GPU_MAX_HW_QUEUES) and the caller's stream takes one.  What
changes is completion: `step()` only enqueues; a chunk's outputs (views into the pool's full-batch tensors)
are complete once `wait(k)` / `wait()` has ordered the caller's stream after it -- the asynchronous env-pool
contract (as EnvPool's async mode), not gym's synchronous one.  Actions are double-buffered on the device,
so the caller may overwrite its action tensor right after `step()` returns.
"""
import collections
import ctypes

import torch

from . import native
from .envs import VecMagicalEnv


# tasks measured faster pipelined (round 4): their scenes run the compile-time robot forms of the step
# kernel (16 envs per workgroup: one workgroup per CU at 4096 envs, the CU's whole LDS)
PIPELINED_TASKS = ("MoveToRegion", "MoveToCorner")


def default_chunks(spec, num_envs):
    """bench.py --chunks auto: 3 for MoveToRegion at >= 4096 envs, 2 for the robot scenes at >= 2048, else 1.
    (Round 6, with the 16-row-band render: a third chunk measured MoveToRegion 3.37 -> 3.42 M env-steps/s at 4096
    envs, two repetitions (profiles/r06_b16/chunks_b16), its render-bound pipeline gaining from the smaller step
    launches; MoveToCorner, whose pipeline is step-bound, 2.59 -> 2.61 M, within noise, and its 0.74 ms step kernel
    then serves 1365 envs instead of 2048 -- kept at 2.  Before the 16-row render, MoveToRegion's third chunk was
    3.16 -> 3.19 M (profiles/r06_d).  A 1365-env chunk's render fills 1.2 rounds of the CUs' workgroup slots, so its
    isolated HBM fraction reads lower than a 2048-env chunk's.)"""
    if spec.task not in PIPELINED_TASKS:
        return 1
    if spec.task == "MoveToRegion" and num_envs >= 4096:
        return 3
    return 2 if num_envs >= 2048 and num_envs % 2 == 0 else 1


class PipelinedVecEnv:
    def __init__(self, env_name, num_envs, chunks=2, device="cuda:0", seeds=None, base_seed=0, **kw):
        num_envs, chunks = int(num_envs), int(chunks)
        if chunks < 1 or chunks > min(num_envs, 3):
            raise ValueError(f"PipelinedVecEnv: {num_envs} envs do not split into {chunks} chunks")
        self.num_envs, self.chunks = num_envs, chunks
        # chunk bounds: equal shares rounded to the step kernel's 16-env workgroups where the count allows
        q = 16 if num_envs >= 16 * chunks else 1
        units = num_envs // q
        self.bounds = [q * (units * k // chunks) for k in range(chunks)] + [num_envs]
        self.device = torch.device(device)
        seeds = list(seeds) if seeds is not None else [base_seed + i for i in range(num_envs)]
        if len(seeds) != num_envs:
            raise ValueError("PipelinedVecEnv: one seed per env")
        b = self.bounds
        self.sims = [VecMagicalEnv(env_name, b[k + 1] - b[k], device=device, seeds=seeds[b[k]:b[k + 1]], **kw)
                     for k in range(chunks)]
        s0 = self.sims[0]
        self.spec, self.lib, self.max_episode_steps = s0.spec, s0.lib, s0.max_episode_steps
        self.action_space, self.observation_space = s0.action_space, s0.observation_space
        if self.spec.preproc is None:
            raise ValueError("PipelinedVecEnv: LoRes preprocessors only (the 384^2 view is rendered on demand)")
        # the pool's full-batch outputs; chunk k writes rows [bounds[k], bounds[k + 1]) on its own stream
        # (PickAndPlace's target included: the auto-reset rewrites it inside the chunk's step, so it is complete
        # only after wait(), like the observations -- ADVICE r4)
        self.buffers = collections.OrderedDict(
            (k, torch.zeros((num_envs,) + tuple(v.shape[1:]), dtype=v.dtype, device=self.device))
            for k, v in s0.output_buffers().items())
        # window rings of the stacked views (VecMagicalEnv window mode): one ring per view for the whole pool,
        # chunk k's envs a contiguous slice of it (env-major), so the pool's stacks are one strided view
        self.window_k = s0.window_k
        self.wring = [None if r is None else torch.zeros((num_envs,) + tuple(r.shape[1:]), dtype=r.dtype, device=self.device)
                      for r in s0.wring]
        for k, sim in enumerate(self.sims):
            views = {key: buf[b[k]:b[k + 1]] for key, buf in self.buffers.items()}
            if self.window_k:
                sim.bind_window(*[None if r is None else r[b[k]:b[k + 1]] for r in self.wring])
            sim.bind_outputs(views, target=views.get("target"))
        # (a high-priority stream for chunk 0 measured no different, round 4: profiles/r04_resetwaves/)
        self.streams = [torch.cuda.Stream(self.device) for _ in range(chunks)]
        self.abuf = torch.zeros((2, num_envs), dtype=torch.uint8, device=self.device)
        # done[k][slot]: chunk k finished the step that read action slot `slot`
        self.done_ev = [[None, None] for _ in range(chunks)]
        self.t = 0
        self.reset_count = 0      # explicit reset() calls (magical_amd.dist checks its frame rings against it)
        self.target = self.buffers.get("target")
        # the observation's float32 target columns, converted on each chunk's stream right after its step (a
        # conversion on the caller's stream inside step() would read the target before the chunk wrote it)
        self.target_f = None if self.target is None else torch.zeros(self.target.shape, dtype=torch.float32,
                                                                     device=self.device)
        self._target_out = None   # bind_outputs' "target" view (magical_amd.dist's packed buffer)
        self._last = []           # the chunk streams' events of the last step() (magical_amd.dist waits on them)

    # -- ordering ------------------------------------------------------------------
    def _caller(self):
        return torch.cuda.current_stream(self.device)

    def _fork(self):
        """The chunk streams wait for the caller's work so far."""
        ev = torch.cuda.Event()
        ev.record(self._caller())
        for st in self.streams:
            st.wait_event(ev)

    def wait(self, chunk=None):
        """Order the caller's stream after chunk `chunk` (all chunks when None): its outputs are then complete."""
        cs = self._caller()
        for k in (range(self.chunks) if chunk is None else [chunk]):
            ev = torch.cuda.Event()
            ev.record(self.streams[k])
            cs.wait_event(ev)

    def step_events(self):
        """Events recorded on every chunk's stream after its last step() (a consumer on another stream, e.g.
        magical_amd.dist's collective, waits on them instead of ordering the caller's stream after the chunks,
        which would make the next step's chunks wait for each other)."""
        return list(self._last)

    def bind_outputs(self, views, frames_only=False):
        """Bind full-batch [num_envs, ...] output views (VecMagicalEnv.bind_outputs keys): chunk k writes rows
        [bounds[k], bounds[k + 1]) of each.  Called between steps (magical_amd.dist binds a packed buffer set per
        step); the chunks' streams are ordered after the caller's stream by the next step()'s fork."""
        b = self.bounds
        for k, sim in enumerate(self.sims):
            sim.bind_outputs({key: v[b[k]:b[k + 1]] for key, v in views.items() if key != "target"},
                             frames_only=frames_only)
        # PickAndPlace: the pool's persistent target is copied into views["target"] on each chunk's stream right
        # after the chunk's step (reset: on the caller's stream), so the view is complete when the chunk is
        self._target_out = views.get("target") if self.target is not None else None

    # -- API -----------------------------------------------------------------------
    def reset(self, mask=None):
        self.wait()
        for k, sim in enumerate(self.sims):
            sim.reset(None if mask is None else mask[self.bounds[k]:self.bounds[k + 1]])
        if self.target_f is not None:   # the resets ran on the caller's stream
            self.target_f.copy_(self.target)
            if self._target_out is not None:
                self._target_out.copy_(self.target)
        self.reset_count += 1
        self._last = []
        self._fork()
        return self._obs()

    def step(self, actions):
        a = actions
        if not (isinstance(a, torch.Tensor) and a.dtype == torch.uint8 and a.device == self.device):
            a = torch.as_tensor(actions).to(self.device, torch.uint8)
        slot = self.t & 1
        cs = self._caller()
        for k in range(self.chunks):   # the step two calls ago has read this slot
            if self.done_ev[k][slot] is not None:
                cs.wait_event(self.done_ev[k][slot])
        self.abuf[slot].copy_(a)
        self._fork()
        b = self.bounds
        for k, (sim, st) in enumerate(zip(self.sims, self.streams)):
            with torch.cuda.stream(st):
                sim.step(self.abuf[slot, b[k]:b[k + 1]])
                if self.target_f is not None:
                    self.target_f[b[k]:b[k + 1]].copy_(self.target[b[k]:b[k + 1]])
                    if self._target_out is not None:
                        self._target_out[b[k]:b[k + 1]].copy_(self.target[b[k]:b[k + 1]])
            ev = torch.cuda.Event()
            ev.record(st)
            self.done_ev[k][slot] = ev
        self._last = [self.done_ev[k][slot] for k in range(self.chunks)]
        self.t += 1
        return self._obs(), self.buffers["reward"], self.buffers["done"], {"eval_score": self.buffers["eval_score"]}

    def _obs(self):
        from .envs import window_stack
        allo, ego, past = self.buffers.get("allo"), self.buffers.get("ego"), self.buffers.get("past_obs")
        if self.window_k:   # every chunk has stepped as often: one window start for the whole pool
            s0, K = self.sims[0].window_start(), self.window_k
            if self.spec.preproc == "LoResStack":
                allo, ego = window_stack(self.wring[0], s0, K), window_stack(self.wring[1], s0, K)
            else:
                past = window_stack(self.wring[0] if self.wring[0] is not None else self.wring[1], s0, K)
        out = collections.OrderedDict([("allo", allo), ("ego", ego)])
        if self.sims[0]._chw:
            out = collections.OrderedDict((k, v.permute(0, 3, 1, 2)) for k, v in out.items())
        if self.target_f is not None:
            t = self.target_f
            out["target_type"], out["target_colour"], out["target_position"] = t[:, 0:1], t[:, 1:2], t[:, 2:4]
        if past is not None:
            out["past_obs"] = past.permute(0, 3, 1, 2) if self.sims[0]._chw else past
        return out

    def random_actions(self, step, key=42, out=None):
        """Device Philox actions for a random policy (chunk k draws with key + k)."""
        out = out if out is not None else torch.empty(self.num_envs, dtype=torch.uint8, device=self.device)
        b = self.bounds
        for k, sim in enumerate(self.sims):
            sim.random_actions(step, key=key + k, out=out[b[k]:b[k + 1]])
        return out

    def set_episode_steps(self, steps):
        self.wait()
        s = torch.as_tensor(steps)
        for k, sim in enumerate(self.sims):
            sim.set_episode_steps(s[self.bounds[k]:self.bounds[k + 1]])
        self._fork()

    def errors(self):
        self.wait()
        return torch.cat([sim.errors() for sim in self.sims])

    def enable_timing(self, steps):
        """Per-chunk HIP-event timing of the kernels (mg_enable_timing on every chunk's simulator)."""
        self.wait()
        for sim in self.sims:
            native.check(self.lib.mg_enable_timing(sim.handle, int(steps)))

    def read_timing(self):
        """[chunks][4] totals over the timed launches (mg_read_timing: step ms, render ms, launches, reset ms)."""
        out = []
        for sim in self.sims:
            tm = (ctypes.c_double * 4)()
            native.check(self.lib.mg_read_timing(sim.handle, tm))
            out.append(list(tm))
        return out

    def close(self):
        for st in self.streams:   # the chunks' queued kernels read the simulators' memory
            st.synchronize()
        for sim in self.sims:
            sim.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
