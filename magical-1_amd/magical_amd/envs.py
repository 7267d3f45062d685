"""Gym-style surfaces over the GPU simulator.

* VecMagicalEnv -- N instances of one registered name on one GPU (batched
  counterpart of gym.make(name) under SB3's DummyVecEnv, train_rl.py:87-92):
  reset() -> dict of uint8 device tensors, step(actions) -> (obs, reward f32,
  done bool, {'eval_score': f64}); finished episodes auto-reset in place.
* MagicalEnv -- one instance with the single-env gym API of
  BaseEnv + preprocessors (base_env.py:190-351, benchmarks/__init__.py:51-190):
  numpy observations, done at max_episode_steps, explicit reset().

Every tensor VecMagicalEnv.reset()/step() returns (observations, reward, done,
info values) is one of the simulator's bound output buffers: it is valid until
the next reset()/step() rewrites it (clone it to keep it).  The frame stacks
(LoRes4E / LoRes4A / CHW past_obs, LoResStack allo / ego) are contiguous [N, 96, 96,
12] tensors; window=True makes them strided views of per-view window rings on the
device instead (mg_bind_window: each frame written once, channel-planar; the stack =
4 consecutive slots; the same values, shape and dtype, channel stride 96 * 96) --
measured 4-7% slower in the render kernel than the materialised stacks, whose
writes hide under the kernel's latency.
"""
import collections
import ctypes

import numpy as np
import torch

from . import native, registry, spaces, tables

_LIBRARY = None


def library():
    global _LIBRARY
    if _LIBRARY is None:
        _LIBRARY = tables.build_library()
    return _LIBRARY


def _obs_shapes(spec):
    pp = spec.preproc
    if pp is None:
        return collections.OrderedDict([("allo", (384, 384, 3)), ("ego", (384, 384, 3))])
    if pp == "LoResStack":
        return collections.OrderedDict([("allo", (96, 96, 12)), ("ego", (96, 96, 12))])
    cf = registry.PREPROCESSORS[pp]["channels_first"]
    shapes = collections.OrderedDict([("allo", (96, 96, 3)), ("ego", (96, 96, 3)), ("past_obs", (96, 96, 12))])
    if cf:
        shapes = collections.OrderedDict((k, (s[2], s[0], s[1])) for k, s in shapes.items())
    return shapes


# PickAndPlace observation extras (pick_and_place.py:23-28), inserted after allo/ego by the base env
# and therefore before the frame stack's past_obs (benchmarks/__init__.py:124-147)
TARGET_KEYS = ("target_type", "target_colour", "target_position")


WINDOW_K = 8   # window ring period: K + 3 slots per env and stacked view (magical_amd.dist uses the same)


def window_views(spec):
    """(allo, ego): which views of a preprocessor are frame stacks a window ring can hold (LoRes3EA's stack is
    allo + 3 ego frames: not one ring's window)."""
    pp = spec.preproc
    return (pp in ("LoResStack", "LoRes4A"), pp in ("LoResStack", "LoRes4E", "LoResCHW4E", "LoResCHW4A"))


def window_stack(ring, s0, K=WINDOW_K):
    """[n, 96, 96, 12] stack view of a window ring u8[n, K + 3, 3, 96, 96] at first slot s0 (include/magical_sim.h
    mg_bind_window): channel c = plane c % 3 of slot s0 + c // 3."""
    fr = 96 * 96 * 3
    return ring.as_strided((ring.shape[0], 96, 96, 12), ((K + 3) * fr, 96, 1, 96 * 96), ring.storage_offset() + s0 * fr)


def observation_space(spec):
    items = [(k, spaces.Box(low=0, high=255, shape=s, dtype=np.uint8)) for k, s in _obs_shapes(spec).items()]
    if spec.task == "PickAndPlace":
        extra = [("target_type", spaces.Box(low=0, high=4, shape=(1,), dtype=np.float32)),
                 ("target_colour", spaces.Box(low=0, high=4, shape=(1,), dtype=np.float32)),
                 ("target_position", spaces.Box(low=-1, high=1, shape=(2,), dtype=np.float32))]
        items = items[:2] + extra + items[2:]
    return spaces.Dict(collections.OrderedDict(items))


class VecMagicalEnv:
    """Batched MAGICAL env on one MI355X (C ABI: include/magical_sim.h)."""

    def __init__(self, env_name, num_envs, device="cuda:0", seeds=None, base_seed=0, auto_reset=True,
                 max_episode_steps=None, debug_reward=None, window=False):
        self.spec = registry.lookup(env_name)
        if not self.spec.gpu_supported:
            raise NotImplementedError(f"{env_name}: task not on the GPU hot path yet")
        pp = self.spec.preproc
        if self.spec.task == "PickAndPlace" and pp == "LoResStack":
            # EagerDictFrameStack concatenates every observation value along the last axis; the
            # scalar target_type / target_colour make that raise in the reference as well
            raise ValueError(f"{env_name}: the reference cannot frame-stack PickAndPlace's scalar observations")
        flags = self.spec.rand_flags
        if debug_reward is not None:  # gym.make(name, debug_reward=...)
            flags = (flags | registry.DEBUG_REWARD) if debug_reward else (flags & ~registry.DEBUG_REWARD)
        self.debug_reward = bool(flags & registry.DEBUG_REWARD)
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        self.lib = native.load()
        self._chw = pp is not None and registry.PREPROCESSORS[pp].get("channels_first", False)
        gpu_pp = {None: 0, "LoRes4E": 1, "LoResStack": 2, "LoRes3EA": 3, "LoRes4A": 4, "LoResCHW4E": 1, "LoResCHW4A": 1}[pp]
        cfg = native.mg_config()
        cfg.task = self.spec.task_id
        cfg.rand_flags = flags
        cfg.preproc = gpu_pp
        cfg.num_envs = self.num_envs
        cfg.device = self.device.index or 0
        self.max_episode_steps = int(max_episode_steps or self.spec.max_episode_steps)
        cfg.max_episode_steps = self.max_episode_steps
        cfg.base_seed = base_seed
        cfg.auto_reset = 1 if auto_reset else 0
        if seeds is not None:
            self._seeds = (ctypes.c_uint32 * self.num_envs)(*[int(s) & 0xffffffff for s in seeds])
            cfg.seeds = self._seeds
        lib_struct = library()
        cfg.library = ctypes.cast(ctypes.pointer(lib_struct), ctypes.c_void_p)
        cfg.library_size = ctypes.sizeof(tables.mg_library)
        torch.cuda.init()
        handle = ctypes.c_void_p()
        native.check(self.lib.mg_create(ctypes.byref(cfg), ctypes.byref(handle)))
        self.handle = handle
        n, dev = self.num_envs, self.device
        u8 = dict(dtype=torch.uint8, device=dev)
        wa, we = window_views(self.spec) if window and pp is not None else (False, False)
        self.window_k = WINDOW_K if (wa or we) else 0
        self.wring = [None, None]
        if self.window_k:
            shape = (n, self.window_k + 3, 3, 96, 96)
            self.wring = [torch.zeros(shape, **u8) if wa else None, torch.zeros(shape, **u8) if we else None]
        if pp is None:
            self.full = torch.empty((n, 2, 384, 384, 3), **u8)
            self.obs_allo = self.obs_ego = self.obs_past = None
        elif pp == "LoResStack":
            self.obs_allo = None if wa else torch.empty((n, 96, 96, 12), **u8)
            self.obs_ego = None if we else torch.empty((n, 96, 96, 12), **u8)
            self.obs_past = None
        else:
            self.obs_allo = torch.empty((n, 96, 96, 3), **u8)
            self.obs_ego = torch.empty((n, 96, 96, 3), **u8)
            self.obs_past = None if self.window_k else torch.empty((n, 96, 96, 12), **u8)
        self.reward = torch.zeros(n, dtype=torch.float32, device=dev)
        self.done = torch.zeros(n, dtype=torch.bool, device=dev)  # the C ABI writes u8 0/1: same bytes
        self.eval_score = torch.zeros(n, dtype=torch.float64, device=dev)
        self.target = torch.zeros((n, 4), dtype=torch.float64, device=dev) if self.spec.task == "PickAndPlace" else None
        self.frames_only = False
        self.reset_count = 0   # explicit reset() calls (magical_amd.dist checks its frame rings against it)
        if self.window_k:
            self._bind_window()
        self._bind()
        self.action_space = spaces.Discrete(18)
        self.observation_space = observation_space(self.spec)

    # -- helpers -----------------------------------------------------------
    def _bind(self):
        buf = native.mg_buffers()
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        buf.obs_allo, buf.obs_ego, buf.obs_past = ptr(self.obs_allo), ptr(self.obs_ego), ptr(self.obs_past)
        buf.reward, buf.done, buf.eval_score = ptr(self.reward), ptr(self.done), ptr(self.eval_score)
        buf.target = ptr(self.target)
        buf.frames_only = 1 if self.frames_only else 0
        native.check(self.lib.mg_bind_outputs(self.handle, ctypes.byref(buf)))

    def _bind_window(self):
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        native.check(self.lib.mg_bind_window(self.handle, ptr(self.wring[0]), ptr(self.wring[1]), self.window_k))

    def bind_window(self, ring_allo, ring_ego):
        """Use caller-owned window rings u8[n, K + 3, 3, 96, 96] (e.g. slices of a pool's rings: every env of a
        magical_amd.pipeline pool in one ring) instead of this env's own; before the next reset()."""
        if not self.window_k:
            raise ValueError("bind_window: this env materialises its stacks (window=False or no stacked view)")
        self.wring = [ring_allo if self.wring[0] is not None else None, ring_ego if self.wring[1] is not None else None]
        self._bind_window()

    def window_start(self):
        """First slot of the current outputs' window (mg_window_start)."""
        s0 = ctypes.c_int32()
        native.check(self.lib.mg_window_start(self.handle, ctypes.byref(s0)))
        return s0.value

    def bind_outputs(self, views, frames_only=False, target=None):
        """Write the following steps' outputs into caller-owned device tensors (e.g. views into one packed
        buffer per step, magical_amd.dist.PackedLayout): keys as output_buffers().  frames_only: 'allo' /
        'ego' receive only the current [n, 96, 96, 3] frames for every LoRes preprocessor (no stacks;
        magical_amd.dist's compact gather restacks on the receivers) -- changing the mode needs a reset.
        PickAndPlace's target (written only at reset) stays in the env's own persistent buffer (views["target"]
        is ignored: a per-step packed buffer would hold a stale one), unless `target` names a persistent [n, 4]
        f64 tensor to use instead -- bind it before the reset that fills it (magical_amd.pipeline)."""
        if self.spec.preproc is None:
            raise ValueError("bind_outputs: the unwrapped 384^2 view is rendered on demand, not bound")
        self.obs_allo, self.obs_ego = views.get("allo"), views.get("ego")   # (window-ring stacks: not bound)
        self.obs_past = None if frames_only else views.get("past_obs")
        self.reward, self.done, self.eval_score = views["reward"], views["done"], views["eval_score"]
        if self.target is not None and target is not None:
            self.target = target
        self.frames_only = bool(frames_only)
        self._bind()

    def output_buffers(self):
        """The currently bound output tensors: raw (HWC) observation buffers, reward, done, eval_score[, target]."""
        out = collections.OrderedDict((k, v) for k, v in (("allo", self.obs_allo), ("ego", self.obs_ego)) if v is not None)
        if self.obs_past is not None:
            out["past_obs"] = self.obs_past
        out["reward"], out["done"], out["eval_score"] = self.reward, self.done, self.eval_score
        if self.target is not None:
            out["target"] = self.target
        return out

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _obs(self):
        if self.spec.preproc is None:
            out = collections.OrderedDict([("allo", self.full[:, 0]), ("ego", self.full[:, 1])])
            past = None
        else:
            allo, ego, past = self.obs_allo, self.obs_ego, self.obs_past
            if self.window_k and not self.frames_only:
                s0 = self.window_start()
                if self.spec.preproc == "LoResStack":
                    allo, ego = window_stack(self.wring[0], s0, self.window_k), window_stack(self.wring[1], s0, self.window_k)
                else:
                    past = window_stack(self.wring[0] if self.wring[0] is not None else self.wring[1], s0, self.window_k)
            out = collections.OrderedDict([("allo", allo), ("ego", ego)])
            if self._chw:
                out = collections.OrderedDict((k, v.permute(0, 3, 1, 2)) for k, v in out.items())
        if self.target is not None:  # as SB3's DummyVecEnv buffers them: float32 per the spaces
            t = self.target.to(torch.float32)
            out["target_type"], out["target_colour"], out["target_position"] = t[:, 0:1], t[:, 1:2], t[:, 2:4]
        if past is not None:
            out["past_obs"] = past.permute(0, 3, 1, 2) if self._chw else past
        return out

    # -- API -----------------------------------------------------------------
    def seed(self, seeds):
        arr = (ctypes.c_uint32 * self.num_envs)(*[int(s) & 0xffffffff for s in seeds])
        native.check(self.lib.mg_seed(self.handle, arr))
        return list(seeds)

    def reset(self, mask=None):
        m = None if mask is None else ctypes.c_void_p(mask.to(self.device, torch.uint8).contiguous().data_ptr())
        native.check(self.lib.mg_reset(self.handle, m, self._stream()))
        self.reset_count += 1
        if self.spec.preproc is None:
            self.render_full(out=self.full)
        return self._obs()

    def step(self, actions):
        a = actions
        if not (isinstance(a, torch.Tensor) and a.dtype == torch.uint8 and a.device == self.device and a.is_contiguous()):
            a = torch.as_tensor(actions).to(self.device, torch.uint8).contiguous()
        self._last_actions = a
        native.check(self.lib.mg_step(self.handle, ctypes.c_void_p(a.data_ptr()), self._stream()))
        if self.spec.preproc is None:
            self.render_full(out=self.full)
        return self._obs(), self.reward, self.done, {"eval_score": self.eval_score}

    def random_actions(self, step, key=42, out=None):
        out = out if out is not None else torch.empty(self.num_envs, dtype=torch.uint8, device=self.device)
        native.check(self.lib.mg_random_actions(self.handle, ctypes.c_void_p(out.data_ptr()), key, step, self._stream()))
        return out

    def set_episode_steps(self, steps):
        """Overwrite every env's episode step counter (throughput runs stagger episode phases)."""
        s = torch.as_tensor(steps).to(self.device, torch.int32).contiguous()
        native.check(self.lib.mg_set_episode_steps(self.handle, ctypes.c_void_p(s.data_ptr()), self._stream()))
        torch.cuda.current_stream(self.device).synchronize()

    def render_full(self, out=None):
        out = out if out is not None else torch.empty((self.num_envs, 2, 384, 384, 3), dtype=torch.uint8,
                                                      device=self.device)
        native.check(self.lib.mg_render_full(self.handle, ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def bodies(self):
        out = torch.empty((self.num_envs, 16, 6), dtype=torch.float64, device=self.device)
        counts = torch.empty((self.num_envs, 4), dtype=torch.int32, device=self.device)
        native.check(self.lib.mg_get_bodies(self.handle, ctypes.c_void_p(out.data_ptr()),
                                            ctypes.c_void_p(counts.data_ptr()), self._stream()))
        return out, counts

    def step_form(self):
        """(form, envs per workgroup, (bodies, shapes, constraints, arbiter slots) caps) of the step kernel
        (mg_step_form)"""
        out = (ctypes.c_int32 * 6)()
        native.check(self.lib.mg_step_form(self.handle, out))
        return int(out[0]), int(out[1]), tuple(int(x) for x in out[2:6])

    def arbiters(self):
        """solved arbiters per env in active order: f64 [N, 48, 28] and contact hashes u64 [N, 48, 2]
        (mg_get_arbiters; the active count is bodies()[1][:, 3])"""
        out = torch.empty((self.num_envs, 48, 28), dtype=torch.float64, device=self.device)
        hs = torch.empty((self.num_envs, 48, 2), dtype=torch.uint64, device=self.device)
        native.check(self.lib.mg_get_arbiters(self.handle, ctypes.c_void_p(out.data_ptr()),
                                              ctypes.c_void_p(hs.data_ptr()), self._stream()))
        return out, hs

    def set_body_pose(self, env, body, x, y, angle):
        """Place body `body` of env `env` (Body.position / Body.angle setters; parity tests)."""
        native.check(self.lib.mg_set_body_pose(self.handle, int(env), int(body), float(x), float(y), float(angle),
                                               self._stream()))

    def errors(self):
        out = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
        native.check(self.lib.mg_get_errors(self.handle, ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self.lib.mg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PlacementError(Exception):
    """geom.py:111: raised by reset() when the layout randomiser gives up (after 10 retries)."""


class MagicalEnv:
    """Single instance with the reference's gym.Env surface (numpy observations)."""

    metadata = {"render.modes": ["rgb_array"]}

    def __init__(self, env_name, device="cuda:0", seed=None, debug_reward=None):
        self.spec = registry.lookup(env_name)
        self._vec = VecMagicalEnv(env_name, 1, device=device, auto_reset=False, debug_reward=debug_reward)
        self.max_episode_steps = self.spec.max_episode_steps
        self.action_space = spaces.Discrete(18)
        self.observation_space = observation_space(self.spec)
        self._episode_steps = None
        self.seed(seed)

    def seed(self, seed=None):
        """base_env.py:134-141: RandomState(seed); None draws from the global numpy RNG."""
        if seed is None:
            seed = np.random.randint(0, (1 << 31) - 1)
        self._vec.seed([seed])
        return [seed]

    def action_to_flags(self, int_action):
        return ACTION_ID_TO_FLAGS[int(int_action)]

    def flags_to_action(self, flags):
        return FLAGS_TO_ACTION_ID[tuple(flags)]

    def _np_obs(self, obs):
        out = collections.OrderedDict()
        for k, v in obs.items():
            if k in TARGET_KEYS:  # pick_and_place.py:103-107: python ints and a float64 array
                t = self._vec.target[0].cpu().numpy()
                out[k] = int(t[0]) if k == "target_type" else int(t[1]) if k == "target_colour" else t[2:4].copy()
            else:
                out[k] = v[0].cpu().numpy()
        return out

    def reset(self):
        self._episode_steps = 0
        obs = self._np_obs(self._vec.reset())
        if int(self._vec.errors()[0].item()) & 2:  # pm_randomise_all_poses raised (geom.py:335-336)
            raise PlacementError("could not place entities after 10 layout retries (geom.py:295-341)")
        return obs

    def step(self, action):
        if self._episode_steps is None:
            raise RuntimeError("call reset() before step()")
        obs, rew, done, info = self._vec.step(torch.tensor([int(action)], dtype=torch.uint8))
        self._episode_steps += 1
        d = bool(done[0].item())
        score = float(info["eval_score"][0].item())
        return self._np_obs(obs), float(rew[0].item()), d, {"eval_score": score}

    def render(self, mode="rgb_array"):
        if mode != "rgb_array":
            raise NotImplementedError("headless: only rgb_array")
        full = self._vec.render_full()[0].cpu().numpy()
        return collections.OrderedDict([("allo", full[0]), ("ego", full[1])])

    def close(self):
        self._vec.close()


# entities.py:148-190
_UD = [0, 1, 2]            # NONE, UP, DOWN
_LR = [0, 4, 8]            # NONE, LEFT, RIGHT
ACTION_NUMS_FLAGS_NAMES = []
for _aid in range(18):
    _grip = 16 if _aid < 9 else 32
    _ud, _lr = _UD[_aid % 3], _LR[(_aid // 3) % 3]
    _names = {0: "", 1: "Up", 2: "Down"}[_ud] + {0: "", 4: "Left", 8: "Right"}[_lr] + ("Open" if _grip == 16 else "Close")
    ACTION_NUMS_FLAGS_NAMES.append((_aid, (_ud, _lr, _grip), _names))
ACTION_ID_TO_FLAGS = {a: f for a, f, _ in ACTION_NUMS_FLAGS_NAMES}
FLAGS_TO_ACTION_ID = {f: a for a, f, _ in ACTION_NUMS_FLAGS_NAMES}
