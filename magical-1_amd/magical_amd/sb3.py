"""Stable-Baselines3 VecEnv surface over the GPU simulator.

The reference trains with `DummyVecEnv([lambda: Monitor(gym.make(name, ...)) for _ in range(32)])`
(train_rl.py:87-92) and `DummyVecEnv([lambda: gym.make('MoveToCorner-Demo-LoRes4E-v0')])`
(train_il.py:216-217).  `MagicalVecEnv(name, n)` is a drop-in for that stack with the N envs on
one GPU:

* `reset()` / `step_async(actions)` / `step_wait()` / `step(actions)` with SB3's conventions:
  observations as an OrderedDict of numpy arrays `[N, ...]` (or device tensors with
  `as_tensors=True`), rewards `float32[N]`, dones `bool[N]`, a list of info dicts;
* finished episodes are reset in place and the returned observation is the first one of the next
  episode; the last observation of the finished one is `info['terminal_observation']`
  (DummyVecEnv), `info['TimeLimit.truncated']` is False (BaseEnv itself ends the episode at the
  step TimeLimit would, benchmarks/__init__.py:232-266), and with `monitor=True`
  `info['episode'] = {'r', 'l', 't'}` as SB3's Monitor records it;
* every info carries `eval_score` (base_env.py:299-303).

When stable_baselines3 is importable the class derives from its VecEnv base, so isinstance checks
and VecEnv wrappers accept it; otherwise it is a duck-typed stand-in with the same methods.
"""
import collections
import time

import numpy as np
import torch

from .envs import VecMagicalEnv

try:  # pragma: no cover - SB3 is not installed in this image
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except Exception:  # SB3 absent: plain object base
    _VecEnvBase = object


class MagicalVecEnv(_VecEnvBase):
    metadata = {"render.modes": ["rgb_array"]}

    def __init__(self, env_name, num_envs, device="cuda:0", seeds=None, base_seed=0, monitor=True,
                 as_tensors=False, debug_reward=None, max_episode_steps=None):
        self.venv = VecMagicalEnv(env_name, num_envs, device=device, seeds=seeds, base_seed=base_seed,
                                  auto_reset=False, debug_reward=debug_reward, max_episode_steps=max_episode_steps)
        self.num_envs = self.venv.num_envs
        self.observation_space = self.venv.observation_space
        self.action_space = self.venv.action_space
        self.render_mode = "rgb_array"
        self.monitor = monitor
        self.as_tensors = as_tensors
        dev = self.venv.device
        self._ep_return = torch.zeros(self.num_envs, dtype=torch.float64, device=dev)
        self._ep_len = torch.zeros(self.num_envs, dtype=torch.int64, device=dev)
        self._t0 = time.time()
        self._actions = None

    # -- conversion ---------------------------------------------------------------
    def _out(self, obs):
        if self.as_tensors:
            return collections.OrderedDict((k, v.clone()) for k, v in obs.items())
        return collections.OrderedDict((k, v.cpu().numpy()) for k, v in obs.items())

    # -- VecEnv API -----------------------------------------------------------------
    def reset(self):
        self._ep_return.zero_()
        self._ep_len.zero_()
        self._t0 = time.time()
        return self._out(self.venv.reset())

    def step_async(self, actions):
        self._actions = torch.as_tensor(np.asarray(actions) if not isinstance(actions, torch.Tensor) else actions)

    def step_wait(self):
        obs, rew, done, info = self.venv.step(self._actions)
        self._ep_return += rew.to(torch.float64)
        self._ep_len += 1
        scores = info["eval_score"].cpu().numpy()
        dones = done.cpu().numpy().astype(bool)
        rewards = rew.cpu().numpy().astype(np.float32)
        infos = [{"eval_score": float(s)} for s in scores]
        if dones.any():
            idx = np.flatnonzero(dones)
            terminal = self._out(obs)
            ret = self._ep_return.cpu().numpy()
            length = self._ep_len.cpu().numpy()
            now = round(time.time() - self._t0, 6)
            for i in idx:
                infos[i]["terminal_observation"] = collections.OrderedDict((k, v[i]) for k, v in terminal.items())
                infos[i]["TimeLimit.truncated"] = False
                if self.monitor:
                    infos[i]["episode"] = {"r": round(float(ret[i]), 6), "l": int(length[i]), "t": now}
            mask = done.to(torch.uint8)
            self._ep_return.masked_fill_(done, 0.0)
            self._ep_len.masked_fill_(done, 0)
            obs = self.venv.reset(mask)  # first observation of the next episode for the finished envs
        return self._out(obs), rewards, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.venv.close()

    def seed(self, seed=None):
        base = 0 if seed is None else int(seed)
        return self.venv.seed([base + i for i in range(self.num_envs)])

    def get_images(self):
        full = self.venv.render_full().cpu().numpy()
        return [full[i, 0] for i in range(self.num_envs)]

    def render(self, mode="rgb_array"):
        return np.stack(self.get_images())

    def get_attr(self, attr_name, indices=None):
        n = len(self._indices(indices))
        return [getattr(self.venv, attr_name)] * n

    def set_attr(self, attr_name, value, indices=None):
        setattr(self.venv, attr_name, value)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        raise NotImplementedError("the envs live on the GPU as one batch; there are no per-env objects")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)
