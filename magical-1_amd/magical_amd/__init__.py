"""magical_amd: MI355X-native batched MAGICAL simulator (drop-in for the
physics + 384^2 render + LoRes preprocessing hot path of khanhptnk/magical-1).

    import magical_amd as magical
    magical.register_envs()                    # gym registration when gym is importable
    env = magical.make('MoveToRegion-Demo-LoRes4E-v0')          # single env, numpy obs
    vec = magical.make_vec('MoveToRegion-Demo-LoRes4E-v0', 4096)  # N envs on one GPU

The compute path is the HIP library libmagical_sim.so (C ABI in
include/magical_sim.h); importing this package does not require gym.
"""
from .registry import (ALL_REGISTERED_ENVS, AVAILABLE_PREPROCESSORS, DEMO_ENVS_TO_TEST_ENVS_MAP, EnvName,  # noqa: F401
                       EnvSpec, lookup, update_magical_env_name)

__all__ = ["ALL_REGISTERED_ENVS", "AVAILABLE_PREPROCESSORS", "DEMO_ENVS_TO_TEST_ENVS_MAP", "EnvName",
           "update_magical_env_name", "register_envs", "make", "make_vec"]

_REGISTERED = False


def make(env_name, device="cuda:0", seed=None, debug_reward=None):
    """gym.make(env_name[, debug_reward=...]) equivalent: one instance, reference single-env API."""
    from .envs import MagicalEnv
    return MagicalEnv(env_name, device=device, seed=seed, debug_reward=debug_reward)


def make_vec(env_name, num_envs, device="cuda:0", seeds=None, base_seed=0, auto_reset=True, max_episode_steps=None,
             debug_reward=None, window=False):
    """num_envs instances of env_name on one GPU (batched, auto-resetting).  max_episode_steps
    overrides the registered episode length (gym.make(..., max_episode_steps=...)).  window: frame stacks as
    strided views of window rings (True) or materialised [N, 96, 96, 12] tensors (False, the default)."""
    from .envs import VecMagicalEnv
    return VecMagicalEnv(env_name, num_envs, device=device, seeds=seeds, base_seed=base_seed, auto_reset=auto_reset,
                         max_episode_steps=max_episode_steps, debug_reward=debug_reward, window=window)


def register_envs():
    """benchmarks/__init__.py:427: register every name with gym if gym is importable.
    Returns False if already registered (as the reference does)."""
    global _REGISTERED
    if _REGISTERED:
        return False
    _REGISTERED = True
    try:
        import gym
    except Exception:
        return True
    for name in ALL_REGISTERED_ENVS:
        spec = lookup(name)
        gym.register(name, entry_point="magical_amd:make", max_episode_steps=spec.max_episode_steps,
                     kwargs={"env_name": name})
    return True
