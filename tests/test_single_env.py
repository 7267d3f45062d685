"""The single-env drop-in surface (magical_amd.make -> MagicalEnv), on the GPU.

Port of the reference's only test, tests/test_rollout_preproc.py:17-36: env.seed(7),
env.action_space.seed(42), 2 episodes of action_space.sample() actions, each exactly
max_episode_steps long.  Run on the BASELINE names and one name per task x
preprocessor; in addition the reset and first steps' observations, rewards and
eval_scores are compared with the CPU oracle driven by the same actions, and
render('rgb_array') must return OrderedDict(allo, ego) of 384^2 frames equal to
the oracle's.
"""
import collections

import numpy as np
import pytest

import pyoracle as po
import magical_amd
from magical_amd import envs as mg_envs
from magical_amd import registry

TASKS = ["MoveToRegion", "MoveToCorner", "ClusterColour", "ClusterShape", "MatchRegions", "MakeLine",
         "FindDupe", "FixColour", "PickAndPlace"]
PREPROCS = [None, "LoRes4E", "LoResStack", "LoRes3EA", "LoRes4A", "LoResCHW4E", "LoResCHW4A"]
VARIANTS = {"PickAndPlace": ["Demo", "Test"]}


def _names():
    out = ["MoveToRegion-Demo-LoRes4E-v0", "MoveToCorner-Demo-LoRes4E-v0", "ClusterColour-Demo-LoResStack-v0",
           "MatchRegions-TestAll-LoRes4E-v0"]
    for t, task in enumerate(TASKS):
        variants = VARIANTS.get(task, ["Demo", "TestAll", "TestJitter"])
        for p, pre in enumerate(PREPROCS):
            if task == "PickAndPlace" and pre == "LoResStack":
                continue  # EagerDictFrameStack rejects its scalar observations (covered in test_gpu_parity)
            var = variants[(t + p) % len(variants)]
            name = f"{task}-{var}-{pre}-v0" if pre else f"{task}-{var}-v0"
            if name in registry.SPECS and name not in out:
                out.append(name)
    return out


N_ROLLOUTS = 2
CHECK_STEPS = 4


def _oracle_obs(spec, flat, orc):
    ref = collections.OrderedDict()
    off = 0
    for k, s in mg_envs._obs_shapes(spec).items():
        n = int(np.prod(s))
        ref[k] = flat[off:off + n].reshape(s)
        off += n
    if spec.task == "PickAndPlace":  # pick_and_place.py:103-107: ints and a float64 pair, after allo/ego
        t = orc.target()          # and before the frame stack's past_obs (benchmarks/__init__.py:136,146)
        extra = [("target_type", int(t[0])), ("target_colour", int(t[1])), ("target_position", t[2:4])]
        items = list(ref.items())
        ref = collections.OrderedDict(items[:2] + extra + items[2:])
    return ref


def _assert_obs(got, ref, where):
    assert list(got.keys()) == list(ref.keys()), where
    for k in ref:
        if isinstance(ref[k], int):
            assert got[k] == ref[k], (where, k)
        else:
            assert got[k].dtype == ref[k].dtype and np.array_equal(got[k], ref[k]), (where, k)


@pytest.mark.gpu
@pytest.mark.parametrize("env_name", _names())
def test_rollouts(env_name):
    spec = registry.lookup(env_name)
    env = magical_amd.make(env_name)
    orc = po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=7)
    try:
        env.seed(7)
        env.action_space.seed(42)
        try:
            obs = env.reset()
        except mg_envs.PlacementError:
            with pytest.raises(po.PlacementError):
                orc.reset()
            return
        _assert_obs(obs, _oracle_obs(spec, orc.reset(), orc), (env_name, "reset"))
        for k, space in env.observation_space.spaces.items():
            assert k in obs
        for ep in range(N_ROLLOUTS):
            done = False
            traj_len = 0
            while not done:
                action = env.action_space.sample()
                obs, rew, done, info = env.step(action)
                if ep == 0 and traj_len < CHECK_STEPS:
                    o, r, d, s = orc.step(int(action))
                    _assert_obs(obs, _oracle_obs(spec, o, orc), (env_name, traj_len))
                    assert rew == np.float32(r) and done == d and info["eval_score"] == s
                    if traj_len == 1:
                        frames = env.render("rgb_array")
                        assert isinstance(frames, collections.OrderedDict) and list(frames) == ["allo", "ego"]
                        a, g = orc.render_full()
                        assert frames["allo"].shape == (384, 384, 3) and np.array_equal(frames["allo"], a)
                        assert np.array_equal(frames["ego"], g)
                assert isinstance(rew, float) and isinstance(done, bool) and "eval_score" in info
                traj_len += 1
            assert traj_len == env.max_episode_steps
            assert 0.0 <= info["eval_score"] <= 1.0
            env.reset()
    finally:
        env.close()


@pytest.mark.gpu
def test_step_before_reset_raises():
    env = magical_amd.make("MoveToRegion-Demo-LoRes4E-v0", seed=0)
    try:
        with pytest.raises(RuntimeError):
            env.step(0)
    finally:
        env.close()


def test_single_env_names_cover_every_task_and_preprocessor():
    names = _names()
    specs = [registry.lookup(n) for n in names]
    assert {s.task for s in specs} == set(TASKS)
    assert {registry.EnvName(n).preproc for n in names} >= {"LoRes4E", "LoResStack", "LoRes3EA", "LoRes4A",
                                                             "LoResCHW4E", "LoResCHW4A", None}
