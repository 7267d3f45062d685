"""Demo data path: saved_trajectories.py's surface (magical_amd.demos).

CPU: the trajectory type, the class-rewriting gzip loader (on a demo file this test writes itself) and
the preprocessor-name splice.  GPU: preprocess_demos_with_wrapper / replay_lores (mg_replay_lores)
against the oracle -- every stored 384^2 frame downsampled with the oracle's cv2 INTER_AREA
restatement, the frame stacks rebuilt here from the reference wrappers' rules
(benchmarks/__init__.py:51-147: the reset observation fills the stack; LoRes3EA = allo_t + ego_t-2..t;
LoRes4E / CHW = ego_t-3..t; LoRes4A = allo_t-3..t; LoResStack = each key's last 4).  Frames: the
oracle's own full renders along random rollouts (so replaying them must also give the simulator's
LoRes observations of the same rollout) and random bytes (every rounding case of the area sum).
"""
import collections
import gzip
import pickle
import sys
import types

import numpy as np
import pytest
import torch

import pyoracle as po
import magical_amd
from magical_amd import demos, registry


def test_trajectory_type_and_splice():
    t = demos.MAGICALTrajectory(acts=np.zeros(3), obs=[{}] * 4, rews=np.zeros(3), infos=None)
    assert t._fields == ("acts", "obs", "rews", "infos")
    assert demos.splice_in_preproc_name("MoveToCorner-Demo-v0", "LoResStack") == "MoveToCorner-Demo-LoResStack-v0"
    with pytest.raises(AssertionError):
        demos.splice_in_preproc_name("MoveToCorner-Demo-v0", "HiRes")


def test_load_demos_rewrites_imitation_trajectory_class(tmp_path):
    """saved_trajectories.py:24-49: pickles that reference imitation.util.rollout.Trajectory load as
    MAGICALTrajectory (the file is written here, with a stand-in module of that name)."""
    mod = types.ModuleType("imitation.util.rollout")

    class Trajectory(tuple):
        def __new__(cls, acts, obs, rews, infos):
            return tuple.__new__(cls, (acts, obs, rews, infos))

        def __reduce__(self):
            return (Trajectory, tuple(self))
    Trajectory.__module__ = "imitation.util.rollout"
    Trajectory.__qualname__ = "Trajectory"
    mod.Trajectory = Trajectory
    for name in ("imitation", "imitation.util"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["imitation.util.rollout"] = mod
    try:
        path = tmp_path / "demo.pkl.gz"
        with gzip.GzipFile(path, "wb") as fp:
            pickle.dump({"env_name": "MoveToCorner-Demo-v0",
                         "trajectory": Trajectory(np.arange(3), [{"a": 1}] * 4, np.ones(3), [{}] * 3)}, fp)
    finally:
        for name in ("imitation.util.rollout", "imitation.util", "imitation"):
            sys.modules.pop(name, None)
    (d,) = list(demos.load_demos([str(path)]))
    assert isinstance(d["trajectory"], demos.MAGICALTrajectory)
    assert list(d["trajectory"].acts) == [0, 1, 2] and d["env_name"] == "MoveToCorner-Demo-v0"


def _oracle_stack(lo, starts, preproc):
    return po.stack_lores(lo, starts, preproc, registry.PREPROCESSORS[preproc].get("channels_first", False))


def _rollout_frames(name, seed, steps):
    spec = registry.lookup(name)
    o = po.OracleEnv(spec.task, spec.rand_flags, None, spec.max_episode_steps, seed=seed)
    o.reset()
    acts = np.random.RandomState(seed).randint(0, 18, steps)
    obs = []
    a, g = o.render_full()
    obs.append({"allo": a, "ego": g})
    for t in range(steps):
        o.step(int(acts[t]))
        a, g = o.render_full()
        obs.append({"allo": a, "ego": g})
    return demos.MAGICALTrajectory(acts=acts, obs=obs, rews=np.zeros(steps, np.float32),
                                   infos=[{"eval_score": 0.0}] * steps)


@pytest.mark.gpu
@pytest.mark.parametrize("preproc", ["LoRes4E", "LoRes3EA", "LoRes4A", "LoResStack", "LoResCHW4E", "LoResCHW4A"])
def test_preprocess_demos_matches_oracle(preproc):
    rs = np.random.RandomState(11)
    trajs = [_rollout_frames("MoveToCorner-Demo-v0", 3, 6), _rollout_frames("ClusterColour-Demo-v0", 4, 2)]
    noise = [{"allo": rs.randint(0, 256, (384, 384, 3), dtype=np.uint8),
              "ego": rs.randint(0, 256, (384, 384, 3), dtype=np.uint8)} for _ in range(5)]
    trajs.append(demos.MAGICALTrajectory(acts=np.arange(4), obs=noise, rews=np.arange(4.0), infos=[None] * 4))
    out = demos.preprocess_demos_with_wrapper(trajs, "MoveToCorner-Demo-v0", preproc)
    for traj, res in zip(trajs, out):
        lo = [(po.downsample(o["allo"]), po.downsample(o["ego"])) for o in traj.obs]
        want = _oracle_stack(lo, [0] * len(lo), preproc)
        assert len(res.obs) == len(traj.obs) and isinstance(res, demos.MAGICALTrajectory)
        for got, ref in zip(res.obs, want):
            assert list(got.keys()) == list(ref.keys())
            for k in ref:
                assert got[k].shape == ref[k].shape and np.array_equal(got[k], ref[k]), (preproc, k)
        assert np.array_equal(res.acts, traj.acts[:len(traj.acts)]) and np.array_equal(res.rews, traj.rews)
        assert res.infos == [i or {} for i in traj.infos]


@pytest.mark.gpu
def test_replay_of_simulator_frames_equals_its_lores_observations():
    """Replaying a GPU rollout's own 384^2 renders through mg_replay_lores gives the LoRes4E observations
    the simulator produced for that rollout, step for step (one episode incl. its reset frame)."""
    name, n, steps = "MoveToRegion-Demo-LoRes4E-v0", 5, 12
    vec = magical_amd.make_vec(name, n, seeds=[50 + i for i in range(n)])
    obs = vec.reset()
    frames, lores = [vec.render_full().clone()], [{k: v.clone() for k, v in obs.items()}]
    acts = np.random.RandomState(2).randint(0, 18, (steps, n))
    for t in range(steps):
        obs, _, _, _ = vec.step(torch.as_tensor(acts[t], dtype=torch.uint8))
        frames.append(vec.render_full().clone())
        lores.append({k: v.clone() for k, v in obs.items()})
    vec.close()
    F = torch.stack(frames, 1).reshape(n * (steps + 1), 2, 384, 384, 3)          # env-major
    starts = torch.tensor([(i // (steps + 1)) * (steps + 1) for i in range(n * (steps + 1))], dtype=torch.int32)
    got = demos.replay_lores(F, starts, "LoRes4E")
    for k in ("allo", "ego", "past_obs"):
        want = torch.stack([lores[t][k] for t in range(steps + 1)], 1).reshape((n * (steps + 1),) + lores[0][k].shape[1:])
        assert torch.equal(got[k], want), k


@pytest.mark.gpu
def test_replay_rejects_bad_arguments():
    with pytest.raises(ValueError):
        demos.replay_lores(torch.zeros((1, 2, 384, 384, 3), dtype=torch.uint8, device="cuda"), [0], "HiRes")
    with pytest.raises(ValueError):
        demos.replay_lores(torch.zeros((1, 2, 96, 96, 3), dtype=torch.uint8, device="cuda"), [0], "LoRes4E")


@pytest.mark.gpu
def test_replay_matches_reference_wrapper_fixtures():
    """mg_replay_lores (through preprocess_demos_with_wrapper) on the synthetic frame sequences of
    tests/golden/ref_wrappers.json -- the REFERENCE's own entry points executed in the build container --
    gives the reference's observations bit for bit (sha256), for every LoRes preprocessor, with the
    sequence's mid-point reset as a second trajectory."""
    import hashlib
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_wrappers.json")))
    ev = g["events"]
    cut = ev.index("reset", 1)
    for case in g["cases"]:
        frames = [np.random.RandomState(1000 * case["case"] + j).randint(0, 256, (2, 384, 384, 3), dtype=np.uint8)
                  for j in range(len(ev))]
        trajs = []
        for lo, hi in ((0, cut), (cut, len(ev))):
            obs = [{"allo": f[0], "ego": f[1]} for f in frames[lo:hi]]
            k = hi - lo - 1
            trajs.append(demos.MAGICALTrajectory(acts=np.zeros(k, np.int64), obs=obs, rews=np.zeros(k, np.float32),
                                                 infos=[{}] * k))
        out = demos.preprocess_demos_with_wrapper(trajs, "MoveToCorner-Demo-v0", case["preproc"])
        got = list(out[0].obs) + list(out[1].obs)
        for j, ref in enumerate(case["obs"]):
            assert [k for k, *_ in ref] == list(got[j]), (case["preproc"], j)
            for k, shape, dtype, h in ref:
                v = np.ascontiguousarray(got[j][k])
                assert list(v.shape) == shape and str(v.dtype) == dtype, (case["preproc"], j, k)
                assert hashlib.sha256(v.tobytes()).hexdigest() == h, (case["preproc"], j, k)
