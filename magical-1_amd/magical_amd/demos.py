"""Demo data path: saved_trajectories.py's surface, with the preprocessing replay
on the GPU.

* MAGICALTrajectory, load_demos, splice_in_preproc_name: saved_trajectories.py:14-61 (same names,
  fields and behaviour; load_demos unpickles the caller's own gzip files, as the reference does).
* preprocess_demos_with_wrapper(trajectories, orig_env_name, preproc_name): saved_trajectories.py:87-149.
  The reference replays each trajectory's stored 384^2 observations through the preprocessor's gym
  wrappers (_MockDemoEnv, :63-84): frame stacks filled by the reset observation, then cv2 INTER_AREA
  to 96^2.  Here every frame of every trajectory goes to the device at once and mg_replay_lores
  (csrc/mg_replay.hip) produces the LoRes observations; the returned trajectories have the
  reference's layout (obs: one dict per step, acts / rews stacked, infos as given).
* replay_lores(frames, episode_start, preproc): the device-level entry for consumers that keep the
  batch on the GPU (imitation training, train_il.py:215-250).
"""
import collections
import ctypes
import gzip
from pickle import Unpickler
from typing import List, NamedTuple, Optional

import numpy as np
import torch

from . import native, registry

_GPU_PREPROC = {"LoRes4E": 1, "LoResCHW4E": 1, "LoResCHW4A": 1, "LoResStack": 2, "LoRes3EA": 3, "LoRes4A": 4}


class MAGICALTrajectory(NamedTuple):
    """Trajectory representation compatible with imitation's trajectory data class
    (saved_trajectories.py:14-21)."""

    acts: np.ndarray
    obs: dict
    rews: np.ndarray
    infos: Optional[List[dict]]


class _TrajRewriteUnpickler(Unpickler):
    """saved_trajectories.py:24-33: references to imitation's / milbench's trajectory classes load as
    MAGICALTrajectory."""

    def find_class(self, module, name):
        if (module, name) in (("imitation.util.rollout", "Trajectory"),
                              ("milbench.baselines.saved_trajectories", "MILBenchTrajectory")):
            return MAGICALTrajectory
        return super().find_class(module, name)


def load_demos(demo_paths, rewrite_traj_cls=True, verbose=False):
    """saved_trajectories.py:36-49: GzipFile + pickle, one demo dict per path (lazily)."""
    n_demos = len(demo_paths)
    for d_num, d_path in enumerate(demo_paths, start=1):
        if verbose:
            print(f"Loading '{d_path}' ({d_num}/{n_demos})")
        with gzip.GzipFile(d_path, "rb") as fp:
            unpickler = _TrajRewriteUnpickler(fp) if rewrite_traj_cls else Unpickler(fp)
            this_dict = unpickler.load()
        yield this_dict


def splice_in_preproc_name(base_env_name, preproc_name):
    """saved_trajectories.py:52-60: MoveToCorner-Demo-v0 + LoResStack -> MoveToCorner-Demo-LoResStack-v0."""
    assert preproc_name in registry.PREPROCESSORS, \
        f"no preprocessor named '{preproc_name}', options are {', '.join(registry.PREPROCESSORS)}"
    return registry.update_magical_env_name(base_env_name, preproc=preproc_name)


def replay_lores(frames, episode_start, preproc, out=None):
    """LoRes observations of stored frames on the GPU.

    frames: u8 [F, 2, 384, 384, 3] (allo, ego) CUDA tensor; episode_start: i32 [F] (index of the first frame
    of each frame's trajectory); preproc: a LoRes preprocessor name.  Returns an OrderedDict of device
    tensors for the F frames: allo/ego [F,96,96,3] and past_obs [F,96,96,12] (LoResStack: allo/ego
    [F,96,96,12]); channels-first preprocessors return permuted views, as VecMagicalEnv does."""
    if preproc not in _GPU_PREPROC:
        raise ValueError(f"replay_lores: {preproc!r} is not a LoRes preprocessor ({', '.join(_GPU_PREPROC)})")
    frames = frames.contiguous()
    if frames.dtype != torch.uint8 or frames.dim() != 5 or tuple(frames.shape[1:]) != (2, 384, 384, 3):
        raise ValueError("replay_lores: frames must be u8 [F, 2, 384, 384, 3]")
    F = frames.shape[0]
    dev = frames.device
    es = torch.as_tensor(episode_start, dtype=torch.int32).to(dev).contiguous()
    if es.shape != (F,):
        raise ValueError("replay_lores: episode_start must be i32 [F]")
    pid = _GPU_PREPROC[preproc]
    u8 = dict(dtype=torch.uint8, device=dev)
    c = 12 if pid == 2 else 3
    allo = torch.empty((F, 96, 96, c), **u8)
    ego = torch.empty((F, 96, 96, c), **u8)
    past = None if pid == 2 else torch.empty((F, 96, 96, 12), **u8)
    scratch = torch.empty((F, 2, 96, 96, 3), **u8)
    lib = native.load()
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    native.check(lib.mg_replay_lores(p(frames), F, p(es), pid, p(scratch), p(allo), p(ego), p(past), stream))
    out = collections.OrderedDict([("allo", allo), ("ego", ego)])
    if past is not None:
        out["past_obs"] = past
    if registry.PREPROCESSORS[preproc].get("channels_first", False):
        out = collections.OrderedDict((k, v.permute(0, 3, 1, 2)) for k, v in out.items())
    return out


def preprocess_demos_with_wrapper(trajectories, orig_env_name, preproc_name=None, wrapper=None, device="cuda:0",
                                  max_frames_per_batch=2048):
    """saved_trajectories.py:87-149 on the GPU for the named LoRes preprocessors.

    Each trajectory has T actions and T + 1 observations (dicts with 'allo' and 'ego' 384^2 frames and
    possibly non-image extras such as PickAndPlace's targets, which pass through as the reference's
    wrappers pass them).  Returns trajectories of the same type with obs an array of T + 1 preprocessed
    dicts (np.stack of the per-step dicts, as the reference builds it), acts / rews stacked and infos
    kept."""
    if wrapper is not None or preproc_name is None:
        raise NotImplementedError("preprocess_demos_with_wrapper: the GPU replay takes a preprocessor name "
                                  f"({', '.join(_GPU_PREPROC)}); custom wrapper constructors are not replayed")
    assert preproc_name in _GPU_PREPROC, preproc_name
    registry.lookup(orig_env_name)   # the reference instantiates orig_env_name: unknown names fail alike
    trajectories = list(trajectories)
    dev = torch.device(device)
    stacked = preproc_name == "LoResStack"
    results = [None] * len(trajectories)
    batch, nf = [], 0

    def flush():
        nonlocal batch, nf
        if not batch:
            return
        frames = np.empty((nf, 2, 384, 384, 3), dtype=np.uint8)
        starts = np.empty(nf, dtype=np.int32)
        off = 0
        for ti, traj in batch:
            T1 = len(traj.acts) + 1
            for k in range(T1):
                o = traj.obs[k]
                frames[off + k, 0] = o["allo"]
                frames[off + k, 1] = o["ego"]
            starts[off:off + T1] = off
            off += T1
        got = replay_lores(torch.from_numpy(frames).to(dev), torch.from_numpy(starts).to(dev), preproc_name)
        got = {k: v.cpu().numpy() for k, v in got.items()}
        off = 0
        for ti, traj in batch:
            T1 = len(traj.acts) + 1
            obs_list = []
            for k in range(T1):
                src = traj.obs[k]
                extras = [(key, val) for key, val in src.items() if key not in ("allo", "ego")]
                if stacked and extras:
                    # EagerDictFrameStack concatenates every value: the reference raises on scalar extras
                    raise ValueError("LoResStack cannot stack non-image observation values "
                                     f"({', '.join(k_ for k_, _ in extras)})")
                d = collections.OrderedDict([("allo", got["allo"][off + k]), ("ego", got["ego"][off + k])])
                d.update(extras)                      # base-env keys keep their order, past_obs goes last
                if "past_obs" in got:
                    d["past_obs"] = got["past_obs"][off + k]
                obs_list.append(d)
            off += T1
            if traj.infos is None:                    # _MockDemoEnv.step indexes traj.infos
                raise TypeError("'NoneType' object is not subscriptable")
            infos = [info or {} for info in traj.infos[:T1 - 1]]
            obs_arr = np.empty(T1, dtype=object)
            obs_arr[:] = obs_list
            results[ti] = type(traj)(acts=np.stack([traj.acts[k] for k in range(T1 - 1)], axis=0),
                                     obs=obs_arr,
                                     rews=np.stack([traj.rews[k] for k in range(T1 - 1)], axis=0),
                                     infos=infos)
        batch, nf = [], 0

    for ti, traj in enumerate(trajectories):
        T1 = len(traj.acts) + 1
        if len(traj.obs) < T1:
            raise IndexError(f"trajectory {ti}: {len(traj.acts)} actions need {T1} observations, got {len(traj.obs)}")
        if nf + T1 > max_frames_per_batch and batch:
            flush()
        batch.append((ti, traj))
        nf += T1
    flush()
    return results
