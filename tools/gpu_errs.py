"""Diagnose per-env error flags at full size: which envs, which bits, and
whether those envs still match the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "magical-1_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import magical_amd  # noqa: E402
import pyoracle as po  # noqa: E402
from magical_amd import registry  # noqa: E402
from test_gpu_parity import oracle_obs_split  # noqa: E402

name, n, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
spec = registry.lookup(name)
seeds = [1000 + i for i in range(n)]
vec = magical_amd.make_vec(name, n, seeds=seeds)
acts = np.random.RandomState(9).randint(0, 18, (steps, n))
vec.reset()
err_first = {}
e = vec.errors().cpu().numpy()
for i in np.flatnonzero(e):
    err_first[int(i)] = (-1, int(e[i]))
obs_hist = []
for t in range(steps):
    obs, rew, done, info = vec.step(torch.as_tensor(acts[t], dtype=torch.uint8))
    e = vec.errors().cpu().numpy()
    for i in np.flatnonzero(e):
        if int(i) not in err_first:
            err_first[int(i)] = (t, int(e[i]))
print("errors (env: first step, flags):", err_first)
for i, (t0, fl) in list(err_first.items())[:6]:
    o = po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=seeds[i])
    o.reset()
    print("env", i, "oracle arbiters per step:", end=" ")
    for t in range(min(steps, t0 + 2)):
        o.step(int(acts[t, i]))
        print(o.num_arbiters(), end=" ")
    print()
    k, ty, c, p = o.entities()
    print("  entities kinds", k.tolist(), "types", ty.tolist())
