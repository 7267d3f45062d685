"""CPU: host-side logic -- env-name registry, C-ABI library exports, the
observation layout helpers and the multi-process sharding path (gloo)."""
import ctypes
import os
import re
import socket
import subprocess
import sys

import numpy as np
import pytest

import magical_amd
from magical_amd import dist as mdist
from magical_amd import native, registry

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


# --------------------------------------------------------------------------- registry
def test_registry_matches_golden_table():
    import json
    g = json.load(open(os.path.join(GOLDEN, "registry.json")))
    assert list(registry.ALL_REGISTERED_ENVS) == g["names"]
    assert len(g["names"]) == 441
    for lit in g["reference_literals"]:
        if lit != "-v0":
            assert lit in registry.SPECS, lit


def test_env_name_grammar_and_update():
    n = registry.EnvName("MoveToCorner-TestAll-LoResStack-v0")
    assert (n.task, n.variant, n.preproc, n.version, n.is_test) == ("MoveToCorner", "TestAll", "LoResStack", "v0", True)
    assert n.demo_env_name == "MoveToCorner-Demo-LoResStack-v0"
    assert registry.update_magical_env_name("MoveToCorner-Demo-v0", preproc="LoRes4E") == "MoveToCorner-Demo-LoRes4E-v0"
    assert registry.update_magical_env_name("MoveToCorner-Demo-LoRes4E-v0", variant="TestJitter") == \
        "MoveToCorner-TestJitter-LoRes4E-v0"
    with pytest.raises(ValueError):
        registry.EnvName("not-an-env")


def test_specs_of_bench_configs():
    s = registry.lookup("MoveToRegion-Demo-LoRes4E-v0")
    assert (s.task, s.rand_flags, s.preproc, s.max_episode_steps) == ("MoveToRegion", 0, "LoRes4E", 40)
    s = registry.lookup("MatchRegions-TestAll-LoRes4E-v0")
    assert s.rand_flags == 2 | 4 | 8 | 16 | 32 and s.max_episode_steps == 120
    s = registry.lookup("ClusterColour-Demo-LoResStack-v0")
    assert s.max_episode_steps == 240 and s.preproc == "LoResStack"
    assert registry.lookup("MoveToCorner-Demo-DebugReward-LoRes4E-v0").preproc is None  # fork quirk
    assert registry.PREPROCESSORS["LoResCHW4A"] == registry.PREPROCESSORS["LoResCHW4E"]
    with pytest.raises(KeyError):
        registry.lookup("MoveToRegion-Demo-LoRes9X-v0")


def test_demo_to_test_map():
    m = registry.DEMO_ENVS_TO_TEST_ENVS_MAP
    assert "MoveToRegion-Demo-v0" in m
    assert "MoveToRegion-TestAll-v0" in m["MoveToRegion-Demo-v0"]
    assert all(registry.EnvName(t).is_test for ts in m.values() for t in ts)


def test_observation_spaces():
    from magical_amd.envs import _obs_shapes
    assert dict(_obs_shapes(registry.lookup("MoveToRegion-Demo-LoRes4E-v0"))) == \
        {"allo": (96, 96, 3), "ego": (96, 96, 3), "past_obs": (96, 96, 12)}
    assert dict(_obs_shapes(registry.lookup("MoveToRegion-Demo-LoResCHW4E-v0")))["past_obs"] == (12, 96, 96)
    shapes = _obs_shapes(registry.lookup("ClusterColour-Demo-LoResStack-v0"))
    assert sum(int(np.prod(s)) for s in shapes.values()) == 2 * 96 * 96 * 12


# --------------------------------------------------------------------------- C ABI
def _header_functions():
    src = open(os.path.join(ROOT, "include", "magical_sim.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mg_[a-z_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert _header_functions() == sorted(native.EXPORTS)


def test_library_loads_and_exports_every_header_symbol():
    lib = native.load()
    for name in _header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (mg_\w+)", out))
    assert set(_header_functions()) <= exported


def test_library_is_gfx950_code_object():
    data = open(native.LIB_PATH, "rb").read()
    assert b"gfx950" in data  # the embedded offload bundle targets amdgcn-amd-amdhsa--gfx950


def test_abi_argument_validation_without_gpu():
    lib = native.load()
    h = ctypes.c_void_p()
    assert lib.mg_create(None, ctypes.byref(h)) != 0
    assert b"null" in lib.mg_last_error()
    cfg = native.mg_config(task=0, rand_flags=0, preproc=1, num_envs=4, device=0, max_episode_steps=40,
                           base_seed=0, auto_reset=1, seeds=None, library=None, library_size=3)
    assert lib.mg_create(ctypes.byref(cfg), ctypes.byref(h)) != 0
    assert b"library_size" in lib.mg_last_error()
    assert lib.mg_step(None, None, None) != 0
    assert lib.mg_read_timing(None, None) != 0


def test_product_path_has_no_cpu_fallback(tmp_path, monkeypatch):
    monkeypatch.setattr(native, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(native, "_lib", None)
    with pytest.raises(native.NativeError):
        native.load()


# --------------------------------------------------------------------------- sharding
def test_shard_seeds_partition_the_global_batch():
    w, n = 4, 5
    allseeds = sum((mdist.shard_seeds(n, r) for r in range(w)), [])
    assert allseeds == [1000 + i for i in range(w * n)]
    assert mdist.shard_range(n, 2) == (10, 15)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = r'''
import os, sys
sys.path[:0] = [{root!r} + "/magical-1_amd", {root!r} + "/oracle"]
import numpy as np, torch, torch.distributed as dist
import pyoracle as po
from magical_amd import dist as mdist, registry
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="env://")
spec = registry.lookup("MoveToRegion-Demo-LoRes4E-v0")
n, steps = 2, 6
envs = [po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=s)
        for s in mdist.shard_seeds(n, rank)]
obs = np.stack([e.reset() for e in envs])
acts = np.random.RandomState(5).randint(0, 18, (steps, world * n))
lo, hi = mdist.shard_range(n, rank)
for t in range(steps):
    obs = np.stack([e.step(int(a))[0] for e, a in zip(envs, acts[t, lo:hi])])
full = mdist.all_gather_batch({{"obs": torch.from_numpy(obs)}})["obs"].numpy()
el = torch.tensor([float(rank + 1)], dtype=torch.float64)
dist.all_reduce(el, op=dist.ReduceOp.MAX)
if rank == 0:
    np.save({out!r}, full)
    assert el.item() == world
dist.destroy_process_group()
'''


def test_two_rank_gloo_sharded_rollout_equals_single_process(tmp_path):
    """world_size 2 on CPU: each rank runs its contiguous shard, the gathered
    batch equals one process running all envs (seed/order bookkeeping of the
    multi-GPU path), and max-over-ranks timing reduction works."""
    out = str(tmp_path / "full.npy")
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, out=out))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    full = np.load(out)
    import pyoracle as po
    spec = registry.lookup("MoveToRegion-Demo-LoRes4E-v0")
    acts = np.random.RandomState(5).randint(0, 18, (6, 4))
    envs = [po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=1000 + i)
            for i in range(4)]
    for e in envs:
        e.reset()
    for t in range(6):
        ref = np.stack([e.step(int(a))[0] for e, a in zip(envs, acts[t])])
    assert np.array_equal(full, ref)


PACKED_WORKER = r'''
import os, sys
sys.path[:0] = [{root!r} + "/magical-1_amd", {root!r} + "/oracle"]
import numpy as np, torch, torch.distributed as dist
import pyoracle as po
from magical_amd import dist as mdist, registry, envs as mg_envs
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="env://")
name = {name!r}
spec = registry.lookup(name)
n, steps = 2, 7

class OracleVec:
    """CPU stand-in for VecMagicalEnv's output binding: the oracle writes each step into the bound views"""
    device = torch.device("cpu")
    def __init__(self, seeds):
        self.envs = [po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=s) for s in seeds]
    def bind_outputs(self, views):
        self.v = views
    def _write(self, i, flat, r=0.0, d=False, sc=0.0):
        off = 0
        for k, s in mg_envs._obs_shapes(spec).items():
            m = int(np.prod(s))
            self.v[k][i].copy_(torch.from_numpy(flat[off:off + m].reshape(self.v[k][i].shape)))
            off += m
        self.v["reward"][i] = r; self.v["done"][i] = d; self.v["eval_score"][i] = sc
    def reset(self):
        for i, e in enumerate(self.envs):
            self._write(i, e.reset())
    def step(self, actions):
        for i, e in enumerate(self.envs):
            o, r, d, sc = e.step(int(actions[i]))
            if d:
                o = e.reset()
            self._write(i, o, r, d, sc)
    def close(self):
        pass

vec = OracleVec(mdist.shard_seeds(n, rank))
env = mdist.ShardedVecEnv(name, n, rank=rank, gather=True, vec=vec, device="cpu")
acts = np.random.RandomState(5).randint(0, 18, (steps, world * n))
lo, hi = mdist.shard_range(n, rank)
obs = env.reset()
handles = []
for t in range(steps):
    handles.append(env.step_async(torch.as_tensor(acts[t, lo:hi])))
obs, rew, done, info = handles[-1].results()
if rank == 0:
    np.savez({out!r}, **{{k: v.numpy() for k, v in obs.items()}}, reward=rew.numpy(), done=done.numpy(),
             score=info["eval_score"].numpy(), nbytes=env.layout.nbytes)
env.close()
dist.destroy_process_group()
'''


@pytest.mark.parametrize("name", ["MoveToRegion-Demo-LoRes4E-v0", "ClusterColour-Demo-LoResStack-v0"])
def test_two_rank_gloo_packed_gather_pipeline(tmp_path, name):
    """ShardedVecEnv(gather=True) with world_size 2 on CPU tensors: each rank's step outputs are
    written into views of one packed buffer, one all_gather_into_tensor per step, two buffers
    alternating (step_async handles of 7 steps kept, the last one read).  The unpacked [W, n, ...]
    views equal one process running all W * n envs: observations, reward, done, eval_score,
    across an episode boundary (MoveToRegion: done at 40 is not reached; LoResStack keys)."""
    out = str(tmp_path / "full.npz")
    script = tmp_path / "worker.py"
    script.write_text(PACKED_WORKER.format(root=ROOT, out=out, name=name))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    got = np.load(out)
    import pyoracle as po
    from magical_amd import envs as mg_envs
    spec = registry.lookup(name)
    steps, W, n = 7, 2, 2
    acts = np.random.RandomState(5).randint(0, 18, (steps, W * n))
    envs = [po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=1000 + i)
            for i in range(W * n)]
    for e in envs:
        e.reset()
    for t in range(steps):
        res = [e.step(int(a)) for e, a in zip(envs, acts[t])]
    shapes = mg_envs._obs_shapes(spec)
    for i, (o, r, d, sc) in enumerate(res):
        off = 0
        for k, s in shapes.items():
            m = int(np.prod(s))
            assert np.array_equal(got[k][i // n, i % n], o[off:off + m].reshape(s)), (k, i)
            off += m
        assert got["reward"][i // n, i % n] == np.float32(r) and bool(got["done"][i // n, i % n]) == d
        assert got["score"][i // n, i % n] == sc
    assert int(got["nbytes"]) % 256 == 0


# --------------------------------------------------------------------------- evaluation protocol
def test_evaluation_protocol_statistics():
    """evaluation.py:13-98: one record per test env of the demo env, mean / t-CI / std (ddof=1),
    extra scores truncated with a warning, too few scores rejected."""
    import warnings
    import numpy as np
    from scipy import stats
    from magical_amd import evaluation

    rs = np.random.RandomState(0)
    table = {}

    class Fixed(evaluation.EvaluationProtocol):
        run_id = "fixed"

        def obtain_scores(self, env_name):
            return table.setdefault(env_name, rs.rand(self.n_rollouts + 2).tolist())

    proto = Fixed("MoveToCorner-Demo-v0", 10)
    assert proto.test_env_names[0] == "MoveToCorner-Demo-v0" and len(proto.test_env_names) == 6
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        frame = proto.do_eval()
    assert len(w) == len(proto.test_env_names)
    assert list(frame["test_env"]) == proto.test_env_names
    for _, row in frame.iterrows():
        s = np.asarray(table[row["test_env"]][:10])
        lo, hi = stats.t.interval(0.95, len(s) - 1, loc=s.mean(), scale=stats.sem(s))
        assert np.isclose(row["mean_score"], s.mean()) and np.isclose(row["std_score"], s.std(ddof=1))
        assert np.isclose(row["ci95_lower"], lo) and np.isclose(row["ci95_upper"], hi)

    class Short(Fixed):
        def obtain_scores(self, env_name):
            return [0.5] * 3
    import pytest
    with pytest.raises(ValueError):
        Short("MoveToCorner-Demo-v0", 10).do_eval()
