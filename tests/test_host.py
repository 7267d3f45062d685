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


_C_TO_CTYPES = {"int32_t": ctypes.c_int32, "uint32_t": ctypes.c_uint32, "int64_t": ctypes.c_int64,
                "double": ctypes.c_double}


def _header_structs():
    """{struct name: [(field, ctypes type or 'ptr')]} of the header's typedef'd structs, in field order."""
    src = open(os.path.join(ROOT, "include", "magical_sim.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for body, name in re.findall(r"typedef struct \{(.*?)\}\s*(\w+);", src, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            m = re.match(r"(?:const\s+)?(\w+)\s*(\*?)\s*(\w+)$", decl)
            assert m, decl
            fields.append((m.group(3), "ptr" if m.group(2) else _C_TO_CTYPES[m.group(1)]))
        out[name] = fields
    return out


def _integration_stub():
    """Execute INTEGRATION.md section 2's ctypes stub with a recorder in place of ctypes.CDLL."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2."):text.index("## 3.")]
    code = re.search(r"```python\n(.*?)```", sec, flags=re.S).group(1)

    class Fn:
        pass

    class Lib:
        def __getattr__(self, name):
            f = Fn()
            object.__setattr__(self, name, f)
            return f

    ns = {"__Lib": Lib, "__name__": "integration_stub"}
    exec(compile(code.replace('ctypes.CDLL("magical_amd/libmagical_sim.so")', "__Lib()"), "INTEGRATION.md", "exec"),
         ns)
    return ns


def _same_ctype(a, b):
    if a is b:
        return True
    # POINTER(X) of two different Structure classes with the same layout
    return (getattr(a, "_type_", None) is not None and getattr(b, "_type_", None) is not None and
            issubclass(a, ctypes._Pointer) and issubclass(b, ctypes._Pointer) and
            [f[0] for f in getattr(a._type_, "_fields_", [])] == [f[0] for f in getattr(b._type_, "_fields_", [])])


def test_integration_stub_matches_binding_and_header():
    """INTEGRATION.md's ctypes stub (what a reference maintainer would copy) declares the same struct fields,
    in the same order with the same types, as magical_amd/native.py and include/magical_sim.h (a short
    mg_buffers makes mg_bind_outputs read past the caller's struct), and the same argument lists for every
    function it binds."""
    ns = _integration_stub()
    header = _header_structs()
    for name in ("mg_config", "mg_buffers"):
        stub = [(f, t) for f, t in ns[name]._fields_]
        ours = [(f, t) for f, t in getattr(native, name)._fields_]
        assert [f for f, _ in stub] == [f for f, _ in ours] == [f for f, _ in header[name]], name
        for (f, ts), (_, to), (_, th) in zip(stub, ours, header[name]):
            assert ts is to, (name, f)
            if th == "ptr":
                assert ts is ctypes.c_void_p or issubclass(ts, ctypes._Pointer), (name, f)
            else:
                assert ts is th, (name, f)
        assert ctypes.sizeof(ns[name]) == ctypes.sizeof(getattr(native, name))
    lib = native.load()
    stub_lib = ns["lib"]
    bound = [k for k in vars(stub_lib) if k.startswith("mg_")]
    assert {"mg_create", "mg_bind_outputs", "mg_step", "mg_restack", "mg_replay_lores"} <= set(bound)
    for fn in bound:
        f = getattr(stub_lib, fn)
        if hasattr(f, "argtypes"):
            ref = getattr(lib, fn).argtypes
            assert len(f.argtypes) == len(ref), fn
            assert all(_same_ctype(a, b) for a, b in zip(f.argtypes, ref)), fn
    # the check itself fails on a removed field
    short = [f for f in ns["mg_buffers"]._fields_ if f[0] != "frames_only"]
    assert [f for f, _ in short] != [f for f, _ in header["mg_buffers"]]


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


PACKED_WORKER = r"""
import os, sys
sys.path[:0] = [{root!r} + "/magical-1_amd", {root!r} + "/oracle"]
import numpy as np, torch, torch.distributed as dist
import pyoracle as po
from magical_amd import dist as mdist, registry, envs as mg_envs
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="env://")
name, mode, L = {name!r}, {mode!r}, {L}
spec = registry.lookup(name)
n, steps = 2, {steps}
CHW = registry.PREPROCESSORS[spec.preproc].get("channels_first", False)

class OracleVec:
    # CPU stand-in for VecMagicalEnv's output binding: the oracle writes each step into the bound views
    # (frames_only: the current frame of each view only, as the simulator's frames-only mode does)
    device = torch.device("cpu")
    def __init__(self, seeds):
        self.envs = [po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, L, seed=s) for s in seeds]
        self.target = torch.zeros((len(seeds), 4), dtype=torch.float64) if spec.task == "PickAndPlace" else None
    def bind_outputs(self, views, frames_only=False):
        self.v, self.fo = views, frames_only
    def _write(self, i, flat, r=0.0, d=False, sc=0.0):
        off = 0
        for k, s in mg_envs._obs_shapes(spec).items():
            m = int(np.prod(s))
            a = flat[off:off + m].reshape(s)
            off += m
            if CHW:   # the oracle writes channels-first bytes; the bound buffers are HWC
                a = a.transpose(1, 2, 0)
            if self.fo:
                if k == "past_obs":
                    continue
                a = a[..., 9:12] if a.shape[-1] == 12 else a   # LoResStack: the newest frame of the stack
            self.v[k][i].copy_(torch.from_numpy(np.ascontiguousarray(a)).reshape(self.v[k][i].shape))
        self.v["reward"][i] = r; self.v["done"][i] = d; self.v["eval_score"][i] = sc
    def _reset_one(self, i):
        o = self.envs[i].reset()
        if self.target is not None:
            self.target[i] = torch.from_numpy(self.envs[i].target())
        return o
    def reset(self):
        for i in range(len(self.envs)):
            self._write(i, self._reset_one(i))
    def step(self, actions):
        for i, e in enumerate(self.envs):
            o, r, d, sc = e.step(int(actions[i]))
            if d:
                o = self._reset_one(i)
            self._write(i, o, r, d, sc)
    def close(self):
        pass

vec = OracleVec(mdist.shard_seeds(n, rank))
lay = mdist.PackedLayout.for_spec(spec, n, frames_only=mode == "frames")
env = mdist.ShardedVecEnv(name, n, rank=rank, gather=True, vec=vec, device="cpu", gather_mode=mode,
                          restacker=po.OracleRestacker(lay, spec.preproc) if mode == "frames" else None)
acts = np.random.RandomState(5).randint(0, 18, (steps, world * n))
lo, hi = mdist.shard_range(n, rank)
rec = {{}}
def keep(t, obs, rew=None, done=None, info=None):
    for k, v in obs.items():
        rec.setdefault(k, []).append(v.clone().numpy())
    if rew is not None:
        rec.setdefault("reward", []).append(rew.clone().numpy()); rec.setdefault("done", []).append(done.clone().numpy())
        rec.setdefault("score", []).append(info["eval_score"].clone().numpy())
        if "target" in info:
            rec.setdefault("target", []).append(info["target"].clone().numpy())
keep(-1, env.reset())
prev = None
for t in range(steps):
    h = env.step_async(torch.as_tensor(acts[t, lo:hi]))
    if prev is not None:      # the previous step's exchange, read after this step was launched
        keep(t - 1, *prev.results())
    prev = h
keep(steps - 1, *prev.results())
if rank == 0:
    np.savez({out!r}, nbytes=env.layout.nbytes, stacked_nbytes=env.stacked_nbytes,
             **{{k: np.stack(v) for k, v in rec.items()}})
env.close()
dist.destroy_process_group()
"""

def test_frames_gather_refuses_a_stale_ring():
    """gather_mode 'frames' rebuilds stacks from the receivers' frame rings, which only reset_async()
    fills -- step_async() raises before the shard's first reset_async() and after a direct reset of the
    VecMagicalEnv underneath; CPU tensors default to gather_mode 'stacked' (no restacker needed); the ring holds
    only the stacked outputs' views."""
    import torch
    import torch.distributed as tdist
    name, n = "MoveToRegion-Demo-LoRes4E-v0", 2
    spec = registry.lookup(name)

    class FakeVec:
        device = torch.device("cpu")
        def __init__(self):
            self.reset_count = 0
        def bind_outputs(self, views, frames_only=False):
            self.v = views
        def reset(self):
            self.reset_count += 1
            for t in self.v.values():
                t.zero_()
        def step(self, actions):
            pass
        def close(self):
            pass

    restacked = []
    stacker = lambda recv, outs, step, all_fresh: restacked.append((step, all_fresh))  # noqa: E731
    assert mdist.ShardedVecEnv(name, n, rank=0, gather=True, vec=FakeVec(), device="cpu").gather_mode == "stacked"
    env = mdist.ShardedVecEnv(name, n, rank=0, gather=True, vec=FakeVec(), device="cpu", restacker=stacker)
    assert env.gather_mode == "frames"
    with pytest.raises(RuntimeError, match="before the first step"):
        env.step_async(torch.zeros(n, dtype=torch.uint8))
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        env.reset_async()
        env.step_async(torch.zeros(n, dtype=torch.uint8))
        env.vec.reset()
        with pytest.raises(RuntimeError, match="reset directly"):
            env.step_async(torch.zeros(n, dtype=torch.uint8))
        env.reset_async()
        env.step_async(torch.zeros(n, dtype=torch.uint8))
        env.close()
    finally:
        tdist.destroy_process_group()
    assert restacked == [(0, True), (1, False), (2, True), (3, False)]
    fr = 96 * 96 * 3
    assert mdist.restack_ring_bytes("LoRes4E", 8, 10) == 4 * 80 * fr
    assert mdist.restack_ring_bytes("LoResStack", 8, 10) == 2 * 4 * 80 * fr
    assert spec.preproc == "LoRes4E"


@pytest.mark.parametrize("preproc,K", [("LoRes4E", 8), ("LoResStack", 8), ("LoRes4A", 4), ("LoRes4E", 5)])
def test_window_ring_view_contract(preproc, K):
    """The window ring's host contract (include/magical_sim.h mg_restack_window, magical_amd.dist.window_view) on
    CPU: a ring filled by the kernel's slot rule -- frame t planar into slot t % K and, when t % K < 3, slot
    K + t % K; a fresh env into the slots of frames t-3 .. t -- read through window_view at s0 = (t + K - 3) % K
    gives the oracle's restatement of the reference's frame-stack rule (po.OracleRestacker) at every step,
    across wraps, duplicate slots, per-env auto-resets and an all-fresh reset.  (The GPU kernel itself is
    checked against both in tests/test_gpu_parity.py.)"""
    import torch
    import pyoracle as po
    name = {"LoRes4E": "MoveToRegion-Demo-LoRes4E-v0", "LoResStack": "ClusterColour-Demo-LoResStack-v0",
            "LoRes4A": "MoveToRegion-Demo-LoRes4A-v0"}[preproc]
    spec = registry.lookup(name)
    W, n = 2, 3
    lay = mdist.PackedLayout.for_spec(spec, n, frames_only=True)
    keys = mdist.stacked_keys(preproc)
    ring = torch.zeros(mdist.window_ring_bytes(preproc, W, n, K) + 7, dtype=torch.uint8)[7:]   # an offset storage
    rv = ring.view(len(keys), W * n, K + 3, 3, 96, 96)
    orc = po.OracleRestacker(lay, preproc)
    rs = np.random.RandomState(5)
    for t in range(3 * K + 2):
        recv = torch.from_numpy(rs.randint(0, 256, W * lay.nbytes).astype(np.uint8))
        v = lay.unpack(recv)
        v["done"].copy_(torch.from_numpy(rs.rand(W, n) < 0.2))
        fresh = t in (0, K + 1)
        done = v["done"].reshape(-1)
        for j, k in enumerate(keys):
            src = "allo" if (preproc == "LoRes4A" or (preproc == "LoResStack" and k == "allo")) else "ego"
            planar = v[src].reshape(W * n, 96, 96, 3).permute(0, 3, 1, 2)
            p = t % K
            for g in range(W * n):
                frames = range(4) if (fresh or bool(done[g])) else range(1)
                for d in frames:
                    f = (p + K - d) % K
                    rv[j, g, f] = planar[g]
                    if f < 3:
                        rv[j, g, K + f] = planar[g]
        want = {k: torch.zeros((W * n, 96, 96, 12), dtype=torch.uint8) for k in keys}
        orc(recv, want, t, fresh)
        s0 = (t + K - 3) % K
        for j, k in enumerate(keys):
            view = mdist.window_view(ring, j, W * n, s0, K)
            assert view.stride() == ((K + 3) * 27648, 96, 1, 9216)
            assert torch.equal(view, want[k]), (t, k)
    assert mdist.window_ring_bytes("LoRes4E", 8, 10) == 80 * 11 * 27648
    assert mdist.window_ring_bytes("LoResStack", 8, 10) == 2 * 80 * 11 * 27648
    assert not mdist.uses_window("LoRes3EA") and mdist.uses_window("LoResCHW4A")


def test_bench_launches_ranks_itself():
    """bench.py --gpus 2 without WORLD_SIZE re-runs itself under torch.distributed.run with 2 ranks
    (before any GPU call); --dry-run swaps the GPU work for a gloo all-reduce, so rank 0 sees 2 ranks and
    the N > 1 gather default is on."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                          "--cpu-steps", "60", "--cpu-workers", "2"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["ranks_seen"] == 2 and line["n_gpus"] == 2 and line["gather"] is True
    # the N > 1 line carries the CPU baseline, measured in the launcher parent before the ranks start
    cpu = line["cpu_baseline"]
    assert cpu["measured_in"] == "launcher parent" and cpu["cores"] == 2 and cpu["kind"] == "port"
    assert cpu["value"] > 0 and cpu["one_core_env_steps_s"] > 0


def test_bench_byte_models():
    """Per-kernel algorithmic bytes: render = observations + frame ring (frames-only mode: 2 frames), restack =
    per stacked view 1 frame read + (1 + 3/K) written with the window ring (materialised: 1 + 3 frames read,
    1 + 4 frames written); the whole-step fraction from ms_per_step."""
    sys.path.insert(0, ROOT)
    import bench
    fr = 96 * 96 * 3
    assert bench.render_bytes("LoRes4E") == 165888 + 4 * fr
    assert bench.render_bytes("LoResStack") == 221184 + 8 * fr
    assert bench.render_bytes("LoRes4E", frames_only=True) == 2 * fr
    assert bench.restack_bytes("LoResStack", window=False) == 2 * 9 * fr
    assert bench.restack_bytes("LoResStack") == round(2 * (1 + 1 + 3 / 8) * fr)
    assert bench.restack_bytes("LoRes3EA") == 9 * fr + fr   # not a window of one ring: materialised
    # roofline.step_frac: the round-4 MoveToRegion line, 4096 envs at 1.3766 ms per step -> 0.0625
    ach, frac = bench.step_fraction("LoRes4E", 4096, 1.3766)
    assert abs(ach - 499.7) < 0.5 and round(frac, 4) == 0.0625
    # roofline.frac: SURVEY 8(d) bytes per env-step (obs + ~2 KB state) for whichever kernel dominates
    assert bench.survey_bytes("LoRes4E") == 167936 and bench.survey_bytes("LoResStack") == 223232
    # MoveToRegion render at 4096 envs, rocprofv3 average 1.0484 ms (profiles/r03_final): 656 GB/s = 0.082
    r = bench.kernel_record("render_kernel", 1.0484, "LoRes4E", 4096,
                            {"bytes_per_launch": 1.272e9, "valu_issue_frac": 0.32, "wait_any_frac": 0.64})
    assert abs(r["achieved_gbs"] - 656.1) < 0.5 and 0.082 <= r["hbm_frac"] <= 0.083
    assert abs(r["traffic_ratio"] - 1.85) < 0.01            # 1.272 GB over 167 936 B x 4096
    assert r["kernel_bytes_per_env_step"] == 165888 + 4 * fr  # the ring-inclusive figure, kept apart
    # the step kernel's traffic ratio is over its 8(d) state bytes: ClusterColour's 4.37 GB at 8192 envs ~ 260x
    s = bench.kernel_record("step_kernel", 3.82, "LoResStack", 8192, {"bytes_per_launch": 4.367e9})
    assert s["bytes_per_env_step"] == 223232 and s["traffic_ratio_basis_bytes_per_env_step"] == 2048
    assert 255 < s["traffic_ratio"] < 265
    assert bench.kernel_record("step_kernel", 1.0, "LoRes4E", 64, None)["traffic_ratio"] is None
    # the step kernel's design bytes: its HBM <-> LDS state transfer at the form's slot caps (csrc/mg_stepk.h),
    # 209 B per live arbiter slot each way; the traffic ratio is then over those
    assert bench.step_state_bytes(5, (6, 5, 10, 20), 0) == 2509      # MoveToRegion, quad form
    assert bench.step_state_bytes(6, (7, 6, 12, 32), 0) == 3011      # MoveToCorner
    assert bench.step_state_bytes(4, (14, 53, 26, 48), 0) == 6939    # the many-block scenes, cooperative form
    assert bench.step_state_bytes(4, (14, 53, 26, 48), 2.5) == 6939 + round(2.5 * 2 * 209)
    s = bench.kernel_record("step_kernel", 2.7, "LoResStack", 8192, {"bytes_per_launch": 98e6}, step_bytes=6939)
    assert s["kernel_bytes_per_env_step"] == 6939 and s["traffic_ratio_basis_bytes_per_env_step"] == 6939
    assert abs(s["traffic_ratio"] - 98e6 / (6939 * 8192)) < 0.01
    os.environ["MG_STEP_VARIANT"] = "4"
    try:
        assert bench.env_overrides().get("MG_STEP_VARIANT") == "4"
    finally:
        del os.environ["MG_STEP_VARIANT"]


GATHER_CASES = [("MoveToRegion-Demo-LoRes4E-v0", "frames"), ("MoveToRegion-Demo-LoRes4E-v0", "stacked"),
                ("ClusterColour-Demo-LoResStack-v0", "frames"), ("ClusterColour-Demo-LoResStack-v0", "stacked"),
                ("MoveToCorner-Demo-LoRes3EA-v0", "frames"), ("MoveToCorner-Demo-LoRes4A-v0", "frames"),
                ("MoveToRegion-Demo-LoResCHW4E-v0", "frames"), ("PickAndPlace-Demo-LoRes4E-v0", "frames")]


@pytest.mark.parametrize("name,mode", GATHER_CASES)
def test_two_rank_gloo_packed_gather_pipeline(tmp_path, name, mode):
    """ShardedVecEnv(gather=True) with world_size 2 on CPU tensors, episodes of 5 steps (max_episode_steps)
    so the 12 steps cross two auto-resets of every env: each rank's step outputs are written into views of
    one packed buffer, one all_gather_into_tensor per step, two buffer sets alternating (each step's
    handle read after the next step was launched).  gather_mode 'frames' gathers only the current frames
    and rebuilds the stacks on the receiver (here with the oracle's restacker; the GPU kernel mg_restack
    is checked against the simulator in tests/test_gpu_parity.py).  Every step's [W, n, ...] results --
    observations (incl. rebuilt stacks across the resets), reward, done, eval_score, PickAndPlace's
    target -- equal one process running all W * n envs.  'frames' moves 3x (LoRes4E) / 4x (LoResStack)
    fewer bytes per rank-step than 'stacked'."""
    out = str(tmp_path / "full.npz")
    script = tmp_path / "worker.py"
    L, steps = 5, 12
    script.write_text(PACKED_WORKER.format(root=ROOT, out=out, name=name, mode=mode, L=L, steps=steps))
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
    W, n = 2, 2
    acts = np.random.RandomState(5).randint(0, 18, (steps, W * n))
    envs = [po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, L, seed=1000 + i) for i in range(W * n)]
    shapes = mg_envs._obs_shapes(spec)
    chw = registry.PREPROCESSORS[spec.preproc].get("channels_first", False)

    def check(t, i, o, res=None, target=None):
        off = 0
        for k, s in shapes.items():
            m = int(np.prod(s))
            assert np.array_equal(got[k][t + 1, i // n, i % n], o[off:off + m].reshape(s)), (t, k, i)
            off += m
        if res is not None:
            r, d, sc = res
            assert got["reward"][t, i // n, i % n] == np.float32(r) and bool(got["done"][t, i // n, i % n]) == d
            assert got["score"][t, i // n, i % n] == sc
        if target is not None:
            assert np.array_equal(got["target"][t, i // n, i % n], target), (t, i)
            assert np.array_equal(got["target_position"][t + 1, i // n, i % n], target[2:4].astype(np.float32))

    for i, e in enumerate(envs):
        check(-1, i, e.reset())
    crossed = 0
    for t in range(steps):
        for i, e in enumerate(envs):
            o, r, d, sc = e.step(int(acts[t, i]))
            if d:
                o = e.reset()
                crossed += 1
            check(t, i, o, (r, d, sc), e.target() if spec.task == "PickAndPlace" else None)
    assert crossed == 2 * W * n
    if chw:
        assert got["past_obs"].shape[-3:] == (12, 96, 96)
    assert int(got["nbytes"]) % 256 == 0
    if mode == "frames":
        ratio = int(got["stacked_nbytes"]) / int(got["nbytes"])
        assert ratio > (3.9 if spec.preproc == "LoResStack" else 2.9), ratio


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


def test_latexify_results_matches_reference():
    """evaluation.py:101-154 latexify_results: the text the reference's own function produced
    (tests/golden/ref_latex.json, make_ref_fixtures.py) for one- and multi-algorithm frames and a custom
    id column, and its error on a duplicated (run, env) record."""
    import json
    import pandas as pd
    import pytest
    from magical_amd import evaluation
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_latex.json")))
    for case in ref["cases"]:
        frame = pd.DataFrame.from_records(case["records"])
        assert evaluation.latexify_results(frame, id_column=case["id_column"]) == case["latex"]
    with pytest.raises(ValueError) as ei:
        evaluation.latexify_results(pd.DataFrame.from_records(ref["duplicate"]["records"]))
    assert str(ei.value) == ref["duplicate"]["error"]


def test_small_render_class_holds_every_robot_scene():
    """The small render class (RG_SMALL, mg_render.h) has no successor in the class chain: an (env, view) it cannot
    hold is an env error.  Its caps must cover every MoveToRegion / MoveToCorner scene the library can build: robot +
    arena + goal, or robot + arena + a block of any shape type (geoms, vertices, solid outline edges, entities,
    outline-mask bits)."""
    from magical_amd import tables as T
    src = open(os.path.join(ROOT, "magical-1_amd", "csrc", "mg_render.h")).read()
    caps = re.search(r"#define RG_SMALL ([^\n]+)", src).group(1).split(",")
    maxg, maxvert, _maxdash, _maxbin, maxsedge, maxe = (int(x) for x in caps[:6])
    band, mbits = int(caps[7]), int(caps[8])
    assert band == 16 and mbits >= 3
    L = T.build_library()

    def size(r0, n):
        polys = [L.rpoly[i] for i in range(r0, r0 + n)]
        return (n, sum(p.npts for p in polys), sum(p.npts for p in polys if p.outline == T.OUTLINE_SOLID))

    base = [size(L.robot_rpoly0, L.robot_nrpoly), size(L.arena_rpoly0, L.arena_nrpoly)]
    scenes = [base + [size(L.goal_rpoly0, L.goal_nrpoly)]]                                       # MoveToRegion
    scenes += [base + [size(L.block_rpoly0[t], L.block_nrpoly[t])] for t in range(T.NUM_SHAPE_TYPES)]  # MoveToCorner
    for sc in scenes:
        g, v, se = (sum(x[k] for x in sc) for k in range(3))
        assert g <= maxg and v <= maxvert and se <= maxsedge and len(sc) <= min(maxe, mbits), (sc, caps)
    assert max(sum(x[0] for x in sc) for sc in scenes) == 26 and max(sum(x[1] for x in sc) for sc in scenes) == 636


def test_pipeline_default_chunks():
    """bench.py --chunks auto: MoveToRegion pipelines 3 chunks at >= 4096 envs, the robot scenes 2 at >= 2048
    (2 at most under the multi-GPU exchange: bench.py), every other scene runs 1."""
    from magical_amd import pipeline
    assert pipeline.default_chunks(registry.lookup("MoveToRegion-Demo-LoRes4E-v0"), 4096) == 3
    assert pipeline.default_chunks(registry.lookup("MoveToRegion-Demo-LoRes4E-v0"), 2048) == 2
    assert pipeline.default_chunks(registry.lookup("MoveToCorner-Demo-LoRes4E-v0"), 4096) == 2
    assert pipeline.default_chunks(registry.lookup("MoveToRegion-Demo-LoRes4E-v0"), 64) == 1
    assert pipeline.default_chunks(registry.lookup("ClusterColour-Demo-LoResStack-v0"), 8192) == 1
    assert pipeline.default_chunks(registry.lookup("MatchRegions-TestAll-LoRes4E-v0"), 8192) == 1


def test_gathered_window_views_raise_when_stale():
    """a step's window-ring stacks are rewritten by the next exchange, so results() of an older
    GatheredStep raises once its shard has issued a later step_async / reset_async (materialised stacks and
    frames-only results are not affected)."""
    class Owner:
        t = 1
    h = mdist.GatheredStep(None, None, {"past_obs": None}, owner=Owner, step=0, windowed=True)
    Owner.t = 2
    with pytest.raises(RuntimeError, match="window-ring"):
        h.results()
    h2 = mdist.GatheredStep(None, None, {}, owner=Owner, step=0, windowed=False)
    with pytest.raises(AttributeError):   # no guard: it goes on to unpack (None layout here)
        h2.results()
