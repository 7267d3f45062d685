"""ctypes binding for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline; the product path
(magical-1_amd) never touches it.  See oracle/oracle.h for what the oracle
restates and how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MG_ORACLE_TRIG=libm: the measurement build with this image's libm sin/cos (tools/libm_vs_cr.py)
_LIBM = os.environ.get("MG_ORACLE_TRIG") == "libm"
LIB_PATH = os.path.join(HERE, "_build", "libmg_oracle_libm.so" if _LIBM else "libmg_oracle.so")

TASKS = {"MoveToRegion": 0, "MoveToCorner": 1, "ClusterColour": 2, "ClusterShape": 3, "MatchRegions": 4,
         "MakeLine": 5, "FindDupe": 6, "FixColour": 7, "PickAndPlace": 8}
PREPROCS = {None: 0, "LoRes4E": 1, "LoResStack": 2, "LoRes3EA": 3, "LoRes4A": 4, "LoResCHW4E": 5, "LoResCHW4A": 5}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE] + (["libm"] if _LIBM else []), check=True)


def lib():
    global _lib
    if _lib is None:
        build()  # make: no-op when up to date
        L = ctypes.CDLL(LIB_PATH)
        d, i, u32, vp = ctypes.c_double, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p
        L.o_crsin.restype = d; L.o_crsin.argtypes = [d]
        L.o_crcos.restype = d; L.o_crcos.argtypes = [d]
        L.o_crtan.restype = d; L.o_crtan.argtypes = [d]
        L.oenv_create.restype = vp; L.oenv_create.argtypes = [i, i, i, i, u32]
        L.oenv_destroy.argtypes = [vp]
        L.oenv_seed.argtypes = [vp, u32]
        L.oenv_obs_bytes.restype = i; L.oenv_obs_bytes.argtypes = [vp]
        L.oenv_reset.restype = i; L.oenv_reset.argtypes = [vp, vp]
        L.oenv_step.restype = i
        L.oenv_step.argtypes = [vp, i, vp, ctypes.POINTER(d), ctypes.POINTER(i), ctypes.POINTER(d)]
        L.oenv_render_full.argtypes = [vp, vp, vp]
        L.oenv_get_bodies.restype = i; L.oenv_get_bodies.argtypes = [vp, vp, i]
        L.oenv_num_arbiters.restype = i; L.oenv_num_arbiters.argtypes = [vp]
        L.oenv_get_arbiters.restype = i; L.oenv_get_arbiters.argtypes = [vp, vp, vp, i]
        L.oenv_placement_retries.restype = i; L.oenv_placement_retries.argtypes = [vp]
        L.oenv_set_max_tries.argtypes = [vp, i]
        L.oenv_get_entities.restype = i; L.oenv_get_entities.argtypes = [vp, vp, vp, vp, vp]
        L.o_mt_seed.argtypes = [vp, u32]
        L.o_mt_next32.restype = u32; L.o_mt_next32.argtypes = [vp]
        L.o_mt_double.restype = d; L.o_mt_double.argtypes = [vp]
        L.o_mt_uniform.restype = d; L.o_mt_uniform.argtypes = [vp, d, d]
        L.o_mt_randint.restype = ctypes.c_int64; L.o_mt_randint.argtypes = [vp, ctypes.c_int64, ctypes.c_int64]
        L.o_longest_line.restype = i; L.o_longest_line.argtypes = [vp, vp, i, d, d]
        L.oenv_set_body_pose.argtypes = [vp, i, d, d, d]
        L.oenv_get_target.argtypes = [vp, vp]
        L.o_mt_interval.restype = ctypes.c_uint64; L.o_mt_interval.argtypes = [vp, ctypes.c_uint64]
        L.o_convex_hull.restype = i; L.o_convex_hull.argtypes = [i, vp, vp, vp, d]
        L.o_moment_for_poly.restype = d
        L.o_star_decomposition.restype = i; L.o_star_decomposition.argtypes = [d, d, vp, vp, i]
        L.o_finger_verts.argtypes = [d, d, d, i, vp, vp]
        L.o_transform_trs.argtypes = [d, d, d, d, d, vp]
        L.o_mat3_mul.argtypes = [vp, vp, vp]
        L.o_allo_view.argtypes = [vp]
        L.o_ego_view.argtypes = [d, d, d, vp]
        L.oenv_get_phys_vars.argtypes = [vp, vp]
        L.o_palette.argtypes = [vp]
        L.o_downsample.argtypes = [vp, vp]
        L.osc_entity.argtypes = [vp, i, vp]
        L.osc_get_pose.argtypes = [vp, i, i, vp]
        L.oenv_get_rng.argtypes = [vp, vp, vp]
        _lib = L
    return _lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class MT:
    """numpy-legacy MT19937 restatement (oracle/rng.c)."""

    def __init__(self, seed):
        self.buf = np.zeros(625 * 4 + 16, dtype=np.uint8)
        lib().o_mt_seed(ptr(self.buf), seed)

    def next32(self):
        return lib().o_mt_next32(ptr(self.buf))

    def double(self):
        return lib().o_mt_double(ptr(self.buf))

    def uniform(self, lo, hi):
        return lib().o_mt_uniform(ptr(self.buf), lo, hi)

    def randint(self, lo, hi):
        return lib().o_mt_randint(ptr(self.buf), lo, hi)

    def interval(self, mx):
        return lib().o_mt_interval(ptr(self.buf), mx)


def star_parts(out_rad, in_rad):
    out = np.zeros((64, 2))
    counts = np.zeros(8, dtype=np.int32)
    n = lib().o_star_decomposition(out_rad, in_rad, ptr(out), ptr(counts), 8)
    parts, off = [], 0
    for k in range(n):
        parts.append(out[off:off + counts[k]].copy())
        off += counts[k]
    return parts


class PlacementError(RuntimeError):
    pass


class OracleEnv:
    """One reference env (single instance, CPU)."""

    def __init__(self, task, rand_flags, preproc, max_steps, seed=0):
        self.L = lib()
        self.h = self.L.oenv_create(TASKS[task] if isinstance(task, str) else task, rand_flags,
                                    PREPROCS[preproc] if not isinstance(preproc, int) else preproc,
                                    max_steps, seed)
        self.nbytes = self.L.oenv_obs_bytes(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oenv_destroy(self.h)
            self.h = None

    def seed(self, s):
        self.L.oenv_seed(self.h, s)

    def reset(self):
        obs = np.zeros(self.nbytes, dtype=np.uint8)
        rc = self.L.oenv_reset(self.h, ptr(obs))
        if rc == -2:
            raise PlacementError("could not place entities after 10 retries (geom.py:335-336)")
        if rc != 0:
            raise RuntimeError("oracle table overflow")
        return obs

    def step(self, action):
        obs = np.zeros(self.nbytes, dtype=np.uint8)
        r, dn, sc = ctypes.c_double(), ctypes.c_int(), ctypes.c_double()
        rc = self.L.oenv_step(self.h, int(action), ptr(obs), ctypes.byref(r), ctypes.byref(dn), ctypes.byref(sc))
        if rc != 0:
            raise RuntimeError("oracle table overflow")
        return obs, r.value, bool(dn.value), sc.value

    def render_full(self):
        a = np.zeros((384, 384, 3), dtype=np.uint8)
        g = np.zeros((384, 384, 3), dtype=np.uint8)
        self.L.oenv_render_full(self.h, ptr(a), ptr(g))
        return a, g

    def bodies(self):
        out = np.zeros((32, 6))
        n = self.L.oenv_get_bodies(self.h, ptr(out), 32)
        return out[:n].copy()

    def set_body_pose(self, body, x, y, angle):
        self.L.oenv_set_body_pose(self.h, int(body), float(x), float(y), float(angle))

    def target(self):
        """PickAndPlace extras: (target_type, target_colour, target_position x, y)"""
        out = np.zeros(4)
        self.L.oenv_get_target(self.h, ptr(out))
        return out

    def phys_vars(self):
        out = np.zeros(5)
        self.L.oenv_get_phys_vars(self.h, ptr(out))
        return out

    def set_max_tries(self, n):
        """pm_randomise_pose max_tries (geom.py:198, 10000); lowered by tests to force layout retries"""
        self.L.oenv_set_max_tries(self.h, int(n))

    def placement_retries(self):
        """failed whole-layout retries of pm_randomise_all_poses in the last reset (geom.py:295-341)"""
        return self.L.oenv_placement_retries(self.h)

    def num_arbiters(self):
        return self.L.oenv_num_arbiters(self.h)

    def arbiters(self):
        """the solved arbiters in active order: f64 [n, 28] (slot, state, count, body a, body b, n.x, n.y, u,
        2 x (r1, r2, jnAcc, jtAcc, nMass, tMass, bias, jBias)) and u64 [n, 2] contact hashes (mg_get_arbiters)"""
        out = np.zeros((64, 28))
        hs = np.zeros((64, 2), dtype=np.uint64)
        n = self.L.oenv_get_arbiters(self.h, ptr(out), ptr(hs), 64)
        return out[:n].copy(), hs[:n].copy()

    def entity_poses(self):
        """per entity after the arena, in add order: (x, y, angle) of each of its bodies (the goal: its static
        body's position, angle 0) -- tests/golden/ref_resets.json's layout"""
        n = len(self.entities()[0])
        out = []
        for ent in range(1, n):
            d = np.zeros(5, dtype=np.int32)
            self.L.osc_entity(self.h, ent, ptr(d))
            poses = []
            for k in range(int(d[2])):
                p = np.zeros(3)
                self.L.osc_get_pose(self.h, ent, k, ptr(p))
                poses.append(p.tolist())
            out.append(poses)
        return out

    def rng_state(self):
        """(key u32[624], pos) of the env's MT19937 -- numpy RandomState.get_state()[1:3]"""
        key = np.zeros(624, dtype=np.uint32)
        pos = ctypes.c_int()
        self.L.oenv_get_rng(self.h, ptr(key), ctypes.byref(pos))
        return key, pos.value

    def entities(self):
        k = np.zeros(32, dtype=np.int32)
        t = np.zeros(32, dtype=np.int32)
        c = np.zeros(32, dtype=np.int32)
        p = np.zeros((32, 4))
        n = self.L.oenv_get_entities(self.h, ptr(k), ptr(t), ptr(c), ptr(p))
        return k[:n].copy(), t[:n].copy(), c[:n].copy(), p[:n].copy()


def palette():
    out = np.zeros((5, 4, 3), dtype=np.uint8)
    lib().o_palette(ptr(out))
    return out


def downsample(frame):
    frame = np.ascontiguousarray(frame, dtype=np.uint8)
    assert frame.shape == (384, 384, 3)
    out = np.zeros((96, 96, 3), dtype=np.uint8)
    lib().o_downsample(ptr(frame), ptr(out))
    return out


class OracleRestacker:
    """Reference frame-stack rule over an all-gathered frames-only batch (TEST INFRASTRUCTURE: the CPU
    counterpart of mg_restack that the gloo tests hand to magical_amd.dist.ShardedVecEnv).

    Restates benchmarks/__init__.py:51-147 per env: EagerDictFrameStack / FlattenFrameStack keep a deque of
    the last `depth` frames, filled with the reset frame at reset (:75-82, :139-147); under SB3's
    DummyVecEnv auto-reset the frame returned with done is the next episode's reset frame.  Stacks are
    the frames oldest..newest concatenated on the channel axis; LoRes3EA puts the current allo frame in
    front of the last 3 ego frames (allo depth 1, ego depth 3)."""

    def __init__(self, layout, preproc):
        self.layout, self.pp = layout, preproc
        self.deq = {}

    def __call__(self, recv, outs, step, all_fresh):
        v = self.layout.unpack(recv)
        W, n = v["done"].shape
        done = v["done"].reshape(-1).numpy().astype(bool)
        cur = {k: v[k].reshape(W * n, 96, 96, 3).numpy() for k in ("allo", "ego")}
        for k, c in cur.items():
            if all_fresh or k not in self.deq:
                d = np.repeat(c[:, None], 4, axis=1)
            else:
                d = np.concatenate([self.deq[k][:, 1:], c[:, None]], axis=1)
                d[done] = c[done][:, None]
            self.deq[k] = d
        cat = lambda frames: np.concatenate(frames, axis=-1)  # noqa: E731
        res = {}
        if self.pp == "LoResStack":
            res["allo"] = cat([self.deq["allo"][:, k] for k in range(4)])
            res["ego"] = cat([self.deq["ego"][:, k] for k in range(4)])
        elif self.pp == "LoRes4A":
            res["past_obs"] = cat([self.deq["allo"][:, k] for k in range(4)])
        elif self.pp == "LoRes3EA":
            res["past_obs"] = cat([cur["allo"]] + [self.deq["ego"][:, k] for k in range(1, 4)])
        else:   # LoRes4E, LoResCHW4E, LoResCHW4A
            res["past_obs"] = cat([self.deq["ego"][:, k] for k in range(4)])
        import torch
        for k, a in res.items():
            outs[k].copy_(torch.from_numpy(a))


def _pure():
    L = lib()
    if not getattr(L, "_pure_set", False):
        d, i, vp = ctypes.c_double, ctypes.c_int, ctypes.c_void_p
        L.o_score_move_to_corner.restype = d; L.o_score_move_to_corner.argtypes = [d, d]
        L.o_shaped_move_to_corner.restype = d; L.o_shaped_move_to_corner.argtypes = [d, d, d, d]
        L.o_cluster_score.restype = d; L.o_cluster_score.argtypes = [i, vp, vp, vp]
        L.o_action_decode.restype = None; L.o_action_decode.argtypes = [i, vp]
        L._pure_set = True
    return L


def score_move_to_corner(rx, ry):
    return _pure().o_score_move_to_corner(float(rx), float(ry))


def shaped_move_to_corner(rx, ry, sx, sy):
    return _pure().o_shaped_move_to_corner(float(rx), float(ry), float(sx), float(sy))


def cluster_score(vals, xy):
    """vals: per block the rank of its characteristic value among the values present; xy: [n, 2]"""
    v = np.ascontiguousarray(vals, dtype=np.int32)
    xy = np.asarray(xy, dtype=np.float64)
    x, y = np.ascontiguousarray(xy[:, 0]), np.ascontiguousarray(xy[:, 1])
    return _pure().o_cluster_score(len(v), ptr(v), ptr(x), ptr(y))


def action_decode(action):
    out = np.zeros(3)
    _pure().o_action_decode(int(action), ptr(out))
    return out


def stack_lores(lo, starts, preproc, channels_first=False):
    """Per-frame LoRes observation dicts from per-frame downsampled (allo, ego) frames by the reference
    wrappers' rules (benchmarks/__init__.py:51-147,232-307): frame f's stacks reach back to the first frame
    of its episode, starts[f] (the reset frame fills every deque slot)."""
    import collections
    out = []
    for f in range(len(lo)):
        back = lambda k: max(f - k, starts[f])  # noqa: E731
        if preproc == "LoResStack":
            out.append(collections.OrderedDict(
                (k, np.concatenate([lo[back(j)][v] for j in (3, 2, 1, 0)], axis=-1)) for v, k in enumerate(("allo", "ego"))))
            continue
        if preproc == "LoRes3EA":
            frames = [lo[f][0]] + [lo[back(j)][1] for j in (2, 1, 0)]
        elif preproc == "LoRes4A":
            frames = [lo[back(j)][0] for j in (3, 2, 1, 0)]
        else:
            frames = [lo[back(j)][1] for j in (3, 2, 1, 0)]
        d = collections.OrderedDict([("allo", lo[f][0]), ("ego", lo[f][1]), ("past_obs", np.concatenate(frames, -1))])
        if channels_first:
            d = collections.OrderedDict((k, np.moveaxis(v, -1, 0)) for k, v in d.items())
        out.append(d)
    return out
