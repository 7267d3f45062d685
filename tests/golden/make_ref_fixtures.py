"""Golden fixtures computed by EXECUTING the reference's own pure numpy/math code
(run in the dev container, where /root/reference exists; the GPU box only reads
the JSON output).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ref_fixtures.py

The reference package cannot be imported here (pygame / pymunk / gym / cv2 are
absent: ModuleNotFoundError, not a permission denial), so the functions below are
taken out of the reference source files with `ast` and executed in a namespace
that supplies numpy, math, itertools and inert stand-ins for the two pygame-bound
names they mention but do not use for arithmetic (`Poly` records its points,
`pygame.Surface` is never drawn on).  Nothing of the reference's source text is
written out: the JSON files hold inputs and the reference's outputs only.

  * ref_render.json  -- render.py:13-35 (make_rect, make_circle), :37-124
                        (Transform, incl. rigid_transform), :127-138 (Stack),
                        :290-304 (ego_cam_matrix), :307-371 (Viewer.set_bounds,
                        Viewer.set_cam_follow) with base_env.py:309-322's camera
                        arguments and style.py's ARENA_ZOOM_OUT; the libm sin/cos
                        the reference's math.sin/cos returned are stored beside
                        each case.
  * ref_outline.json -- render.py:202-287 (Poly._render, Poly.draw_outline): the
                        pygame.draw.polygon / lines / line calls the reference makes
                        (points, width) for solid and dashed outlines, recorded by a
                        stand-in pygame.draw on pixel-space polygons (goal
                        rectangles through allo and ego views, random quads, exact
                        axis-aligned and .5-tie edges).
  * ref_make_line.json -- benchmarks/make_line.py:31-72 (longest_line) on random
                        point sets and on near-collinear sets that sit at the
                        scorer's inlier / separation thresholds.
  * ref_wrappers.json -- benchmarks/__init__.py:31-307: the preprocessor entry
                        points of every LoRes name (lores_ea_entry_point /
                        lores_stack_entry_point with FlattenFrameStack /
                        EagerDictFrameStack, ResizeDictObservation, ChannelsFirst),
                        run on synthetic 384^2 frame sequences with resets; gym's
                        Wrapper / Box / Dict, SB3's is_image_space and cv2.resize
                        are stand-ins (cv2 INTER_AREA 4x = the oracle's
                        o_downsample, pinned separately).  Stored: observation
                        keys, shapes, dtypes and a sha256 per value and event.
  * ref_latex.json    -- evaluation.py:101-154 (latexify_results) on synthetic do_eval() frames.
  * ref_scorers.json  -- cluster.py:166-216 (BaseClusterEnv.score_on_end_of_traj)
                        on random, clustered and near-threshold block layouts;
                        move_to_corner.py:67-100 (score_on_end_of_traj and
                        debug_shaped_reward) on random robot / block positions.
  * ref_actions.json  -- entities.py:148-190 (RobotAction, ACTION_NUMS_FLAGS_NAMES)
                        and Robot.set_action (:435-453) for every action id.
"""
import ast
import collections
import enum
import functools
import hashlib
import importlib.util
import itertools
import json
import math
import os
import sys
import types
import typing

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/magical"
sys.dont_write_bytecode = True


def _node_name(n):
    if isinstance(n, (ast.FunctionDef, ast.ClassDef)):
        return n.name
    if isinstance(n, ast.Assign) and len(n.targets) == 1 and isinstance(n.targets[0], ast.Name):
        return n.targets[0].id
    return None


def _extract(path, names, namespace):
    """Execute the top-level definitions / assignments `names` of the reference file `path` in `namespace`
    (in file order)."""
    tree = ast.parse(open(path).read(), filename=path)
    nodes = [n for n in tree.body if _node_name(n) in names]
    missing = set(names) - {_node_name(n) for n in nodes}
    assert not missing, missing
    mod = ast.Module(body=nodes, type_ignores=[])
    exec(compile(mod, path, "exec"), namespace)
    return namespace


class _Poly:
    """stand-in for render.Poly: keeps the points and the outline flag"""

    def __init__(self, points, outline):
        self.points, self.outline, self.dashed = [tuple(map(float, p)) for p in points], outline, False


class _Geom:
    @staticmethod
    def convert_color(*rgb):
        return rgb


def _render_namespace():
    ns = {"__name__": "ref_render", "np": np, "math": math, "dataclasses": __import__("dataclasses"),
          "abc": __import__("abc"), "List": typing.List, "Tuple": typing.Tuple, "Union": typing.Union,
          "Poly": _Poly, "Geom": _Geom,
          "pygame": types.SimpleNamespace(Surface=lambda *a, **k: None)}
    ns["CoordType"] = typing.Union[typing.Tuple[float, float], typing.List[float], np.ndarray]
    ns["ArrayLike"] = typing.Union[typing.List[ns["CoordType"]], typing.Tuple[ns["CoordType"]]]
    return _extract(os.path.join(REF, "render.py"),
                    ["make_rect", "make_circle", "make_square", "Transform", "Stack", "ego_cam_matrix", "Viewer"], ns)


def _zoom_out():
    spec = importlib.util.spec_from_file_location("ref_style", os.path.join(REF, "style.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.ARENA_ZOOM_OUT


def _m(a):
    return np.asarray(a, dtype=np.float64).ravel().tolist()


def ref_render():
    R = _render_namespace()
    Z = _zoom_out()
    rs = np.random.RandomState(2024)
    out = {"arena_zoom_out": Z, "res": 384}
    # base_env.py:318-322: the arena is [-1, 1]^2
    v = R["Viewer"](384, 384)
    v.set_bounds(left=-1 * Z, right=1 * Z, bottom=-1 * Z, top=1 * Z)
    out["allo_view"] = _m(v.transform.matrix)
    out["pygame_transform"] = _m(v.pygame_transform.matrix)
    ego = []
    angles = list(rs.uniform(-7, 7, 300)) + [0.0, -2.13, 0.83693, -1.2 * math.pi, 0.55 * math.pi, 3.83, 0.347,
                                             0.718, math.pi, -math.pi, 1e-9, -3.7e-5]
    for a in angles:
        x, y = rs.uniform(-1.1, 1.1, 2)
        v.set_cam_follow(source_xy_world=(x, y), target_xy_01=(0.5, 0.15), viewport_hw_world=(2 * Z, 2 * Z),
                         rotation=float(a))
        ego.append({"x": float(x), "y": float(y), "a": float(a), "m": _m(v.transform.matrix),
                    "libm_sin": math.sin(-float(a)), "libm_cos": math.cos(-float(a))})
    out["ego_view"] = ego
    trs = []
    for _ in range(200):
        t = rs.uniform(-400, 400, 2)
        r = float(rs.uniform(-7, 7))
        s = rs.uniform(-200, 200, 2)
        tr = R["Transform"](translation=(float(t[0]), float(t[1])), rotation=r, scale=(float(s[0]), float(s[1])))
        trs.append({"t": _m(t), "r": r, "s": _m(s), "m": _m(tr.matrix), "libm_sin": math.sin(r),
                    "libm_cos": math.cos(r)})
    out["transform"] = trs
    stacks = []
    for _ in range(60):
        st = R["Stack"]()
        mats = []
        for _k in range(int(rs.randint(1, 5))):
            m = rs.uniform(-3, 3, (3, 3))
            m[2] = (0.0, 0.0, 1.0)
            st.push(R["Transform"].from_matrix(m))
            mats.append(_m(m))
        pts = rs.uniform(-1.5, 1.5, (6, 2))
        stacks.append({"mats": mats, "top": _m(st.stack[-1]), "pts": _m(pts),
                       "pts_out": _m(st.apply_current_matrix(pts))})
    out["stack"] = stacks
    # render.py polygons used by entities.py: make_circle(r, 100) for the robot body / eye / pupil and the
    # circle block, make_rect for the arena and goal regions, make_square for the square block
    circles = []
    for radius in (0.2, 0.2 * 0.2, 0.12 * 0.2, 0.2 * 0.6):
        p = R["make_circle"](radius, 100, True)
        circles.append({"radius": radius, "res": 100, "pts": [list(q) for q in p.points],
                        "libm": [[math.cos(2 * math.pi * i / 100), math.sin(2 * math.pi * i / 100)]
                                 for i in range(100)]})
    out["circle"] = circles
    rects = []
    for w, h in [(2.0, 2.0), (0.75, 0.76), (0.6, 0.7), (0.72, 0.67), (0.427, 0.468)] + \
            [tuple(rs.uniform(0.4, 0.8, 2)) for _ in range(8)]:
        rects.append({"w": float(w), "h": float(h), "pts": [list(q) for q in R["make_rect"](float(w), float(h), True).points]})
    out["rect"] = rects
    side = math.sqrt(math.pi) * 0.2 * 0.6
    out["square"] = {"side": side, "pts": [list(q) for q in R["make_square"](side, True).points]}
    return out


class _Recorder:
    """stand-in for pygame.draw: records each call's points and width"""

    def __init__(self):
        self.calls = []

    def polygon(self, surface, color, points, width=0):
        self.calls.append(["polygon", [[float(c) for c in p] for p in points], width])

    def lines(self, surface, color, closed, points, width=1):
        self.calls.append(["lines", [[float(c) for c in p] for p in points], width, bool(closed)])

    def line(self, surface, color, start, end, width=1):
        self.calls.append(["line", [[float(c) for c in start], [float(c) for c in end]], width])

    def circle(self, surface, color, pos, radius, width=0):
        self.calls.append(["circle", [[float(c) for c in pos]], radius])


def ref_outline():
    rec = _Recorder()

    class _GeomBase:
        def __init__(self):
            self._color = (1, 2, 3, 1)
            self._outline_color = (4, 5, 6, 1)

    ns = {"__name__": "ref_outline", "np": np, "math": math, "abc": __import__("abc"), "Geom": _GeomBase,
          "pygame": types.SimpleNamespace(Surface=object, draw=rec)}
    ns["ArrayLike"] = typing.Any
    _extract(os.path.join(REF, "render.py"), ["Poly"], ns)
    Poly = ns["Poly"]
    R = _render_namespace()
    Z = _zoom_out()
    rs = np.random.RandomState(77)
    polys = []
    v = R["Viewer"](384, 384)
    for k in range(160):
        w, h = rs.uniform(0.4, 0.8, 2)
        x, y = rs.uniform(-1.0, 1.0 - w), rs.uniform(-1.0 + h, 1.0)
        corners = np.array(R["make_rect"](float(w), float(h), True).points) + np.array([x + w / 2, y - h / 2])
        if k % 2 == 0:
            v.set_bounds(left=-1 * Z, right=1 * Z, bottom=-1 * Z, top=1 * Z)
        else:
            rx, ry = rs.uniform(-1, 1, 2)
            v.set_cam_follow(source_xy_world=(float(rx), float(ry)), target_xy_01=(0.5, 0.15),
                             viewport_hw_world=(2 * Z, 2 * Z), rotation=float(rs.uniform(-7, 7)))
        st = R["Stack"]()
        st.push(v.pygame_transform)
        st.push(v.transform)
        polys.append(st.apply_current_matrix(corners))
    for _ in range(40):
        polys.append(rs.uniform(-60, 444, (4, 2)))
    polys.append(np.array([[10.0, 20.0], [200.0, 20.0], [200.0, 300.5], [10.0, 300.5]]))
    polys.append(np.array([[-30.5, 5.5], [420.5, 5.5], [420.5, 390.0], [-30.5, 390.0]]))
    polys.append(np.array([[17.5, 12.5], [372.5, 33.5], [352.5, 371.5], [27.5, 342.5]]))
    out = []
    for pts in polys:
        for dashed in (True, False):
            p = Poly(pts.tolist(), True)
            p.dashed = dashed
            p.geom = np.asarray(pts, dtype=np.float64)
            rec.calls = []
            p._render(None)
            out.append({"pts": _m(pts), "dashed": dashed, "calls": rec.calls})
    return {"cases": out}


def ref_make_line():
    ns = _extract(os.path.join(REF, "benchmarks", "make_line.py"), ["longest_line"],
                  {"__name__": "ref_make_line", "np": np, "it": itertools})
    longest_line = ns["longest_line"]
    rs = np.random.RandomState(0)
    shape_rad = 0.2 * 0.6
    inlier, sep = shape_rad * 1.5, shape_rad * 3.5   # make_line.py: inlier_dist / max_sep defaults
    cases = [rs.uniform(-1, 1, (rs.randint(1, 5), 2)) for _ in range(700)]
    for _ in range(900):  # points near a random line, spacing around the separation threshold
        n = rs.randint(3, 5)
        o, d = rs.uniform(-0.5, 0.5, 2), rs.uniform(-1, 1, 2)
        d /= np.linalg.norm(d)
        t = np.cumsum(rs.uniform(0.3, 0.5, n))
        off = rs.uniform(-1, 1, n) * rs.choice([0.0, 0.17, 0.18, 0.19])
        cases.append(o + t[:, None] * d + off[:, None] * np.array([-d[1], d[0]]))
    out = []
    for p in cases:
        out.append({"pts": p.ravel().tolist(), "best": int(longest_line(p, inlier, sep))})
    return {"inlier_dist": inlier, "max_sep": sep, "cases": out}


# ---- preprocessor wrappers (benchmarks/__init__.py) -----------------------------------------------
class _Box:
    """stand-in for gym.spaces.Box (bounds as arrays, like gym 0.17)"""

    def __init__(self, low, high, shape=None, dtype=np.float32):
        dtype = np.dtype(dtype)
        if shape is not None:
            low, high = np.full(shape, low, dtype=dtype), np.full(shape, high, dtype=dtype)
        self.low, self.high = np.asarray(low, dtype=dtype), np.asarray(high, dtype=dtype)
        self.shape, self.dtype = self.low.shape, dtype


class _Dict:
    def __init__(self, spaces):
        self.spaces = collections.OrderedDict(spaces)

    def __getitem__(self, k):
        return self.spaces[k]

    def __setitem__(self, k, v):
        self.spaces[k] = v


class _Wrapper:
    def __init__(self, env):
        self.env = env
        self.observation_space = env.observation_space

    def step(self, action):
        return self.env.step(action)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)


class _ObservationWrapper(_Wrapper):
    def step(self, action):
        o, r, d, i = self.env.step(action)
        return self.observation(o), r, d, i

    def reset(self, **kwargs):
        return self.observation(self.env.reset(**kwargs))


def _is_image_space(box):
    """stable_baselines3.common.preprocessing.is_image_space (channels-last uint8 Box in [0, 255])"""
    return isinstance(box, _Box) and len(box.shape) == 3 and box.dtype == np.uint8 and \
        np.all(box.low == 0) and np.all(box.high == 255)


def _cv2_resize(img, size, interpolation=None):
    """cv2.resize(INTER_AREA) 384^2 -> 96^2, per channel: the oracle's o_downsample on each 3 channels"""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
    import pyoracle as po
    assert img.shape[:2] == (384, 384) and tuple(size) == (96, 96) and img.shape[2] % 3 == 0
    return np.concatenate([po.downsample(np.ascontiguousarray(img[..., c:c + 3])) for c in range(0, img.shape[2], 3)],
                          axis=-1)


class SyntheticFrames:
    """Base env emitting random 384^2 allo / ego frames: the j-th observation of a case is
    RandomState(1000 * case + j).randint(0, 256, (2, 384, 384, 3), dtype=uint8)."""

    def __init__(self, case):
        self.case, self.j = case, 0
        img = _Box(0, 255, (384, 384, 3), np.uint8)
        self.observation_space = _Dict([("allo", img), ("ego", _Box(0, 255, (384, 384, 3), np.uint8))])

    def _obs(self):
        f = np.random.RandomState(1000 * self.case + self.j).randint(0, 256, (2, 384, 384, 3), dtype=np.uint8)
        self.j += 1
        return collections.OrderedDict([("allo", f[0]), ("ego", f[1])])

    def reset(self):
        return self._obs()

    def step(self, action):
        return self._obs(), 0.0, False, {}


WRAPPER_EVENTS = ["reset", "step", "step", "step", "step", "step", "reset", "step", "step"]


def _digest(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.tobytes()).hexdigest()


def ref_wrappers():
    gym = types.SimpleNamespace(Wrapper=_Wrapper, ObservationWrapper=_ObservationWrapper,
                                spaces=types.SimpleNamespace(Box=_Box, Dict=_Dict))
    ns = {"__name__": "ref_wrappers", "np": np, "collections": collections, "functools": functools,
          "gym": gym, "Box": _Box, "Dict": _Dict, "Discrete": None, "Optional": typing.Optional,
          "is_image_space": _is_image_space, "cv2": types.SimpleNamespace(resize=_cv2_resize, INTER_AREA=3),
          "ResizeObservation": None, "cls_lookup": None}
    _extract(os.path.join(REF, "benchmarks", "__init__.py"),
             ["_gym_tree_map", "EagerDictFrameStack", "FlattenFrameStack", "ResizeDictObservation", "ChannelsFirst",
              "get_cls", "lores_stack_entry_point", "lores_ea_entry_point", "DEFAULT_PREPROC_ENTRY_POINT_WRAPPERS"], ns)
    out = {"events": WRAPPER_EVENTS, "cases": []}
    for case, (pp, make) in enumerate(ns["DEFAULT_PREPROC_ENTRY_POINT_WRAPPERS"].items()):
        env = make(lambda c=case: SyntheticFrames(c))()
        space = [[k, list(b.shape), str(b.dtype)] for k, b in env.observation_space.spaces.items()]
        obs_log = []
        for ev in WRAPPER_EVENTS:
            o = env.reset() if ev == "reset" else env.step(0)[0]
            obs_log.append([[k, list(np.shape(v)), str(np.asarray(v).dtype), _digest(v)] for k, v in o.items()])
        out["cases"].append({"preproc": pp, "case": case, "space": space, "obs": obs_log})
    return out


# ---- scorers and the action table --------------------------------------------------------------------
def _pos(x, y):
    return types.SimpleNamespace(shape_body=types.SimpleNamespace(position=types.SimpleNamespace(x=float(x), y=float(y))))


def ref_scorers():
    class _Base:
        pass

    ns = {"__name__": "ref_cluster", "np": np, "abc": __import__("abc"), "enum": enum, "BaseEnv": _Base, "EzPickle": object, "ez_init": lambda **k: (lambda f: f)}
    _extract(os.path.join(REF, "benchmarks", "cluster.py"), ["BaseClusterEnv"], ns)
    C = ns["BaseClusterEnv"]
    rs = np.random.RandomState(31)
    values = ["blue", "green", "red", "yellow"]
    cases = []

    def run(vals, xy):
        env = object.__new__(C)
        by = {}
        for v, (x, y) in zip(vals, xy):
            by.setdefault(values[v], []).append(_pos(x, y))
        env._BaseClusterEnv__characteristic_values = np.unique([values[v] for v in vals])
        env._BaseClusterEnv__blocks_by_characteristic = by
        return float(env.score_on_end_of_traj())

    for k in range(600):
        n = int(rs.randint(7, 11))
        vals = list(range(4)) + list(rs.randint(0, 4, n - 4))
        rs.shuffle(vals)
        kind = k % 3
        if kind == 0:     # random layout
            xy = rs.uniform(-1, 1, (n, 2))
        else:             # clustered around per-value centres, spread scanned across the margin threshold
            centres = rs.uniform(-0.7, 0.7, (4, 2))
            spread = rs.choice([0.02, 0.05, 0.08, 0.1, 0.12, 0.15, 0.2]) if kind == 1 else rs.uniform(0.03, 0.2)
            xy = centres[vals] + rs.normal(0, spread, (n, 2))
        cases.append({"vals": [int(v) for v in vals], "xy": xy.ravel().tolist(), "score": run(vals, xy)})
    mtc_ns = {"__name__": "ref_mtc", "np": np, "math": math, "BaseEnv": _Base, "EzPickle": object,
              "ez_init": lambda **k: (lambda f: f), "warnings": None, "geom": None, "en": None}
    _extract(os.path.join(REF, "benchmarks", "move_to_corner.py"), ["MoveToCornerEnv"], mtc_ns)
    M = mtc_ns["MoveToCornerEnv"]
    mtc = []
    for k in range(600):
        r = rs.uniform(-1.2, 1.2, 2) if k % 4 else np.array([-1.0, 1.0]) + rs.uniform(-0.8, 0.8, 2)
        sh = rs.uniform(-1.2, 1.2, 2) if k % 5 else r + rs.uniform(-0.25, 0.25, 2)
        env = object.__new__(M)
        env.robot = types.SimpleNamespace(robot_body=types.SimpleNamespace(position=(float(r[0]), float(r[1]))))
        env._robot = env.robot
        env._MoveToCornerEnv__shape_ref = types.SimpleNamespace(
            shape_body=types.SimpleNamespace(position=(float(sh[0]), float(sh[1]))))
        mtc.append({"robot": r.tolist(), "shape": sh.tolist(), "score": float(env.score_on_end_of_traj()),
                    "shaped": float(env.debug_shaped_reward())})
    return {"cluster_values": values, "cluster": cases, "move_to_corner": mtc}


def ref_actions():
    ns = {"__name__": "ref_entities", "enum": enum}
    _extract(os.path.join(REF, "entities.py"),
             ["RobotAction", "ACTION_NUMS_FLAGS_NAMES", "ACTION_ID_TO_FLAGS", "FLAGS_TO_ACTION_ID"], ns)
    tree = ast.parse(open(os.path.join(REF, "entities.py")).read())
    robot = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Robot")
    set_action = next(n for n in robot.body if isinstance(n, ast.FunctionDef) and n.name == "set_action")
    exec(compile(ast.Module(body=[set_action], type_ignores=[]), "entities.py", "exec"), ns)
    rows = []
    for act_id, flags, name in ns["ACTION_NUMS_FLAGS_NAMES"]:
        bot = types.SimpleNamespace(radius=0.2, finger_rot_limit_outer=math.pi / 8, finger_rot_limit_inner=0,
                                    target_finger_angle=123.0)
        action_flag = ns["RobotAction"].NONE
        for f in flags:
            action_flag |= f
        ns["set_action"](bot, action_flag)
        rows.append({"id": act_id, "flags": [int(f) for f in flags], "name": name, "bits": int(action_flag),
                     "target_speed": bot.target_speed, "rel_turn_angle": bot.rel_turn_angle,
                     "target_finger_angle": float(bot.target_finger_angle),
                     "flags_to_action": ns["FLAGS_TO_ACTION_ID"][tuple(flags)]})
    return {"actions": rows, "flag_values": {m.name: int(m.value) for m in ns["RobotAction"]}}


def ref_latex():
    """evaluation.py:101-154 (latexify_results) on synthetic do_eval() frames: one and two algorithms over
    a demo env and its test variants, env order as first seen; plus the duplicate-id error message."""
    import io
    import pandas as pd
    ns = {"io": io}
    _extract(os.path.join(REF, "evaluation.py"), ["latexify_results"], ns)
    rs = np.random.RandomState(77)
    envs = ["MoveToCorner-Demo-v0", "MoveToCorner-TestJitter-v0", "MoveToCorner-TestColour-v0", "MoveToCorner-TestAll-v0"]
    cases = []
    for algs, col in ((["bc"], "run_id"), (["bc", "gail", "dagger"], "run_id"), (["x", "y"], "algo")):
        recs = [{"demo_env": envs[0], "test_env": e, "mean_score": float(rs.uniform(0, 1)),
                 "std_score": float(rs.uniform(0, 0.5)), col: a} for a in algs for e in envs]
        cases.append({"records": recs, "id_column": col,
                      "latex": ns["latexify_results"](pd.DataFrame.from_records(recs), id_column=col)})
    dup = cases[0]["records"] + cases[0]["records"][:1]
    try:
        ns["latexify_results"](pd.DataFrame.from_records(dup))
        err = None
    except ValueError as ex:
        err = str(ex)
    return {"cases": cases, "duplicate": {"records": dup, "error": err}}


def main():
    only = set(sys.argv[1:])
    for fn, make in (("ref_render.json", ref_render), ("ref_make_line.json", ref_make_line),
                     ("ref_outline.json", ref_outline), ("ref_wrappers.json", ref_wrappers),
                     ("ref_scorers.json", ref_scorers), ("ref_actions.json", ref_actions),
                     ("ref_latex.json", ref_latex)):
        if only and fn not in only:
            continue
        data = make()
        with open(os.path.join(HERE, fn), "w") as f:
            json.dump(data, f, indent=None, separators=(",", ":"))
            f.write("\n")
        print("wrote", fn)


if __name__ == "__main__":
    main()
