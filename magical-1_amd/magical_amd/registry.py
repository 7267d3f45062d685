"""Env-name registry: the reference's 441 names, grammar and variant tables.

Restates benchmarks/__init__.py:269-307 (preprocessor table), :308-424
(EnvName grammar, update_magical_env_name) and :427-1102 (register_envs
variant tables, episode lengths, DebugReward names).  Each name resolves to an
EnvSpec: task, rand_* flags (bit mask shared with the C ABI), preprocessor,
max_episode_steps.
"""
import collections
import re
from dataclasses import dataclass
from typing import Optional

# rand flag bits (include/magical_sim.h, mg_common.h)
LAYOUT_MINOR, LAYOUT_FULL, COLOUR, SHAPE_TYPE, SHAPE_COUNT, DYNAMICS = 1, 2, 4, 8, 16, 32
DEBUG_REWARD = 64  # debug_reward=True: dense shaped reward (move_to_corner.py:85-100, pick_and_place.py:108-124)

TASK_IDS = {"MoveToRegion": 0, "MoveToCorner": 1, "ClusterColour": 2, "ClusterShape": 3, "MatchRegions": 4,
            "MakeLine": 5, "FindDupe": 6, "FixColour": 7, "PickAndPlace": 8}
GPU_TASKS = set(TASK_IDS)

PREPROCESSORS = collections.OrderedDict([
    ("LoRes3EA", dict(kind="ea", allo_frames=1, ego_frames=3, channels_first=False)),
    ("LoRes4E", dict(kind="ea", allo_frames=0, ego_frames=4, channels_first=False)),
    ("LoRes4A", dict(kind="ea", allo_frames=4, ego_frames=0, channels_first=False)),
    ("LoResStack", dict(kind="stack", frames=4)),
    ("LoResCHW4E", dict(kind="ea", allo_frames=0, ego_frames=4, channels_first=True)),
    # benchmarks/__init__.py:301-306: LoResCHW4A is registered with ego_frames=4 (identical to CHW4E)
    ("LoResCHW4A", dict(kind="ea", allo_frames=0, ego_frames=4, channels_first=True)),
])
AVAILABLE_PREPROCESSORS = list(PREPROCESSORS)
# C-ABI preprocessor ids
PREPROC_IDS = {None: 0, "LoRes4E": 1, "LoResStack": 2, "LoRes3EA": 3, "LoRes4A": 4, "LoResCHW4E": 5,
               "LoResCHW4A": 5}

_ENV_NAME_RE = re.compile(
    r'^(?P<name_prefix>[^-]+)(?P<demo_test_spec>-(Demo|Test[^-]*))'
    r'(?P<env_name_suffix>(-[^-]+)*)(?P<version_suffix>-v\d+)$')


class EnvName:
    """benchmarks/__init__.py:350-424"""

    def __init__(self, env_name):
        match = _ENV_NAME_RE.match(env_name)
        if match is None:
            raise ValueError(f"env name '{env_name}' does not match _ENV_NAME_RE spec")
        g = match.groupdict()
        self.name_prefix = g['name_prefix']
        self.demo_test_spec = g['demo_test_spec']
        self.env_name_suffix = g['env_name_suffix']
        self.version_suffix = g['version_suffix']
        assert env_name == self.env_name
        if not self.is_test:
            assert self.demo_env_name == self.env_name, (self.demo_env_name, self.env_name)

    @property
    def env_name(self):
        return self.name_prefix + self.demo_test_spec + self.env_name_suffix + self.version_suffix

    @property
    def is_test(self):
        return self.demo_test_spec.startswith('-Test')

    @property
    def demo_env_name(self):
        return self.name_prefix + '-Demo' + self.env_name_suffix + self.version_suffix

    @property
    def task(self):
        return self.name_prefix

    @property
    def variant(self):
        return self.demo_test_spec.strip('-')

    @property
    def preproc(self):
        return self.env_name_suffix.strip('-') if self.env_name_suffix else None

    @property
    def version(self):
        return self.version_suffix.strip('-')


def update_magical_env_name(env_name, *, task=None, variant=None, preproc=None, version=None):
    """benchmarks/__init__.py:318-347"""
    ename = EnvName(env_name)
    parts = [task if task is not None else ename.task, variant if variant is not None else ename.variant]
    if preproc is None:
        preproc = ename.preproc
    if preproc is not None:
        parts.append(preproc)
    parts.append(version if version is not None else ename.version)
    return '-'.join(parts)


@dataclass(frozen=True)
class EnvSpec:
    name: str
    task: str
    variant: str
    rand_flags: int
    preproc: Optional[str]
    max_episode_steps: int
    debug_reward: bool = False

    @property
    def task_id(self):
        return TASK_IDS[self.task]

    @property
    def gpu_supported(self):
        return self.task in GPU_TASKS


def _f(**kw):
    bits = 0
    if kw.get("minor"): bits |= LAYOUT_MINOR
    if kw.get("full"): bits |= LAYOUT_FULL
    if kw.get("colour"): bits |= COLOUR
    if kw.get("shape"): bits |= SHAPE_TYPE
    if kw.get("count"): bits |= SHAPE_COUNT
    if kw.get("dyn"): bits |= DYNAMICS
    if kw.get("debug"): bits |= DEBUG_REWARD
    return bits


# (task, variant name, episode length, flags) in registration order
_STD7 = [("Demo", _f()), ("TestJitter", _f(minor=1)), ("TestColour", _f(colour=1)), ("TestShape", _f(shape=1)),
         ("TestLayout", _f(full=1)), ("TestCountPlus", _f(colour=1, shape=1, count=1, full=1)),
         ("TestDynamics", _f(dyn=1)), ("TestAll", _f(colour=1, shape=1, count=1, full=1, dyn=1))]
_BASE = []
for _task in ("ClusterShape", "ClusterColour"):
    _BASE += [(_task, v, 240, fl) for v, fl in _STD7]
for _task, _len in (("FindDupe", 100), ("FixColour", 60), ("MakeLine", 180), ("MatchRegions", 120)):
    _BASE += [(_task, v, _len, fl) for v, fl in _STD7]
_BASE += [("MoveToCorner", v, 80, fl) for v, fl in [
    ("Demo", _f()), ("TestColour", _f(colour=1)), ("TestShape", _f(shape=1)), ("TestJitter", _f(minor=1)),
    ("TestDynamics", _f(dyn=1)), ("TestAll", _f(colour=1, shape=1, minor=1, dyn=1))]]
_BASE += [("MoveToRegion", v, 40, fl) for v, fl in [
    ("Demo", _f()), ("TestJitter", _f(minor=1)), ("TestColour", _f(colour=1)), ("TestLayout", _f(full=1)),
    ("TestDynamics", _f(dyn=1)), ("TestAll", _f(full=1, colour=1, dyn=1))]]
# benchmarks/__init__.py:441-455: rand_shape_colour, rand_shape_type, rand_poses (unrestricted: layout
# full); the Demo variant is registered with debug_reward=True
_BASE += [("PickAndPlace", "Demo", 80, _f(colour=1, shape=1, full=1, debug=1)),
          ("PickAndPlace", "Test", 80, _f(colour=1, shape=1, full=1))]

ALL_REGISTERED_ENVS = []
SPECS = collections.OrderedDict()
DEMO_ENVS_TO_TEST_ENVS_MAP = collections.OrderedDict()


def _register_all():
    for task, variant, ep_len, flags in _BASE:
        name = f"{task}-{variant}-v0"
        ALL_REGISTERED_ENVS.append(name)
        SPECS[name] = EnvSpec(name, task, variant, flags, None, ep_len, debug_reward=bool(flags & DEBUG_REWARD))
        for pp in PREPROCESSORS:
            new = update_magical_env_name(name, preproc=pp)
            ALL_REGISTERED_ENVS.append(new)
            SPECS[new] = EnvSpec(new, task, variant, flags, pp, ep_len, debug_reward=bool(flags & DEBUG_REWARD))
    train_to_test = {}
    for name in ALL_REGISTERED_ENVS:
        p = EnvName(name)
        if p.is_test:
            train_to_test.setdefault(p.demo_env_name, []).append(p.env_name)
    DEMO_ENVS_TO_TEST_ENVS_MAP.update(sorted((k, tuple(v)) for k, v in train_to_test.items()))
    # benchmarks/__init__.py:1074-1100: registered with the UNWRAPPED env (no preprocessing)
    dbg = "MoveToCorner-Demo-DebugReward-v0"
    ALL_REGISTERED_ENVS.append(dbg)
    SPECS[dbg] = EnvSpec(dbg, "MoveToCorner", "Demo", DEBUG_REWARD, None, 80, debug_reward=True)
    for pp in PREPROCESSORS:
        n = f"MoveToCorner-Demo-DebugReward-{pp}-v0"
        ALL_REGISTERED_ENVS.append(n)
        SPECS[n] = EnvSpec(n, "MoveToCorner", "Demo", DEBUG_REWARD, None, 80, debug_reward=True)


_register_all()


def lookup(name) -> EnvSpec:
    try:
        return SPECS[name]
    except KeyError:
        raise KeyError(f"unknown MAGICAL env name {name!r}") from None
