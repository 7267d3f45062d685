"""CPU: the oracle's frame-stack rule, scorers and action decode, and the product's host tables, against
outputs of the REFERENCE'S OWN CODE executed in the build container (tests/golden/make_ref_fixtures.py):

* ref_wrappers.json -- the preprocessor entry points of benchmarks/__init__.py:232-307 (FlattenFrameStack /
  EagerDictFrameStack :51-147, ResizeDictObservation :150-190, ChannelsFirst :193-216), every LoRes
  preprocessor, over synthetic 384^2 frame sequences with a mid-sequence reset;
* ref_scorers.json -- cluster.py:166-216 and move_to_corner.py:67-100 on explicit positions;
* ref_actions.json -- entities.py:148-190 and Robot.set_action (:435-453).

The GPU's own stacks are checked against these fixtures in tests/test_demos.py (mg_replay_lores) and
against the oracle rule in tests/test_gpu_parity.py (render kernel, mg_restack)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

import pyoracle as po
from magical_amd import dist as mdist
from magical_amd import envs as mg_envs
from magical_amd import registry

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def synthetic_frames(case, j):
    """the j-th observation of fixture case `case` (make_ref_fixtures.SyntheticFrames)"""
    f = np.random.RandomState(1000 * case + j).randint(0, 256, (2, 384, 384, 3), dtype=np.uint8)
    return f[0], f[1]


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def fixture_lores(case, events):
    lo, starts, start = [], [], 0
    for j, ev in enumerate(events):
        if ev == "reset":
            start = j
        a, g = synthetic_frames(case, j)
        lo.append((po.downsample(a), po.downsample(g)))
        starts.append(start)
    return lo, starts


WRAPPERS = golden("ref_wrappers.json")


@pytest.mark.parametrize("case", WRAPPERS["cases"], ids=lambda c: c["preproc"])
def test_stack_rule_matches_reference_wrappers(case):
    """po.stack_lores (the rule the GPU replay / demo tests check against) reproduces the reference
    entry point's observations: key order, shapes, dtypes and bytes, across the reset."""
    pp = case["preproc"]
    lo, starts = fixture_lores(case["case"], WRAPPERS["events"])
    chw = registry.PREPROCESSORS[pp].get("channels_first", False)
    got = po.stack_lores(lo, starts, pp, chw)
    for j, ref in enumerate(case["obs"]):
        assert [k for k, *_ in ref] == list(got[j]), (pp, j)
        for (k, shape, dtype, h), (k2, v) in zip(ref, got[j].items()):
            assert list(v.shape) == shape and str(v.dtype) == dtype and digest(v) == h, (pp, j, k)


@pytest.mark.parametrize("case", WRAPPERS["cases"], ids=lambda c: c["preproc"])
def test_observation_space_matches_reference_wrappers(case):
    spec = registry.lookup(f"MoveToRegion-Demo-{case['preproc']}-v0")
    space = mg_envs.observation_space(spec)
    assert [[k, list(b.shape), str(np.dtype(b.dtype))] for k, b in space.spaces.items()] == case["space"]


@pytest.mark.parametrize("case", WRAPPERS["cases"], ids=lambda c: c["preproc"])
def test_oracle_restacker_matches_reference_wrappers(case):
    """The receiver-side restack rule of the compact multi-GPU gather (po.OracleRestacker, whose GPU
    counterpart mg_restack is checked against it in tests/test_gpu_parity.py) rebuilds the reference's
    stacks from the current frames alone: reset events are all-fresh gathers, steps carry done = 0."""
    pp = case["preproc"]
    spec = registry.lookup(f"MoveToRegion-Demo-{pp}-v0")
    lay = mdist.PackedLayout.for_spec(spec, 1, frames_only=True)
    rs = po.OracleRestacker(lay, pp)
    lo, _ = fixture_lores(case["case"], WRAPPERS["events"])
    keys = mdist.stacked_keys(pp)
    for j, ev in enumerate(WRAPPERS["events"]):
        recv = torch.zeros(lay.nbytes, dtype=torch.uint8)
        v = lay.views(recv)
        v["allo"][0] = torch.from_numpy(lo[j][0])
        v["ego"][0] = torch.from_numpy(lo[j][1])
        outs = {k: torch.zeros((1, 96, 96, 12), dtype=torch.uint8) for k in keys}
        rs(recv, outs, j, ev == "reset")
        ref = {k: h for k, _, _, h in case["obs"][j]}
        for k in keys:
            a = outs[k][0].numpy()
            if registry.PREPROCESSORS[pp].get("channels_first", False):
                a = np.moveaxis(a, -1, 0)
            assert digest(a) == ref[k], (pp, j, k)


def test_cluster_scorer_matches_reference():
    """o_cluster_score (the oracle's cluster.py:166-216; the GPU scorer is checked against it on placed
    blocks in tests/test_gpu_parity.py) equals the reference's score_on_end_of_traj bit for bit on random,
    clustered and near-threshold layouts of 7-10 blocks."""
    g = golden("ref_scorers.json")
    scores = set()
    for c in g["cluster"]:
        xy = np.asarray(c["xy"]).reshape(-1, 2)
        got = po.cluster_score(c["vals"], xy)
        assert got == c["score"], c
        scores.add(round(got, 6))
    assert len(scores) >= 8   # intermediate scores, not only 0 / 1


def test_move_to_corner_scorer_and_shaped_reward_match_reference():
    g = golden("ref_scorers.json")
    for c in g["move_to_corner"]:
        assert po.score_move_to_corner(*c["robot"]) == c["score"], c
        assert po.shaped_move_to_corner(*c["robot"], *c["shape"]) == c["shaped"], c
    assert any(0.0 < c["score"] < 1.0 for c in g["move_to_corner"])


def test_action_table_and_decode_match_reference():
    """entities.py:148-190 (ids, flags, names, FLAGS_TO_ACTION_ID) against the host table
    (magical_amd.envs) and Robot.set_action's control targets against the oracle's decode (the GPU's
    robot_set_action is checked against the oracle in every rollout)."""
    g = golden("ref_actions.json")
    assert g["flag_values"] == {"NONE": 0, "UP": 1, "DOWN": 2, "LEFT": 4, "RIGHT": 8, "OPEN": 16, "CLOSE": 32}
    assert len(g["actions"]) == 18
    for row in g["actions"]:
        a = row["id"]
        assert mg_envs.ACTION_NUMS_FLAGS_NAMES[a] == (a, tuple(row["flags"]), row["name"])
        assert mg_envs.ACTION_ID_TO_FLAGS[a] == tuple(row["flags"])
        assert mg_envs.FLAGS_TO_ACTION_ID[tuple(row["flags"])] == row["flags_to_action"] == a
        speed, turn, finger = po.action_decode(a)
        assert (speed, turn, finger) == (row["target_speed"], row["rel_turn_angle"], row["target_finger_angle"]), row
