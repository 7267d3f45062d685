"""CPU: the oracle's resets against the REFERENCE'S OWN reset control flow.

tests/golden/ref_resets.json was produced by executing base_env.py's BaseEnv.reset (with
PhysicsVariables.sample, _make_robot, _make_shape, add_entities), the task on_reset methods
(move_to_region.py, move_to_corner.py, cluster.py, match_regions.py) and geom.py's randomisers
(pm_randomise_all_poses / pm_randomise_pose / pm_shift_bodies / randomise_hw) from /root/reference
on numpy RandomState(seed), over a stand-in pymunk Space whose entity geometry, pose setters, shape
filters and shape queries are the oracle's own (tests/golden/make_ref_fixtures.py, ref_resets).  So
every RNG draw, its order, each rejection-sampling try, the per-retry filter capture
(geom.py:302-309), the rollback on PlacementError (:249-254), the rel_*_limit clamps (:180-198) and
the whole-layout retries (:295-341) are the reference's; the geometry and the collision predicate
are the oracle's (pinned separately).  Lowered try budgets (max_tries, an AST parameter in the
generator, MG_DEBUG_MAX_TRIES / set_max_tries on our side) force retries and PlacementErrors.

The oracle's own reset (oracle/scene.c) must reach the same final pose of every body (bit for bit),
the same retry count, the same PlacementError outcome and the same MT19937 state (so the same number
of draws).  The GPU equals the oracle (tests/test_gpu_parity.py).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import pyoracle as po

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _cases():
    with open(os.path.join(GOLDEN, "ref_resets.json")) as f:
        return json.load(f)["cases"]


CASES = _cases()


def test_fixture_exercises_the_control_flow():
    names = {c["name"] for c in CASES}
    assert "MatchRegions-TestAll-v0" in names and len(CASES) >= 600
    assert sum(1 for c in CASES if c["name"] == "MatchRegions-TestAll-v0") >= 200
    assert sum(1 for c in CASES if c["retries"] > 0) >= 10       # whole-layout retries happened
    assert sum(1 for c in CASES if c["error"]) >= 3              # ... and PlacementErrors (rollback + raise)
    assert any(c["retries"] > 0 and not c["error"] for c in CASES)


@pytest.mark.parametrize("name", sorted({c["name"] for c in CASES}))
def test_oracle_resets_follow_the_reference_control_flow(name):
    n = 0
    for c in CASES:
        if c["name"] != name:
            continue
        env = po.OracleEnv(c["task"], c["flags"], None, 100, seed=c["seed"])
        env.set_max_tries(c["max_tries"])
        try:
            env.reset()
            err = False
        except po.PlacementError:
            err = True
        tag = f"{name} seed {c['seed']} max_tries {c['max_tries']}"
        assert err == c["error"], tag
        # the oracle counts every failed layout attempt; the reference prints all but the last (which raises)
        assert env.placement_retries() == c["retries"] + (1 if err else 0), tag
        poses = env.entity_poses()
        assert len(poses) == len(c["poses"]), tag
        for k, (got, ref) in enumerate(zip(poses, c["poses"])):
            assert np.array_equal(np.asarray(got), np.asarray(ref)), f"{tag} entity {k + 1}"
        key, pos = env.rng_state()
        assert pos == c["rng_pos"], tag
        assert hashlib.sha256(key.tobytes()).hexdigest() == c["rng_key_sha256"], tag
        n += 1
    assert n > 0
