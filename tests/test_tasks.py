"""Task scorers and resets of the SURVEY.md 8(f) F1 tasks in the CPU oracle (no GPU).

MakeLine's longest_line (make_line.py:31-72) is pinned to the reference's own function, executed
on random and near-collinear point sets (tests/test_reference_fixtures.py).
"""
import numpy as np
import pytest

import pyoracle as po
from magical_amd import registry

SHAPE_RAD = 0.2 * 0.6


@pytest.mark.parametrize("name", ["MakeLine-Demo-v0", "MakeLine-TestJitter-v0", "MakeLine-TestColour-v0",
                                  "MakeLine-TestShape-v0", "MakeLine-TestLayout-v0", "MakeLine-TestCountPlus-v0",
                                  "MakeLine-TestAll-v0"])
def test_make_line_resets(name):
    """make_line.py:86-132: blocks first (3-4 with a random count), robot last, every entity placed
    inside the arena; the Demo layout is the reference's default one."""
    spec = registry.lookup(name)
    for seed in range(4):
        env = po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=seed)
        env.reset()
        kinds, types, cols, _ = env.entities()
        assert kinds[0] == 0 and kinds[-1] == 2  # arena first, robot last (oscene.h ENT_*)
        nblk = int((kinds == 3).sum())
        assert nblk == (4 if not spec.rand_flags & registry.SHAPE_COUNT else nblk) and 3 <= nblk <= 4
        b = env.bodies()
        assert np.all(np.abs(b[:nblk + 1, 0:2]) <= 1.0 + 1e-9)  # sampled poses: blocks, robot body
        if name == "MakeLine-Demo-v0":
            assert np.allclose(b[0, 0:2], (0.790, -0.820)) and np.allclose(b[nblk, 0:2], (0.702, -0.255))
