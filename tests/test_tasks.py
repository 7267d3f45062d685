"""Task scorers and resets of the SURVEY.md 8(f) F1 tasks in the CPU oracle (no GPU).

MakeLine's longest_line (make_line.py:33-74) is checked against an independent numpy
restatement of the reference algorithm (all-pairs inlier lines, sorted projections, longest
run of separations <= max_sep) evaluated with numpy itself, on random point sets and on
exactly / nearly collinear sets that sit at the inlier and separation thresholds.
"""
import itertools

import numpy as np
import pytest

import pyoracle as po
from magical_amd import registry

SHAPE_RAD = 0.2 * 0.6


def np_longest_line(points, inlier_dist, max_separation):
    points = np.asarray(points, dtype=np.float64)
    n = len(points)
    best = min(1, n)
    for i in range(n - 1):
        for j in range(i + 1, n):
            offs = points - points[i][None]
            unit = offs[j] / np.linalg.norm(offs[j])
            proj = np.squeeze(offs @ unit[:, None], axis=1)
            dist = np.linalg.norm(offs - proj[:, None] * unit, axis=1)
            inl = np.nonzero(dist <= inlier_dist)[0]
            if len(inl) <= best:
                continue
            seps = np.abs(np.diff(np.sort(proj[inl])))
            runs = [len(list(g)) for ok, g in itertools.groupby(seps <= max_separation) if ok]
            best = max(best, max(runs, default=0) + 1)
    return best


def c_longest_line(points, inlier_dist, max_sep):
    import ctypes
    p = np.ascontiguousarray(np.asarray(points, dtype=np.float64))
    x, y = np.ascontiguousarray(p[:, 0]), np.ascontiguousarray(p[:, 1])
    return po.lib().o_longest_line(x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p),
                                   len(p), inlier_dist, max_sep)


def test_longest_line_matches_numpy():
    rs = np.random.RandomState(0)
    inlier, sep = SHAPE_RAD * 1.5, SHAPE_RAD * 3.5
    cases = [rs.uniform(-1, 1, (rs.randint(1, 5), 2)) for _ in range(3000)]
    for _ in range(3000):  # points near a random line, spacing around the separation threshold
        n = rs.randint(3, 5)
        o, d = rs.uniform(-0.5, 0.5, 2), rs.uniform(-1, 1, 2)
        d /= np.linalg.norm(d)
        t = np.cumsum(rs.uniform(0.3, 0.5, n))
        off = rs.uniform(-1, 1, n) * rs.choice([0.0, 0.17, 0.18, 0.19])
        cases.append(o + t[:, None] * d + off[:, None] * np.array([-d[1], d[0]]))
    for p in cases:
        assert c_longest_line(p, inlier, sep) == np_longest_line(p, inlier, sep), p


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
