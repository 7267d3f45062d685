"""Known answers of the oracle's narrowphase (cpCollide) and contact persistence, and their GPU twin.

The reference's collision arithmetic is Chipmunk2D 7.0.x inside pymunk 5.6, absent from this image; the
reference's shapes are built at entities.py:604-620 (SQUARE: Poly.create_box with a 0.01 * side bevel radius),
:650-652 / :720-721 (STAR: autogeometry.convex_decomposition parts, one shape filter group), :498-533 (arena
walls: radius-1 segments, friction 0.8) and the robot's circle body / finger polys; base_env.py:206-208 builds
the Space.  These tests pin oracle/phys.c's restatement of cpCollide to geometry
worked out by hand -- contact normal, penetration depth, contact points, feature hashes, which path (GJK or
EPA) a configuration takes -- and cpArbiterUpdate / cpArbiterApplyCachedImpulse / cpSpaceArbiterSetFilter
(A.4) to exact velocity changes: warm starts reused by feature hash, kept across 1-2 steps apart, dropped
after collisionPersistence = 3, friction u = uA * uB saturating the tangent clamp.

Conventions (Chipmunk's): a collision (a, b) has a = the lower shape type (circle < segment < poly), n the
unit normal from a to b, contact k the points p1 (on a's surface) and p2 (on b's); its separation is
dot(p2 - p1, n) (negative: penetrating; cpArbiterPreStep's `dist`).

GPU twin (`-m gpu`): the same kinds of configurations placed in real scenes (ClusterColour: circle, star,
square, pentagon blocks against each other, the walls and the robot; MoveToCorner: the quad step form)
through mg_set_body_pose, stepped, and the arbiter tables (mg_get_arbiters) and bodies compared with the
oracle's, step by step.
"""
import ctypes
import math

import numpy as np
import pytest

import pyoracle as po
from test_oracle_known_answers import DT, Space, _lib

d, i_, vp = ctypes.c_double, ctypes.c_int, ctypes.c_void_p
TOL = 1e-12
SHAPE_RAD = 0.12                          # entities.py SHAPE_RAD (shape_size of the benchmark blocks)
SIDE = math.sqrt(math.pi) * SHAPE_RAD     # entities.py:617 create_box side
BEVEL = 0.01 * SIDE                       # entities.py:620


def _L():
    L = _lib()
    if not getattr(L, "_osb_np_ready", False):
        L.osb_collide.restype = i_; L.osb_collide.argtypes = [vp, i_, i_, vp, vp]
        L.osb_epa_runs.restype = ctypes.c_long; L.osb_epa_runs.argtypes = []
        L.osb_set_pose.argtypes = [vp, i_, d, d, d]
        L.osb_set_iterations.argtypes = [vp, i_]
        L.osb_arbiter_ex.restype = i_; L.osb_arbiter_ex.argtypes = [vp, i_, vp, vp]
        L.osb_arbiter_set_impulse.argtypes = [vp, i_, i_, d, d]
        L._osb_np_ready = True
    return L


class Sandbox(Space):
    def __init__(self):
        super().__init__()
        self.X = _L()

    def collide(self, a, b):
        out = np.zeros(12)
        h = np.zeros(2, dtype=np.uint64)
        n = self.X.osb_collide(self.h, a, b, po.ptr(out), po.ptr(h))
        con = [(out[4 + 4 * k:6 + 4 * k].copy(), out[6 + 4 * k:8 + 4 * k].copy()) for k in range(n)]
        return dict(count=n, swapped=int(out[1]), n=out[2:4].copy(), con=con, hash=[int(x) for x in h[:n]])

    def pose(self, b, x, y, a=0.0):
        self.X.osb_set_pose(self.h, b, x, y, a)

    def iterations(self, k):
        self.X.osb_set_iterations(self.h, k)

    def arbiter(self, i=0):
        out = np.zeros(28)
        h = np.zeros(2, dtype=np.uint64)
        n = self.X.osb_arbiter_ex(self.h, i, po.ptr(out), po.ptr(h))
        cons = [dict(r1=out[8 + 10 * k:10 + 10 * k], r2=out[10 + 10 * k:12 + 10 * k], jn=out[12 + 10 * k],
                     jt=out[13 + 10 * k], hash=int(h[k])) for k in range(n)]
        return dict(slot=int(out[0]), state=int(out[1]), count=n, n=out[5:7].copy(), u=out[7], con=cons)

    def set_impulse(self, i, k, jn, jt=0.0):
        self.X.osb_arbiter_set_impulse(self.h, i, k, jn, jt)

    def narrowphase_arbiters(self):
        return self.L.osb_num_arbiters(self.h)


HASH_COEF = 3344921057                  # chipmunk_private.h CP_HASH_COEF


def hash_pair(a, b):
    """CP_HASH_PAIR(A, B) = A * CP_HASH_COEF ^ B * CP_HASH_COEF on 64-bit cpHashValue"""
    m = 2 ** 64 - 1
    return ((a * HASH_COEF) & m) ^ ((b * HASH_COEF) & m)


def epa_runs():
    return _L().osb_epa_runs()


def box_verts(h, w=None):
    w = h if w is None else w
    return [(w, -h), (w, h), (-w, h), (-w, -h)]


def sep(c, n):
    """cpContact separation dot(p2 - p1, n) of contact c = (p1, p2)"""
    return float(np.dot(c[1] - c[0], n))


def assert_contacts(got, want, tol=TOL):
    """got: [(p1, p2)], want: [((x1, y1), (x2, y2))] in any order"""
    assert len(got) == len(want), (got, want)
    left = list(want)
    for p1, p2 in got:
        for k, (q1, q2) in enumerate(left):
            if np.abs(p1 - q1).max() <= tol and np.abs(p2 - q2).max() <= tol:
                del left[k]
                break
        else:
            raise AssertionError(f"contact {p1}, {p2} not expected in {want}")


def test_circle_circle():
    """CircleToCircle: n along the centre line, one contact at each surface, hash 0; coincident centres take
    n = (1, 0); touching exactly (dist == r1 + r2) is not a contact (distsq < mindist^2)."""
    s = Sandbox()
    a = s.body(0.5, 0.01, (0.3, -0.2)); ca = s.circle(a, 0.1)
    b = s.body(0.5, 0.01, (0.42, -0.04)); cb = s.circle(b, 0.15)     # delta (0.12, 0.16): dist 0.2
    r = s.collide(ca, cb)
    assert r["count"] == 1 and r["swapped"] == 0 and r["hash"] == [0]
    assert np.abs(r["n"] - (0.6, 0.8)).max() <= TOL
    assert_contacts(r["con"], [((0.36, -0.12), (0.33, -0.16))])
    assert abs(sep(r["con"][0], r["n"]) - (0.2 - 0.25)) <= TOL
    r = s.collide(cb, ca)                                             # same type: no swap, n reversed
    assert r["swapped"] == 0 and np.abs(r["n"] - (-0.6, -0.8)).max() <= TOL
    s.pose(b, 0.3, -0.2)
    r = s.collide(ca, cb)
    assert r["count"] == 1 and tuple(r["n"]) == (1.0, 0.0)
    assert abs(sep(r["con"][0], r["n"]) + 0.25) <= TOL
    s.pose(b, 0.3 + 0.25, -0.2)                                       # exactly touching
    assert s.collide(ca, cb)["count"] == 0
    s.pose(b, 0.3 + 0.2499, -0.2)
    assert s.collide(ca, cb)["count"] == 1


def test_circle_against_arena_wall():
    """CircleToSegment against a radius-1 arena wall (entities.py:498-533): the segment's core is 1 behind
    the wall surface; face region (closest point inside the segment) and end-cap region (clamped to the
    end point); the pair is collided as (circle, segment) whichever order it is asked in."""
    s = Sandbox()
    w = s.segment((-2.0, -2.0), (2.0, -2.0), 1.0)                     # surface y = -1
    b = s.body(0.5, 0.0036, (0.3, -0.95)); c = s.circle(b, 0.12)
    r = s.collide(w, c)
    assert r["count"] == 1 and r["swapped"] == 1 and r["hash"] == [0]
    assert np.abs(r["n"] - (0.0, -1.0)).max() <= TOL
    assert_contacts(r["con"], [((0.3, -1.07), (0.3, -1.0))])
    assert abs(sep(r["con"][0], r["n"]) + 0.07) <= TOL
    s.pose(b, 2.6, -1.2)                                              # beyond the end point (2, -2)
    r = s.collide(c, w)
    assert r["count"] == 1 and r["swapped"] == 0
    assert np.abs(r["n"] - (-0.6, -0.8)).max() <= TOL
    assert_contacts(r["con"], [((2.528, -1.296), (2.6, -1.2))])
    assert abs(sep(r["con"][0], r["n"]) + 0.12) <= TOL
    s.pose(b, 0.3, -1.0 + 0.12 + 1e-9)                                 # just off the surface
    assert s.collide(c, w)["count"] == 0


def test_circle_poly_face_vertex_and_deep():
    """CircleToPoly: GJK's closest points between the circle centre and the polygon, so the face region
    gives the face normal and the vertex region the centre-to-vertex direction; a centre inside the polygon
    takes the EPA path and the normal of the nearest face (depth = radius + centre-to-face distance)."""
    s = Sandbox()
    a = s.body(0.5, 0.01, (0.0, 0.0)); p = s.poly(a, box_verts(0.1))
    b = s.body(0.5, 0.01, (0.13, 0.02)); c = s.circle(b, 0.05)
    e0 = epa_runs()
    r = s.collide(p, c)                                               # face region, 0.02 deep
    assert r["count"] == 1 and r["swapped"] == 1 and r["hash"] == [0]
    assert np.abs(r["n"] - (-1.0, 0.0)).max() <= TOL
    assert_contacts(r["con"], [((0.08, 0.02), (0.1, 0.02))])
    assert abs(sep(r["con"][0], r["n"]) + 0.02) <= TOL
    assert epa_runs() == e0
    s.pose(b, 0.12, 0.13)                                             # vertex region (0.1, 0.1)
    r = s.collide(c, p)
    dist = math.hypot(0.02, 0.03)
    n = np.array([-0.02, -0.03]) / dist
    assert r["count"] == 1 and np.abs(r["n"] - n).max() <= TOL
    assert_contacts(r["con"], [(np.array([0.12, 0.13]) + 0.05 * n, np.array([0.1, 0.1]))])
    assert abs(sep(r["con"][0], r["n"]) - (dist - 0.05)) <= TOL
    assert epa_runs() == e0
    s.pose(b, 0.08, 0.0)                                              # centre inside: EPA
    r = s.collide(c, p)
    assert epa_runs() == e0 + 1
    assert r["count"] == 1 and np.abs(r["n"] - (-1.0, 0.0)).max() <= TOL
    assert_contacts(r["con"], [((0.03, 0.0), (0.1, 0.0))])
    assert abs(sep(r["con"][0], r["n"]) + 0.07) <= TOL
    s.pose(b, 0.16, 0.0)                                              # 0.01 clear of the face
    assert s.collide(c, p)["count"] == 0


def test_poly_poly_axis_aligned_overlap_two_clipped_contacts():
    """PolyToPoly, overlapping cores (EPA): the minimum-penetration axis is the x faces, and the two contacts
    are the ends of the faces' overlap interval clipped onto each face (ContactPoints, A.3): y in {-0.05, 0.1},
    p1 on A's face x = 0.1, p2 on B's face x = 0.05, both 0.05 deep; each contact's hash pairs one feature
    (vertex) of each polygon, so the two hashes differ."""
    s = Sandbox()
    a = s.body(0.5, 0.01, (0.0, 0.0)); pa = s.poly(a, box_verts(0.1))
    b = s.body(0.5, 0.01, (0.15, 0.05)); pb = s.poly(b, box_verts(0.1))
    e0 = epa_runs()
    r = s.collide(pa, pb)
    assert epa_runs() == e0 + 1
    assert r["count"] == 2 and r["swapped"] == 0
    assert np.abs(r["n"] - (1.0, 0.0)).max() <= TOL
    assert_contacts(r["con"], [((0.1, 0.1), (0.05, 0.1)), ((0.1, -0.05), (0.05, -0.05))])
    for c in r["con"]:
        assert abs(sep(c, r["n"]) + 0.05) <= TOL
    # hashes: hull order 0 (-h,-h), 1 (h,-h), 2 (h,h), 3 (-h,h); A's support edge toward n is its right face
    # 1 -> 2 (the first max-dot vertex is 1, and face 2's normal beats face 1's), B's toward -n its left face
    # 3 -> 0; contact (e1.a, e2.b) is the lower end, (e1.b, e2.a) the upper (shape hashids A 0, B 1)
    want = {-0.05: hash_pair(hash_pair(0, 1), hash_pair(1, 0)), 0.1: hash_pair(hash_pair(0, 2), hash_pair(1, 3))}
    for (p1, _), h in zip(r["con"], r["hash"]):
        assert h == want[round(float(p1[1]), 6)]
    s.pose(b, 0.03, 0.01)                                             # deep: 0.17 on x beats 0.19 on y
    r = s.collide(pa, pb)
    assert r["count"] == 2 and np.abs(r["n"] - (1.0, 0.0)).max() <= TOL
    assert_contacts(r["con"], [((0.1, 0.1), (-0.07, 0.1)), ((0.1, -0.09), (-0.07, -0.09))])
    for c in r["con"]:
        assert abs(sep(c, r["n"]) + 0.17) <= TOL
    s.pose(b, 0.01, 0.17)                                             # y faces now: n = (0, 1), 0.03 deep
    r = s.collide(pa, pb)
    assert r["count"] == 2 and np.abs(r["n"] - (0.0, 1.0)).max() <= TOL
    assert_contacts(r["con"], [((0.1, 0.1), (0.1, 0.07)), ((-0.09, 0.1), (-0.09, 0.07))])


def test_corner_into_face_one_contact():
    """A box turned 45 degrees pushing its corner 0.02 into another box's top face: one contact (the second
    clipped point lies off the corner's edge, outside the face, with positive separation), n = (0, 1)."""
    s = Sandbox()
    a = s.body(0.5, 0.01, (0.0, 0.0)); pa = s.poly(a, box_verts(0.1))
    b = s.body(0.5, 0.01, (0.0, 0.1 + 0.1 * math.sqrt(2.0) - 0.02), math.pi / 4); pb = s.poly(b, box_verts(0.1))
    r = s.collide(pa, pb)
    assert r["count"] == 1
    assert np.abs(r["n"] - (0.0, 1.0)).max() <= 1e-12
    assert_contacts(r["con"], [((0.0, 0.1), (0.0, 0.08))], tol=1e-12)
    assert abs(sep(r["con"][0], r["n"]) + 0.02) <= 1e-12


def test_rounded_square_bevel_adds_to_depth():
    """SQUARE blocks (create_box with radius 0.01 * side, entities.py:604-620): cores 0.01 * side apart are
    not touching, but the bevels overlap by 0.01 * side -- GJK's distance (no EPA) minus both radii; the
    contact points sit on the bevelled surfaces (face + n * r)."""
    h = SIDE / 2
    s = Sandbox()
    a = s.body(0.5, 0.01, (0.0, 0.0)); pa = s.poly(a, box_verts(h), r=BEVEL)
    gap = 0.01 * SIDE
    b = s.body(0.5, 0.01, (2 * h + gap, 0.0)); pb = s.poly(b, box_verts(h), r=BEVEL)
    e0 = epa_runs()
    r = s.collide(pa, pb)
    assert epa_runs() == e0
    assert r["count"] == 2 and np.abs(r["n"] - (1.0, 0.0)).max() <= TOL
    x1, x2 = h + BEVEL, h + gap - BEVEL
    assert_contacts(r["con"], [((x1, h), (x2, h)), ((x1, -h), (x2, -h))])
    for c in r["con"]:
        assert abs(sep(c, r["n"]) - (gap - 2 * BEVEL)) <= TOL
    s.pose(b, 2 * h + 2 * BEVEL + 1e-9, 0.0)                          # bevels apart
    assert s.collide(pa, pb)["count"] == 0
    # the same bevel against a radius-1 wall (segment-poly): the block's bevel adds to the wall's radius
    w = s.segment((-2.0, -2.0), (2.0, -2.0), 1.0)
    s.pose(b, 0.3, -1.0 + h + BEVEL - 0.004)
    r = s.collide(w, pb)
    assert r["count"] == 2 and r["swapped"] == 0 and np.abs(r["n"] - (0.0, 1.0)).max() <= TOL
    assert_contacts(r["con"], [((0.3 - h, -1.0), (0.3 - h, -1.004)), ((0.3 + h, -1.0), (0.3 + h, -1.004))])


def test_block_pressed_into_wall_segment_poly():
    """SegmentToPoly (a block pushed into an arena wall): two contacts at the block's bottom corners, the wall
    surface 1 above the segment's core, n from the wall to the block, 0.03 deep, no EPA (the cores stay 0.97
    apart)."""
    s = Sandbox()
    w = s.segment((-2.0, -2.0), (2.0, -2.0), 1.0)
    b = s.body(0.5, 0.01, (0.3, -1.0 + 0.1 - 0.03)); p = s.poly(b, box_verts(0.1))
    e0 = epa_runs()
    r = s.collide(p, w)
    assert epa_runs() == e0
    assert r["count"] == 2 and r["swapped"] == 1 and np.abs(r["n"] - (0.0, 1.0)).max() <= TOL
    assert_contacts(r["con"], [((0.2, -1.0), (0.2, -1.03)), ((0.4, -1.0), (0.4, -1.03))])
    # feature hashes, cpCollision.c: the wall edge's ends hash (w, 0) / (w, 1) (the wall's normal points away
    # from n, so its support edge runs tb -> ta), the block's bottom edge its hull vertices 0 -> 1 (hull order
    # from the lowest-x-then-y vertex, CCW); contact 1 pairs (e1.a, e2.b), contact 2 (e1.b, e2.a).  With
    # Chipmunk's XOR pair hash and these small hashids (wall 0, block 1) both contacts hash alike -- as in
    # Chipmunk, whose warm-start match then gives both new contacts the last old contact with that hash.
    wall_id, block_id = 0, 1
    e1a, e1b = hash_pair(wall_id, 1), hash_pair(wall_id, 0)
    e2a, e2b = hash_pair(block_id, 0), hash_pair(block_id, 1)
    assert r["hash"] == [hash_pair(e1a, e2b), hash_pair(e1b, e2a)]
    assert r["hash"][0] == r["hash"][1] == (HASH_COEF * HASH_COEF) % 2 ** 64


def test_contact_hash_identity_across_pose_changes():
    """The feature hash of a contact (HASH_PAIR of the two features' shape-hashid/vertex hashes) is what
    cpArbiterUpdate matches warm starts by: a small move of the same configuration keeps both hashes, a move
    that brings other features into contact changes them."""
    s = Sandbox()
    a = s.body(0.5, 0.01, (0.0, 0.0)); pa = s.poly(a, box_verts(0.1))
    b = s.body(0.5, 0.01, (0.15, 0.05)); pb = s.poly(b, box_verts(0.1))
    h0 = sorted(s.collide(pa, pb)["hash"])
    s.pose(b, 0.151, 0.048, 0.002)
    assert sorted(s.collide(pa, pb)["hash"]) == h0
    s.pose(b, 0.01, 0.17)                                             # top face instead of the right face
    h1 = s.collide(pa, pb)["hash"]
    assert len(h1) == 2 and not set(h1) & set(h0)
    s.pose(b, 0.15, 0.05, math.pi / 2)                                # same place, vertices renumbered
    h2 = s.collide(pa, pb)["hash"]
    assert len(h2) == 2 and sorted(h2) != h0


def _resting_circle(iterations):
    s = Sandbox()
    s.segment((-2.0, -2.0), (2.0, -2.0), 1.0, u=0.8)
    m, r = 0.5, 0.12
    b = s.body(m, 0.5 * m * r * r, (0.25, -1.0 + r - 0.005))       # 0.005 deep: inside collision_slop
    s.circle(b, r, u=0.5)
    s.iterations(iterations)
    return s, b, m


def test_warm_start_reuse_persistence_and_drop():
    """cpArbiterUpdate copies jnAcc / jtAcc into the new contacts by hash; cpArbiterApplyCachedImpulse applies
    them (times dt / prev_dt = 1) unless the arbiter is in its first-collision state; cpSpaceArbiterSetFilter
    caches an arbiter that missed a step and frees it after collisionPersistence = 3 steps.  With the solver
    iterations at 0 the warm start is the only impulse, so it shows exactly in the circle's velocity:
    j = n * jn applied to the wall, -j to the circle: dv = -n * jn / m = (0, jn / m), no spin (r1 along n)."""
    s, b, m = _resting_circle(0)
    s.step()
    assert s.narrowphase_arbiters() == 1
    arb = s.arbiter()
    assert arb["state"] == 0 and arb["count"] == 1 and np.abs(arb["n"] - (0.0, -1.0)).max() <= TOL  # FIRST
    J = 0.01
    s.set_impulse(0, 0, J)
    s.step()                                                          # NORMAL: the cached impulse applies
    st = s.state(b)
    assert st[3] == 0.0 and abs(st[4] - J / m) <= 1e-15 and st[5] == 0.0
    assert s.arbiter()["state"] == 1 and s.arbiter()["con"][0]["jn"] == J
    s.velocity(b, 0.0, 0.0, 0.0)
    s.step()                                                          # again: same hash, same impulse
    assert abs(s.state(b)[4] - J / m) <= 1e-15
    for apart in (1, 2, 3):
        s.velocity(b, 0.0, 0.0, 0.0)
        y0 = s.state(b)[1]
        s.pose(b, 0.25, 0.5)                                          # lifted clear of the wall
        for _ in range(apart):
            s.step()
            assert s.narrowphase_arbiters() == 0
        s.pose(b, 0.25, y0)
        s.velocity(b, 0.0, 0.0, 0.0)
        s.step()
        arb = s.arbiter()
        if apart < 3:      # cached: found again, first-collision state (no cached impulse), jnAcc carried
            assert arb["state"] == 0 and arb["con"][0]["jn"] == J and s.state(b)[4] == 0.0
        else:              # freed after 3 steps: a new arbiter, accumulators from zero
            assert arb["state"] == 0 and arb["con"][0]["jn"] == 0.0 and s.state(b)[4] == 0.0
        s.step()           # the next step applies whatever was carried
        assert abs(s.state(b)[4] - (J / m if apart < 3 else 0.0)) <= 1e-15
        s.set_impulse(0, 0, J)


@pytest.mark.parametrize("vx,saturated", [(1.0, True), (0.05, False)])
def test_friction_is_product_and_clamps(vx, saturated):
    """Friction u = uA * uB (cpArbiterUpdate; circle 0.5 against the wall's 0.8, entities.py:521 / :683):
    a circle (I = m r^2 / 2) arriving at the wall with vy = -0.2 and slip vx.  The normal row stops it in
    one iteration (jn = m |vy|: r1 is along n, nMass = m); the tangent row's impulse jt = (vx + r w) tMass,
    tMass = 1 / (1/m + r^2 / I) = m / 3, is clamped to u jn: saturated for vx = 1 (dvx = -u |vy|,
    dw = -r u jn / I), a rolling contact for vx = 0.05 (dvx = -vx / 3, vx' + r w' = 0)."""
    s, b, m = _resting_circle(10)
    r, vy, u = 0.12, -0.2, 0.5 * 0.8
    I = 0.5 * m * r * r
    s.velocity(b, vx, vy, 0.0)
    s.step()
    arb = s.arbiter()
    assert arb["u"] == 0.5 * 0.8
    st = s.state(b)
    jn = arb["con"][0]["jn"]
    assert abs(jn - m * abs(vy)) <= 1e-15 and abs(st[4]) <= 1e-15
    jt = arb["con"][0]["jt"]
    if saturated:
        assert abs(jt) == u * jn
        assert abs(st[3] - (vx - u * abs(vy))) <= 1e-14
        assert abs(st[5] - (-r * u * jn / I)) <= 1e-12
    else:
        assert abs(jt) < u * jn
        assert abs(st[3] - (vx - vx / 3)) <= 1e-14
        assert abs(st[3] + r * st[5]) <= 1e-14


# ---------------------------------------------------------------- star decomposition ----------------------------

def _area(poly):
    p = np.asarray(poly, dtype=np.float64)
    x, y = p[:, 0], p[:, 1]
    return 0.5 * float(np.sum(x * np.roll(y, -1) - np.roll(x, -1) * y))


def _monotone_hull(points):
    """Andrew's monotone chain (independent of QuickHull): CCW, starting at the lexicographic minimum (the
    lowest x, then the lowest y -- cpConvexHull's first vertex), collinear points dropped."""
    pts = sorted(set(map(tuple, points)))
    if len(pts) <= 2:
        return pts

    def cross(o, a, b):
        return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0])
    lower, upper = [], []
    for p in pts:
        while len(lower) >= 2 and cross(lower[-2], lower[-1], p) <= 0:
            lower.pop()
        lower.append(p)
    for p in reversed(pts):
        while len(upper) >= 2 and cross(upper[-2], upper[-1], p) <= 0:
            upper.pop()
        upper.append(p)
    return lower[:-1] + upper[:-1]


def _star(n_points, out_rad, in_rad):
    """geom.py:49-63 compute_star_verts: outer point i at angle 2 pi i / n of (0, out_rad), inner point
    between them at (2 i + 1) pi / n of (0, in_rad) (rotation of (0, r) by t = (-r sin t, r cos t))"""
    v = []
    for i in range(n_points):
        t = i * 2 * math.pi / n_points
        v.append((-out_rad * math.sin(t), out_rad * math.cos(t)))
        t = (2 * i + 1) * math.pi / n_points
        v.append((-in_rad * math.sin(t), in_rad * math.cos(t)))
    return v


def _on_boundary(p, poly, tol):
    P = np.asarray(poly)
    for k in range(len(P)):
        a, b = P[k], P[(k + 1) % len(P)]
        d = b - a
        t = np.clip(np.dot(p - a, d) / np.dot(d, d), 0.0, 1.0)
        if np.linalg.norm(a + t * d - p) <= tol:
            return True
    return False


def _inside_star(x, star):
    """even-odd ray test against the star polygon itself"""
    P = np.asarray(star)
    inside = False
    for k in range(len(P)):
        a, b = P[k], P[(k + 1) % len(P)]
        if (a[1] > x[1]) != (b[1] > x[1]):
            if a[0] + (x[1] - a[1]) * (b[0] - a[0]) / (b[1] - a[1]) > x[0]:
                inside = not inside
    return inside


def _inside_convex(p, poly):
    P = np.asarray(poly)
    s = [(P[(k + 1) % len(P)][0] - P[k][0]) * (p[1] - P[k][1]) - (P[(k + 1) % len(P)][1] - P[k][1]) * (p[0] - P[k][0])
         for k in range(len(P))]
    return min(s), all(v > 0 for v in s)


@pytest.mark.parametrize("size", [SHAPE_RAD, SHAPE_RAD - 0.01])
def test_star_decomposition_properties(size):
    """autogeom.convex_decomposition of the STAR (entities.py:650-652: 5 points, outer 1.3 size, inner half of
    it), checked without reference to any decomposition code: every part is strictly convex and CCW, every
    part vertex lies on the star's boundary (star vertices or Steiner points on its edges), the parts' areas
    sum to the star's, the parts tile the star (sampled points inside the star lie in exactly one part, points
    outside in none), and each part's physics polygon (pm.Poly -> cpConvexHull, as the GPU library and the
    oracle build it) is the part's convex hull CCW from its lexicographically lowest vertex."""
    from magical_amd import tables
    out_rad = 1.3 * size
    in_rad = 0.5 * out_rad
    star = _star(5, out_rad, in_rad)
    assert np.abs(np.asarray(star) - np.asarray(tables.star_verts(5, out_rad, in_rad))).max() <= 1e-15
    parts = [np.asarray(p) for p in po.star_parts(out_rad, in_rad)]
    assert len(parts) >= 5
    total = 0.0
    for p in parts:
        q = p[:-1] if np.array_equal(p[0], p[-1]) else p
        assert len(q) >= 3
        for k in range(len(q)):
            a, b, c = q[k], q[(k + 1) % len(q)], q[(k + 2) % len(q)]
            assert (b[0] - a[0]) * (c[1] - b[1]) - (b[1] - a[1]) * (c[0] - b[0]) > 0.0, "part not strictly convex CCW"
        for v in q:   # star vertices, or Steiner points of the cuts (on the boundary or inside the star)
            assert _on_boundary(v, star, 1e-12) or _inside_star(v, star), f"part vertex {v} outside the star"
        total += _area(q)
        hull = _monotone_hull(q)
        assert [tuple(v) for v in q] == hull, "part not in cpConvexHull order"
    assert abs(total - _area(star)) <= 1e-15 * 100
    # physics polygons of the GPU library: the hull of each part, first vertex the lexicographic minimum
    phys = tables.block_tables()[tables.STAR]["polys"] if size == SHAPE_RAD else None
    if phys is not None:
        assert len(phys) == len(parts)
        for (verts, rad), p in zip(phys, parts):
            assert rad == 0.0
            assert [tuple(v) for v in verts] == _monotone_hull(p)
    rs = np.random.RandomState(0)
    pts = rs.uniform(-out_rad, out_rad, (20000, 2))
    for x in pts:
        inside_parts, margin = 0, math.inf
        for p in parts:
            q = p[:-1] if np.array_equal(p[0], p[-1]) else p
            m, ins = _inside_convex(x, q)
            margin = min(margin, abs(m))
            inside_parts += ins
        if margin < 1e-9:
            continue
        inside = _inside_star(x, star)
        assert inside_parts == (1 if inside else 0), (x, inside_parts, inside)


# ---------------------------------------------------------------- GPU twin --------------------------------------

import torch  # noqa: E402

# circumradius of each block type (oracle.h SHAPE_*: 1 square incl. its bevel, 2 pentagon, 5 circle, 6 star)
_BLOCK_R = {1: SIDE / 2 * math.sqrt(2.0) + BEVEL, 2: SHAPE_RAD, 5: SHAPE_RAD, 6: 1.3 * SHAPE_RAD}
TWIN = [
    ("ClusterColour-Demo-LoResStack-v0", 48, {}),                      # cooperative form (one env per wavefront)
    ("ClusterColour-Demo-LoResStack-v0", 16, {"MG_STEP_VARIANT": "0"}),  # HBM-state form
    ("MatchRegions-TestAll-LoRes4E-v0", 32, {}),
    ("MoveToCorner-Demo-LoRes4E-v0", 48, {}),                          # robot + one block: the quad form
]


def _twin_layout(kinds, types, poses, rs, robot_first=True):
    """Block poses for one env: blocks in pairs at grid cells away from the robot, the second of a pair at
    0.55-1.0 of the two circumradii from the first in a random direction, both at random angles (face,
    vertex, corner, deep (EPA) and near-miss contacts between every pair of block types); every third block
    pressed into a wall or a corner; one block against the robot's body."""
    robot = [k for k, kd in enumerate(kinds) if kd == 2][0]
    rx, ry = poses[robot][0], poses[robot][1]
    blocks = [k for k, kd in enumerate(kinds) if kd == 3]
    rs.shuffle(blocks)
    cells = [(x, y) for x in (-0.6, 0.0, 0.6) for y in (-0.6, 0.0, 0.6) if math.hypot(x - rx, y - ry) > 0.75]
    rs.shuffle(cells)
    out = {}
    R = lambda b: _BLOCK_R.get(int(types[b]), SHAPE_RAD)  # noqa: E731
    if blocks and robot_first:   # against the robot body (ROBOT_RAD 0.2, base_env.py:62)
        b = blocks.pop()
        t = rs.uniform(0, 2 * math.pi)
        dist = 0.2 + R(b) * rs.uniform(0.55, 1.0)
        out[b] = (rx + dist * math.cos(t), ry + dist * math.sin(t), rs.uniform(-3, 3))
    while blocks:
        if len(blocks) % 3 == 0 or len(blocks) == 1 or not cells:   # into a wall (surfaces at +-1) or a corner
            b = blocks.pop()
            depth = rs.uniform(-0.005, 0.04)
            side = rs.randint(5)
            u = rs.uniform(-0.6, 0.6)
            e = 1.0 - R(b) * rs.uniform(0.7, 1.0) + depth
            out[b] = [(u, -e), (u, e), (-e, u), (e, u), (e * np.sign(u), e)][side] + (rs.uniform(-3, 3),)
            continue
        cx, cy = cells.pop()
        a = blocks.pop()
        out[a] = (cx, cy, rs.uniform(-3, 3))
        if blocks:
            b = blocks.pop()
            t = rs.uniform(0, 2 * math.pi)
            dist = (R(a) + R(b)) * rs.uniform(0.55, 1.0)
            out[b] = (cx + dist * math.cos(t), cy + dist * math.sin(t), rs.uniform(-3, 3))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,env", TWIN, ids=[t[0].split("-")[0] + "".join(f"-{k}{v}" for k, v in t[2].items())
                                                   for t in TWIN])
def test_gpu_narrowphase_twin(name, n, env, monkeypatch):
    """Blocks placed into contact configurations (Body.position / angle setters on both sides), then 6
    steps: after every step the GPU's arbiter table (slots, first-collision / normal states, contact counts,
    bodies, normals, friction, r1 / r2, accumulated impulses, masses, biases, feature hashes) and bodies equal
    the oracle's, whose narrowphase the known answers above pin."""
    from magical_amd import registry
    import magical_amd
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    spec = registry.lookup(name)
    seeds = [9100 + i for i in range(n)]
    vec = magical_amd.make_vec(name, n, seeds=seeds)
    vec.reset()
    orc, rob = [], []
    for i in range(n):
        o = po.OracleEnv(spec.task, spec.rand_flags, spec.preproc, spec.max_episode_steps, seed=seeds[i])
        o.reset()
        kinds, types, cols, poses = o.entities()
        body0, nb = {}, 0
        for k, kind in enumerate(kinds):   # bodies in entity add order: blocks 1, robot 6, others 0
            body0[k] = nb
            nb += 1 if kind == 3 else 6 if kind == 2 else 0
        r0 = body0[[k for k, kind in enumerate(kinds) if kind == 2][0]]
        rob.append(set(range(r0, r0 + 6)))
        for b, (x, y, a) in _twin_layout(kinds, types, poses, np.random.RandomState(i),
                                                 robot_first=i % 2 == 0).items():
            o.set_body_pose(body0[b], x, y, a)
            vec.set_body_pose(i, body0[b], x, y, a)
        orc.append(o)
    acts = np.random.RandomState(5).randint(0, 18, (6, n))
    e0 = epa_runs()
    seen = dict(arbiters=0, two=0, one=0, wall=0, block_block=0, robot=0)
    for t in range(6):
        vec.step(torch.as_tensor(acts[t], dtype=torch.uint8))
        bodies, counts = vec.bodies()
        arbs, hs = vec.arbiters()
        bodies, counts, arbs, hs = bodies.cpu().numpy(), counts.cpu().numpy(), arbs.cpu().numpy(), hs.cpu().numpy()
        for i in range(n):
            o = orc[i]
            o.step(int(acts[t, i]))
            b = o.bodies()
            assert np.abs(bodies[i, :len(b)] - b).max() <= 1e-9, f"step {t} env {i} bodies"
            ra, rh = o.arbiters()
            na = len(ra)
            assert counts[i, 3] == na, f"step {t} env {i}: {counts[i, 3]} arbiters vs {na}"
            for k in range(na):
                g, w = arbs[i, k], ra[k]
                assert np.array_equal(g[:5], w[:5]), f"step {t} env {i} arbiter {k}: {g[:5]} vs {w[:5]}"
                cnt = int(w[2])
                assert np.abs(g[5:8 + 10 * cnt] - w[5:8 + 10 * cnt]).max() <= 1e-9, f"step {t} env {i} arbiter {k}"
                assert np.array_equal(hs[i, k, :cnt], rh[k, :cnt]), f"step {t} env {i} arbiter {k} hashes"
                seen["arbiters"] += 1
                seen["two" if cnt == 2 else "one"] += 1
                ba, bb = int(w[3]), int(w[4])
                seen["wall"] += ba < 0 or bb < 0
                seen["robot"] += (ba in rob[i]) != (bb in rob[i])
                seen["block_block"] += ba >= 0 and bb >= 0 and ba not in rob[i] and bb not in rob[i]
    need = [k for k in seen if k != "block_block" or spec.task != "MoveToCorner"]   # MoveToCorner: one block
    assert min(seen[k] for k in need) > 0 and seen["arbiters"] >= 2 * n, seen
    assert epa_runs() > e0, "no configuration took the EPA path"
    print(name, env, seen, "EPA runs", epa_runs() - e0)
    assert int(vec.errors().abs().sum().item()) == 0
    vec.close()

