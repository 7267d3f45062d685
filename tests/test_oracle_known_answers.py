"""Known-answer tests of the oracle's Chipmunk-7 and pygame-1.9.6 restatements.

The reference's arithmetic for physics and rasterisation lives in pymunk 5.6 (Chipmunk2D 7.0.x)
and pygame 1.9.6, neither of which exists in this image, and the reference's own tests hold no
golden vectors for them (tests/test_rollout_preproc.py:33 asserts only episode length).  These
tests pin the restatement (oracle/phys.c, oracle/raster.c) to analytic behaviour instead:

physics (the constants base_env.py:206-208 and entities.py set):
  * free flight integrates p += v dt, a += w dt exactly;
  * the robot's PivotJoint (maxBias 0, maxForce 3) drags the body to the control body's
    velocity at exactly maxForce dt / m per step (entities.py:312-320);
  * its GearJoint (errorBias 0, maxBias 2.5, maxForce 1) ramps the turn rate the same way;
  * a contact's bias velocity shrinks a penetration to collision_slop geometrically with ratio
    (1 - biasCoef), biasCoef = 1 - (0.9^60)^dt, without moving the body's real velocity; a
    penetration below the slop never moves anything;
  * RotaryLimitJoint (errorBias 0) puts the body back on the limit in one step;
  * SimpleMotor holds b.w - a.w = -rate, and ramps at maxForce dt / I when force-limited;
  * DampedRotarySpring damps the relative spin by exp(-c dt / I) per step (the analytic decay at
    step times) and oscillates with period 2 pi sqrt(I / k).

raster (pygame 1.9.6 draw.c):
  * draw_fillpoly fills the last row and truncates edge intersections toward zero;
  * drawline's Bresenham pixel sequence; width 2/4 offsets; Cohen-Sutherland with a float32 slope;
  * the dashed goal outline's dash endpoints equal the calls the reference's own
    Poly._render / draw_outline (render.py:202-287) makes -- fixture tests/golden/ref_outline.json,
    produced by executing that code (tests/golden/make_ref_fixtures.py).
"""
import ctypes
import json
import math
import os

import numpy as np
import pytest

import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
DT = 1.0 / 8 / 10                     # benchmarks/__init__.py:435 fps=8, base_env.py:248 phys_steps=10
BIAS_COEF = 1.0 - (0.9 ** 60) ** DT  # cpSpace collisionBias default, SURVEY.md A.2 step 8
SLOP = 0.01                           # base_env.py:207
DYN, KIN = 0, 1
PIVOT, GEAR, ROTLIMIT, MOTOR, SPRING = 0, 1, 2, 3, 4

d, i_, vp = ctypes.c_double, ctypes.c_int, ctypes.c_void_p


def _lib():
    L = po.lib()
    if not getattr(L, "_osb_ready", False):
        L.osb_new.restype = vp
        L.osb_free.argtypes = [vp]
        L.osb_add_body.restype = i_; L.osb_add_body.argtypes = [vp, i_, d, d, d, d, d]
        L.osb_set_velocity.argtypes = [vp, i_, d, d, d]
        L.osb_get_body.argtypes = [vp, i_, vp]
        L.osb_add_circle.restype = i_; L.osb_add_circle.argtypes = [vp, i_, d, d, d, d]
        L.osb_add_segment.restype = i_; L.osb_add_segment.argtypes = [vp, d, d, d, d, d, d]
        L.osb_add_poly.restype = i_; L.osb_add_poly.argtypes = [vp, i_, i_, vp, d, d]
        L.osb_add_constraint.restype = i_; L.osb_add_constraint.argtypes = [vp, i_, i_, i_, d, d, d]
        L.osb_set_constraint.argtypes = [vp, i_, d, d, d]
        L.osb_constraint_impulse.restype = d; L.osb_constraint_impulse.argtypes = [vp, i_]
        L.osb_step.argtypes = [vp, d]
        L.osb_num_arbiters.restype = i_; L.osb_num_arbiters.argtypes = [vp]
        L.osb_arbiter.restype = i_; L.osb_arbiter.argtypes = [vp, i_, vp]
        L.o_fill_poly.argtypes = [vp, vp, vp, i_, vp]
        L.o_clipline.restype = i_; L.o_clipline.argtypes = [vp]
        L.o_line_width.argtypes = [vp, vp, i_, vp]
        L.o_dash_segments.restype = i_; L.o_dash_segments.argtypes = [d, d, d, d, vp, i_]
        L._osb_ready = True
    return L


class Space:
    def __init__(self):
        self.L = _lib()
        self.h = self.L.osb_new()

    def __del__(self):
        if getattr(self, "h", None):
            self.L.osb_free(self.h)

    def body(self, m, i, p=(0.0, 0.0), a=0.0, kind=DYN):
        return self.L.osb_add_body(self.h, kind, m, i, p[0], p[1], a)

    def velocity(self, b, vx, vy, w):
        self.L.osb_set_velocity(self.h, b, vx, vy, w)

    def state(self, b):
        out = np.zeros(9)
        self.L.osb_get_body(self.h, b, po.ptr(out))
        return out

    def circle(self, b, r, u=0.5):
        return self.L.osb_add_circle(self.h, b, r, 0.0, 0.0, u)

    def segment(self, a, b, r, u=0.8):
        return self.L.osb_add_segment(self.h, a[0], a[1], b[0], b[1], r, u)

    def poly(self, b, verts, r=0.0, u=0.5):
        v = np.ascontiguousarray(verts, dtype=np.float64)
        return self.L.osb_add_poly(self.h, b, len(v), po.ptr(v), r, u)

    def cons(self, kind, a, b, p0=0.0, p1=0.0, p2=0.0, max_force=math.inf, max_bias=math.inf,
             error_bias=0.9 ** 60):
        c = self.L.osb_add_constraint(self.h, kind, a, b, p0, p1, p2)
        self.L.osb_set_constraint(self.h, c, max_force, max_bias, error_bias)
        return c

    def step(self, dt=DT):
        self.L.osb_step(self.h, dt)


# ---------------------------------------------------------------- physics ---------------------------------------

def test_free_flight_integrates_exactly():
    """cpBodyUpdatePosition: p += (v + v_bias) dt, a += (w + w_bias) dt; no gravity, damping 1
    (base_env.py:206) => velocity constant, position a plain running sum."""
    s = Space()
    b = s.body(0.5, 0.0036, (0.1, -0.2), 0.3)
    s.velocity(b, 0.7, -0.4, 1.1)
    px, py, a = 0.1, -0.2, 0.3
    for _ in range(400):
        s.step()
        px += 0.7 * DT; py += -0.4 * DT; a += 1.1 * DT
    st = s.state(b)
    assert (st[0], st[1], st[2]) == (px, py, a)
    assert (st[3], st[4], st[5]) == (0.7, -0.4, 1.1)
    assert abs(st[0] - (0.1 + 400 * 0.7 * DT)) < 1e-12 and abs(st[2] - (0.3 + 400 * 1.1 * DT)) < 1e-12


def test_robot_pivot_reaches_control_velocity_at_max_force():
    """Robot translation (entities.py:312-320): PivotJoint(control, body) with maxBias 0 and
    maxForce robot_pos_joint_max_force = 3.  With m = 1 each step adds exactly maxForce * dt = 0.0375
    to the speed (the warm-started impulse is re-clamped every step) until it equals the kinematic
    control body's 0.8 (UP, entities.py:443) -- then stays there exactly."""
    s = Space()
    ctl = s.body(math.inf, math.inf, kind=KIN)
    body = s.body(1.0, 0.02)
    s.cons(PIVOT, ctl, body, 0.0, 0.0, max_force=3.0, max_bias=0.0)
    s.velocity(ctl, 0.0, 0.8, 0.0)
    for k in range(1, 60):
        s.step()
        vy = s.state(body)[4]
        assert abs(vy - min(0.8, 3.0 * DT * k)) < 1e-12, (k, vy)
        assert s.state(body)[3] == 0.0


def test_robot_gear_turn_rate_ramps_and_converges():
    """Robot rotation (entities.py:321-327): GearJoint(control, body) with errorBias 0 (bias
    coefficient 1), maxBias 2.5 and maxForce robot_rot_joint_max_force = 1: the turn rate grows by
    maxForce dt / I = 0.625 rad/s per step up to maxBias, then the angle converges onto the control
    body's (LEFT: +1.5 rad, entities.py:447)."""
    s = Space()
    ctl = s.body(math.inf, math.inf, a=1.5, kind=KIN)
    body = s.body(1.0, 0.02)
    s.cons(GEAR, ctl, body, 0.0, 1.0, max_force=1.0, max_bias=2.5, error_bias=0.0)
    ws = []
    for k in range(1, 200):
        s.step()
        ws.append(s.state(body)[5])
    assert np.allclose(ws[:4], [0.625, 1.25, 1.875, 2.5], rtol=0, atol=1e-12)
    assert max(np.abs(np.diff(ws))) <= 0.625 + 1e-12
    assert max(ws) <= 2.5 + 1e-12
    st = s.state(body)
    assert abs(st[2] - 1.5) < 1e-9 and abs(st[5]) < 1e-9


def _wall_and_circle(pen):
    s = Space()
    s.segment((-2.0, -2.0), (2.0, -2.0), 1.0)         # arena wall: radius 1, surface at y = -1 (entities.py:498-533)
    b = s.body(0.5, 0.0036, (0.25, -1.0 + 0.12 - pen))  # circle block, SHAPE_RAD 0.12 (entities.py:580-754)
    s.circle(b, 0.12)
    return s, b


def test_contact_bias_pushes_penetration_to_slop_geometrically():
    """Circle resting on a wall, penetrating by 0.05: one contact through the centre, so the bias
    impulse solves exactly -- each step's bias velocity (applied by the next step's position integration,
A.2 steps 3 and 11) moves the body out by biasCoef * (penetration - slop).  The
    real velocity stays 0 (bias velocities are separate and cleared after integration, A.1/A.2)."""
    pen0 = 0.05
    s, b = _wall_and_circle(pen0)
    y_rest = -1.0 + 0.12 - SLOP
    for k in range(1, 121):
        s.step()
        st = s.state(b)
        deficit = (y_rest - st[1])
        assert abs(deficit - (pen0 - SLOP) * (1 - BIAS_COEF) ** (k - 1)) < 1e-12, k
        assert st[3] == 0.0 and st[4] == 0.0 and st[5] == 0.0
        assert st[0] == 0.25 and st[2] == 0.0
    assert s.L.osb_num_arbiters(s.h) == 1


def test_contact_within_slop_never_moves():
    """Penetration 0.005 < collision_slop: bias = -biasCoef * min(0, d + slop) / dt = 0, no impulse,
    the block stays put to the last bit over 500 steps (no drift)."""
    s, b = _wall_and_circle(0.005)
    st0 = s.state(b)
    for _ in range(500):
        s.step()
    assert np.array_equal(s.state(b), st0)


def test_box_on_wall_rises_to_slop_without_rotating():
    """A SQUARE block (Poly.create_box with radius 0.01 side, entities.py:604-620) sunk 0.03 into a
    wall: two contacts (segment-poly ContactPoints, A.3), symmetric, so the block moves straight up to
    penetration = slop with no rotation and no sideways drift."""
    side = math.sqrt(math.pi) * 0.12
    r = 0.01 * side
    h = side / 2
    s = Space()
    s.segment((-2.0, -2.0), (2.0, -2.0), 1.0)
    b = s.body(0.5, 0.5 * (side * side) / 6.0, (0.0, -1.0 + h + r - 0.03))
    s.poly(b, [(-h, -h), (h, -h), (h, h), (-h, h)], r)
    for _ in range(300):
        s.step()
    st = s.state(b)
    pen = (-1.0 + h + r) - st[1]
    assert abs(pen - SLOP) < 1e-9
    assert abs(st[0]) < 1e-12 and abs(st[2]) < 1e-12 and np.abs(st[3:6]).max() < 1e-12
    out = np.zeros(14)
    assert s.L.osb_arbiter(s.h, 0, po.ptr(out)) == 2


def test_rotary_limit_returns_body_to_limit_in_one_step():
    """RotaryLimitJoint(static, finger, 0, pi/8) with errorBias 0 (entities.py:342-352): the step
    after the angle passes max, bias = (d - max) / dt and the solved spin lands the angle on max."""
    s = Space()
    f = s.body(0.125, 0.0050065)
    s.velocity(f, 0.0, 0.0, 5.0)
    s.cons(ROTLIMIT, -1, f, 0.0, math.pi / 8, error_bias=0.0)
    prev = 0.0
    for k in range(1, 40):
        s.step()
        a = s.state(f)[2]
        if prev > math.pi / 8:
            assert abs(a - math.pi / 8) < 1e-12, (k, a)
            assert abs(s.state(f)[5] - (math.pi / 8 - prev) / DT) < 1e-9
            break
        assert a <= math.pi / 8 + 5.0 * DT
        prev = a
    else:
        pytest.fail("the limit was never reached")


def test_simple_motor_holds_rate_and_ramps_when_force_limited():
    """SimpleMotor (entities.py:353-361): drives b.w - a.w to -rate; unlimited it gets there in the
    first step, with maxForce F it ramps by F dt / I per step (A.5)."""
    s = Space()
    f = s.body(0.125, 0.005)
    s.cons(MOTOR, -1, f, 2.0)
    s.step()
    assert abs(s.state(f)[5] + 2.0) < 1e-12
    s = Space()
    f = s.body(0.125, 0.005)
    s.cons(MOTOR, -1, f, -1.0, max_force=0.1)
    for k in range(1, 12):
        s.step()
        assert abs(s.state(f)[5] - min(1.0, k * 0.1 * DT / 0.005)) < 1e-12, k


def test_damped_rotary_spring_decays_as_exp():
    """DampedRotarySpring with k = 0 (entities.py:296-306, the eye springs): the damping term applies
    once per step with w_coef = 1 - exp(-c dt (1/Ia + 1/Ib)) (A.5), i.e. the analytic decay
    w(t) = w0 exp(-c t / I) sampled at step times."""
    s = Space()
    eye = s.body(0.1, 0.002)
    s.velocity(eye, 0.0, 0.0, 1.0)
    s.cons(SPRING, -1, eye, 0.0, 0.0, 3e-3)
    for k in range(1, 300):
        s.step()
        w = s.state(eye)[5]
        assert abs(w - math.exp(-3e-3 * k * DT / 0.002)) < 1e-12 * max(1.0, k), k


def test_rotary_spring_oscillation_period():
    """DampedRotarySpring with stiffness k and no damping: the explicit spring impulse plus symplectic
    integration oscillates with period 2 pi sqrt(I / k) (to the step's O(dt^2) phase error)."""
    s = Space()
    I, k = 0.002, 0.1
    eye = s.body(0.1, I, a=0.2)
    s.cons(SPRING, -1, eye, 0.0, k, 0.0)
    angles = []
    for _ in range(1000):
        s.step()
        angles.append(s.state(eye)[2])
    angles = np.array(angles)
    up = np.where((angles[:-1] < 0) & (angles[1:] >= 0))[0]
    period = np.diff(up).mean() * DT
    assert abs(period - 2 * math.pi * math.sqrt(I / k)) / (2 * math.pi * math.sqrt(I / k)) < 0.01
    assert np.abs(angles).max() < 0.2 * 1.01


# ---------------------------------------------------------------- raster ----------------------------------------

RES = 384
BG = np.array([1, 2, 3], np.uint8)
COL = np.array([200, 100, 50], np.uint8)


def _frame():
    f = np.zeros((RES, RES, 3), np.uint8)
    f[:] = BG
    return f


def _mask(f):
    return np.all(f == COL, axis=2)


def _fill(vx, vy):
    f = _frame()
    x = np.ascontiguousarray(vx, np.int32)
    y = np.ascontiguousarray(vy, np.int32)
    _lib().o_fill_poly(po.ptr(f), po.ptr(x), po.ptr(y), len(x), po.ptr(COL))
    return _mask(f)


def _line(pts, width):
    f = _frame()
    p = np.ascontiguousarray(pts, np.int32)
    _lib().o_line_width(po.ptr(f), po.ptr(COL), width, po.ptr(p))
    return _mask(f)


def test_fillpoly_rectangle_includes_last_row():
    """pygame 1.9.6 draw_fillpoly: rows miny..maxy, the last row through the (y == maxy) rule, columns
    inclusive: the closed rectangle (10,20)-(30,25) covers 21 x 6 pixels (pygame 2 differs here)."""
    m = _fill([10, 30, 30, 10, 10], [20, 20, 25, 25, 20])
    ys, xs = np.nonzero(m)
    assert m.sum() == 21 * 6 and ys.min() == 20 and ys.max() == 25 and xs.min() == 10 and xs.max() == 30


def test_fillpoly_truncates_toward_zero():
    """x = (y - y1) (x2 - x1) / (y2 - y1) + x1 with C integer division: a negative-slope edge rounds
    its intersection toward zero (up in x), not down as floor division would."""
    m = _fill([0, 7, 0, 0], [0, 10, 10, 0])   # right edge from (0,0) to (7,10)
    for y in range(0, 10):
        right = (y * 7) // 10                   # positive numerator: trunc == floor
        assert np.nonzero(m[y])[0].max() == right
    m = _fill([7, 0, 7, 7], [0, 10, 10, 0])   # left edge from (7,0) to (0,10): numerator (y)(-7) < 0
    for y in range(1, 10):
        left = 7 + int(-7 * y / 10)             # C: truncation toward zero
        assert np.nonzero(m[y])[0].min() == left, y
        assert left != 7 + (-7 * y) // 10 or (7 * y) % 10 == 0


def test_fillpoly_clips_off_screen_spans():
    m = _fill([-50, 500, 500, -50, -50], [-5, -5, 3, 3, -5])
    assert m[:4].all() and not m[4:].any()


def test_bresenham_pixel_sequence():
    """drawline: deltax = |dx| + 1 major steps, error += deltay, minor step when error >= deltax."""
    m = _line([0, 0, 5, 2], 1)
    assert sorted(zip(*np.nonzero(m.T))) == [(0, 0), (1, 0), (2, 1), (3, 1), (4, 2), (5, 2)]
    m = _line([3, 0, 1, 5], 1)                 # steep, negative x
    assert sorted(zip(*np.nonzero(m.T)), key=lambda p: p[1]) == [(3, 0), (3, 1), (2, 2), (2, 3), (1, 4), (1, 5)]


def test_line_width_offsets():
    """clip_and_draw_line_width: +1 offset copy (y for x-major lines, x otherwise) for width 2,
    offsets 0, +1, -1, +2 for width 4 (the dashed goal outline)."""
    m = _line([10, 50, 40, 50], 2)
    assert set(np.nonzero(m)[0]) == {50, 51} and m.sum() == 2 * 31
    m = _line([100, 10, 100, 40], 4)
    assert set(np.nonzero(m)[1]) == {99, 100, 101, 102} and m.sum() == 4 * 31
    m = _line([0, 0, 30, 0], 4)                # the -1 copy falls off the top edge and is clipped
    assert set(np.nonzero(m)[0]) == {0, 1, 2}


def _clip(x1, y1, x2, y2, f32=np.float32):
    """Cohen-Sutherland of pygame 1.9.6 draw.c clipline on [0, 383]^2 with the float32 slope."""
    L_, R_, B_, T_ = 1, 2, 4, 8

    def enc(x, y):
        return (L_ if x < 0 else 0) | (R_ if x > 383 else 0) | (T_ if y < 0 else 0) | (B_ if y > 383 else 0)
    while True:
        c1, c2 = enc(x1, y1), enc(x2, y2)
        if not (c1 | c2):
            return (x1, y1, x2, y2)
        if c1 & c2:
            return None
        if not c1:
            x1, y1, x2, y2, c1 = x2, y2, x1, y1, c2
        m = f32(f32(y2 - y1) / f32(x2 - x1)) if x2 != x1 else f32(1.0)
        if c1 & L_:
            y1 += int(f32(f32(0 - x1) * m)); x1 = 0
        elif c1 & R_:
            y1 += int(f32(f32(383 - x1) * m)); x1 = 383
        elif c1 & B_:
            if x2 != x1:
                x1 += int(f32(f32(383 - y1) / m))
            y1 = 383
        elif c1 & T_:
            if x2 != x1:
                x1 += int(f32(f32(0 - y1) / m))
            y1 = 0


def test_cohen_sutherland_clip_uses_float32_slope():
    rs = np.random.RandomState(5)
    L = _lib()
    differs = 0
    cases = [rs.randint(-3000, 3400, 4) for _ in range(3000)]
    # lines entering through the left edge: where the float32 slope's truncated intercept differs
    cases += [np.array([rs.randint(-2000, 0), rs.randint(-400, 800), rs.randint(0, 384), rs.randint(0, 384)])
              for _ in range(20000)]
    cases.append(np.array([-809, 954, 0, 36]))   # float32: y = 36, float64: y = 37
    for pts in cases:
        got = np.ascontiguousarray(pts, np.int32)
        ok = L.o_clipline(po.ptr(got))
        want = _clip(*[int(v) for v in pts])
        assert (ok == 1) == (want is not None)
        if want is not None:
            assert tuple(got) == want, (pts, tuple(got), want)
            differs += want != _clip(*[int(v) for v in pts], f32=np.float64)
    assert differs > 0, "no case separated the float32 slope from a float64 one"
    inside = np.array([5, 6, 300, 200], np.int32)
    assert L.o_clipline(po.ptr(inside)) == 1 and tuple(inside) == (5, 6, 300, 200)


def test_dashed_and_solid_outline_calls_match_reference_render():
    """render.py:202-287 executed on pixel-space goal rectangles (allo and ego views), random quads and
    exact axis-aligned / .5-tie edges: the dashed branch's pygame.draw.line(start, end, 4) calls --
    np.arange stepping, Python round() half-even, zip truncation -- equal the oracle's dash list, and the
    solid branch draws each edge as lines([a, b], 2)."""
    with open(os.path.join(HERE, "golden", "ref_outline.json")) as f:
        cases = json.load(f)["cases"]
    L = _lib()
    seg = np.zeros(4 * 256, np.int32)
    ndash = 0
    for c in cases:
        pts = np.array(c["pts"]).reshape(-1, 2)
        calls = c["calls"]
        assert calls[0][0] == "polygon" and calls[0][1] == pts.tolist() + [pts[0].tolist()]
        edges = [(pts[i], pts[(i + 1) % len(pts)]) for i in range(len(pts))]
        if not c["dashed"]:
            assert [cl[0] for cl in calls[1:]] == ["lines"] * len(edges)
            for cl, (a, b) in zip(calls[1:], edges):
                assert cl[1] == [a.tolist(), b.tolist()] and cl[2] == 2 and cl[3] is False
            continue
        want = [cl for cl in calls[1:]]
        assert all(cl[0] == "line" and cl[2] == 4 for cl in want)
        got = []
        for a, b in edges:
            n = L.o_dash_segments(a[0], a[1], b[0], b[1], po.ptr(seg), 256)
            got += [[[float(seg[4 * k]), float(seg[4 * k + 1])], [float(seg[4 * k + 2]), float(seg[4 * k + 3])]]
                    for k in range(n)]
        assert got == [cl[1] for cl in want], c["pts"]
        ndash += len(got)
    assert ndash > 1000
