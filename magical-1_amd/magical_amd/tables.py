"""Scene library for the GPU simulator, built from MAGICAL's own formulas.

Everything here is evaluated once on the host and copied to the device as an
``mg_library`` (layout: magical-1_amd/csrc/mg_common.h).  Each value follows the
reference expression it cites, with the reference's operation order:

* robot geometry / masses: entities.py:238-433 (make_finger_vertices :193-214)
* block geometry / masses: entities.py:580-754, geom.py:13-63
* pymunk/Chipmunk details: Poly() runs cpConvexHull on its vertices,
  Poly.create_box keeps the raw (r,b),(r,t),(l,t),(l,b) order, the star uses
  pymunk.autogeometry.convex_decomposition (cpPolylineConvexDecomposition_BETA)
  and to_convex_hull, moments use cpMomentForPoly / cpMomentForCircle
* render polygons and transform chains: render.py:13-36, entities.py:374-433,
  524-533, 710-749, 793-801; views: base_env.py:309-322, render.py:290-371
* palette: style.py (colorsys lighten / darken)

sin / cos / tan are evaluated correctly rounded (decimal arithmetic), the libm
behaviour of the reference's era; 3x3 products use numpy matmul exactly as
render.py does.
"""
import colorsys
import ctypes
import math
from decimal import Decimal, localcontext

import numpy as np

# ---------------------------------------------------------------------------
# constants shared with mg_common.h
MAX_PVERTS = 8
MAX_LIB_POLYS = 32
MAX_RPOLYS = 64
MAX_RPTS = 2400
MAX_STATIC_XF = 8
NUM_SHAPE_TYPES = 7

TRIANGLE, SQUARE, PENTAGON, HEXAGON, OCTAGON, CIRCLE, STAR = range(7)
RED, GREEN, BLUE, YELLOW, GREY = range(5)
SHAPE_TYPE_NAMES = {"triangle": TRIANGLE, "square": SQUARE, "pentagon": PENTAGON, "hexagon": HEXAGON,
                    "octagon": OCTAGON, "circle": CIRCLE, "star": STAR}
COLOUR_NAMES = {"red": RED, "green": GREEN, "blue": BLUE, "yellow": YELLOW, "grey": GREY}
RC_ENT_BASE, RC_ENT_DARK, RC_ENT_LIGHT2, RC_GREY_BASE, RC_GREY_DARK, RC_GREY_LIGHT4, RC_WHITE, RC_PUPIL = range(8)
XF_MAIN, XF_FINGER_L, XF_FINGER_R, XF_PUPIL_L, XF_PUPIL_R = range(5)
XF_STATIC0 = 8
OUTLINE_NONE, OUTLINE_SOLID, OUTLINE_DASHED = range(3)


class mg_rpoly(ctypes.Structure):
    _fields_ = [("npts", ctypes.c_int32), ("pts_off", ctypes.c_int32), ("outline", ctypes.c_int32),
                ("col_ref", ctypes.c_int32), ("ocol_ref", ctypes.c_int32), ("nxf", ctypes.c_int32),
                ("xf", ctypes.c_int32 * 4)]


_d = ctypes.c_double
_i = ctypes.c_int32


class mg_library(ctypes.Structure):
    _fields_ = [
        ("dt", _d), ("collision_bias_coef", _d), ("slop", _d), ("default_bias_coef", _d), ("spring_w_coef", _d),
        ("robot_radius", _d), ("robot_mass", _d), ("robot_inertia", _d), ("eye_mass", _d), ("eye_inertia", _d),
        ("finger_mass", _d), ("finger_inertia", _d * 2), ("finger_rel", (_d * 2) * 2), ("finger_lim", (_d * 2) * 2),
        ("finger_angle_off", _d * 2), ("finger_poly", _i * 4),
        ("block_nshapes", _i * NUM_SHAPE_TYPES), ("block_poly", (_i * 8) * NUM_SHAPE_TYPES),
        ("block_mass", _d * NUM_SHAPE_TYPES), ("block_inertia", _d * NUM_SHAPE_TYPES), ("block_circle_r", _d),
        ("n_polys", _i), ("poly_count", _i * MAX_LIB_POLYS), ("poly_r", _d * MAX_LIB_POLYS),
        ("poly_v", ((_d * 2) * MAX_PVERTS) * MAX_LIB_POLYS), ("poly_n", ((_d * 2) * MAX_PVERTS) * MAX_LIB_POLYS),
        ("n_rpolys", _i), ("rpoly", mg_rpoly * MAX_RPOLYS), ("rpts", (_d * 2) * MAX_RPTS),
        ("arena_rpoly0", _i), ("arena_nrpoly", _i), ("goal_rpoly0", _i), ("goal_nrpoly", _i),
        ("robot_rpoly0", _i), ("robot_nrpoly", _i),
        ("block_rpoly0", _i * NUM_SHAPE_TYPES), ("block_nrpoly", _i * NUM_SHAPE_TYPES),
        ("static_xf", (_d * 9) * MAX_STATIC_XF), ("allo_view", _d * 9),
        ("ego_scale_m", _d * 9), ("ego_tr1_m", _d * 9), ("pygame_m", _d * 9),
        ("palette", ((ctypes.c_uint8 * 4) * 4) * 5),
        ("white", ctypes.c_uint8 * 4), ("pupil", ctypes.c_uint8 * 4), ("background", ctypes.c_uint8 * 4),
    ]


# ---------------------------------------------------------------------------
# correctly rounded trigonometry (decimal, 50 digits)
_PI_STR = ("3.14159265358979323846264338327950288419716939937510582097494459230781640628620899862803482534"
           "211706798214808651328230664709384460955058223172535940812848111745028410270193852110555964462")


def _dec_sincos(x):
    with localcontext() as ctx:
        ctx.prec = 70
        pi = Decimal(_PI_STR)
        d = Decimal(x)
        two_pi = 2 * pi
        k = (d / two_pi).to_integral_value()
        r = d - k * two_pi
        r2 = r * r
        s = term = r
        n = 1
        while True:
            term = -term * r2 / ((n + 1) * (n + 2))
            n += 2
            if abs(term) < Decimal(10) ** -68:
                break
            s += term
        c = term = Decimal(1)
        n = 0
        while True:
            term = -term * r2 / ((n + 1) * (n + 2))
            n += 2
            if abs(term) < Decimal(10) ** -68:
                break
            c += term
        return s, c


def crsin(x):
    if x == 0.0:
        return x
    return float(_dec_sincos(x)[0])


def crcos(x):
    return float(_dec_sincos(x)[1])


def crtan(x):
    s, c = _dec_sincos(x)
    with localcontext() as ctx:
        ctx.prec = 70
        return float(s / c)


def rotated(v, angle):
    """pymunk 5.6 Vec2d.rotated: (x cos - y sin, x sin + y cos)."""
    c, s = crcos(angle), crsin(angle)
    x, y = v
    return (x * c - y * s, x * s + y * c)


# ---------------------------------------------------------------------------
# Chipmunk helpers restated in Python (chipmunk.c / cpPolyline.c / cpPolyShape.c)
def _cross(a, b):
    return a[0] * b[1] - a[1] * b[0]


def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def convex_hull(verts, tol=0.0):
    """cpConvexHull (QuickHull); returns (hull, first)."""
    res = [tuple(v) for v in verts]
    count = len(res)
    start = end = 0
    mn = mx = res[0]
    for i in range(1, count):
        v = res[i]
        if v[0] < mn[0] or (v[0] == mn[0] and v[1] < mn[1]):
            mn = v
            start = i
        elif v[0] > mx[0] or (v[0] == mx[0] and v[1] > mx[1]):
            mx = v
            end = i
    if start == end:
        return [res[0]], 0
    res[0], res[start] = res[start], res[0]
    j = start if end == 0 else end
    res[1], res[j] = res[j], res[1]
    a, b = res[0], res[1]

    def partition(lo, count_, a_, b_):
        if count_ == 0:
            return 0
        mxv, pivot = 0.0, 0
        delta = _sub(b_, a_)
        value_tol = tol * math.sqrt(delta[0] * delta[0] + delta[1] * delta[1])
        head, tail = 0, count_ - 1
        while head <= tail:
            value = _cross(_sub(res[lo + head], a_), delta)
            if value > value_tol:
                if value > mxv:
                    mxv, pivot = value, head
                head += 1
            else:
                res[lo + head], res[lo + tail] = res[lo + tail], res[lo + head]
                tail -= 1
        if pivot != 0:
            res[lo], res[lo + pivot] = res[lo + pivot], res[lo]
        return head

    out = []

    def reduce(lo, count_, a_, pivot, b_):
        if count_ < 0:
            return
        if count_ == 0:
            out.append(pivot)
            return
        left = partition(lo, count_, a_, pivot)
        reduce(lo + 1, left - 1, a_, res[lo] if lo < len(res) else None, pivot)
        out.append(pivot)
        right = partition(lo + left, count_ - left, pivot, b_)
        nxt = res[lo + left] if lo + left < len(res) else None  # unused when right == 0
        reduce(lo + left + 1, right - 1, pivot, nxt, b_)

    out.append(a)
    reduce(2, count - 2, a, b, a)
    return out, start


def normalize(v):
    ln = math.sqrt(v[0] * v[0] + v[1] * v[1])
    inv = 1.0 / (ln + 2.2250738585072014e-308)
    return (v[0] * inv, v[1] * inv)


def poly_planes(verts):
    """cpPolyShape SetVerts: normal of edge (i-1 -> i) = normalize(rperp(b - a))."""
    n = len(verts)
    out = []
    for i in range(n):
        a, b = verts[(i - 1 + n) % n], verts[i]
        d = _sub(b, a)
        out.append(normalize((d[1], -d[0])))
    return out


def moment_for_poly(m, verts, offset=(0.0, 0.0)):
    """cpMomentForPoly (radius ignored)."""
    sum1 = sum2 = 0.0
    n = len(verts)
    for i in range(n):
        v1 = (verts[i][0] + offset[0], verts[i][1] + offset[1])
        w = verts[(i + 1) % n]
        v2 = (w[0] + offset[0], w[1] + offset[1])
        a = v2[0] * v1[1] - v2[1] * v1[0]
        b = (v1[0] * v1[0] + v1[1] * v1[1]) + (v1[0] * v2[0] + v1[1] * v2[1]) + (v2[0] * v2[0] + v2[1] * v2[1])
        sum1 += a * b
        sum2 += a
    return (m * sum1) / (6.0 * sum2)


def moment_for_circle(m, r1, r2):
    """cpMomentForCircle with offset (0, 0)."""
    return m * (0.5 * (r1 * r1 + r2 * r2) + (0.0 * 0.0 + 0.0 * 0.0))


def convex_decomposition(closed_polyline):
    """pymunk.autogeometry.convex_decomposition(line, 0) ->
    cpPolylineConvexDecomposition_BETA.  Returns parts as closed vertex lists.
    Chipmunk reads verts[count] when a cut lands at t = 1 of the last edge: at
    the top level that slot holds the closing duplicate; in recursive calls it
    is never written (poisoned with NaN here, which never arises for the star)."""
    parts = []

    def nexti(i, count):
        return (i + 1) % count

    def find_steiner(verts, count, notch_i, notch_v, notch_n):
        mn, feature = math.inf, -1.0
        for i in range(1, count - 1):
            index = (notch_i + i) % count
            a, b = verts[index], verts[nexti(index, count)]
            ta = notch_n[0] * (a[1] - notch_v[1]) - notch_n[1] * (a[0] - notch_v[0])
            tb = notch_n[0] * (b[1] - notch_v[1]) - notch_n[1] * (b[0] - notch_v[0])
            if ta * tb <= 0.0:
                t = ta / (ta - tb) if (ta - tb) != 0.0 else math.nan
                lx, ly = a[0] * (1.0 - t) + b[0] * t, a[1] * (1.0 - t) + b[1] * t
                dist = notch_n[0] * (lx - notch_v[0]) + notch_n[1] * (ly - notch_v[1])
                if dist >= 0.0 and dist <= mn:
                    mn, feature = dist, index + t
        return feature

    def deepest_notch(verts, count, hull, first):
        nd, ni, nv, nn = 0.0, 0, (0.0, 0.0), (0.0, 0.0)
        j = nexti(first, count)
        for i in range(len(hull)):
            a, b = hull[i], hull[nexti(i, len(hull))]
            n = normalize((a[1] - b[1], -(a[0] - b[0])))
            d = n[0] * a[0] + n[1] * a[1]
            v = verts[j]
            while not (v[0] == b[0] and v[1] == b[1]):
                depth = (n[0] * v[0] + n[1] * v[1]) - d
                if depth > nd:
                    nd, ni, nv, nn = depth, j, v, n
                j = nexti(j, count)
                v = verts[j]
            j = nexti(j, count)
        return nd, ni, nv, nn

    def decomp(verts, count):
        hull, first = convex_hull(verts[:count], 0.0)
        if len(hull) != count:
            nd, ni, nv, nn = deepest_notch(verts, count, hull, first)
            if nd > 0.0:
                sit = find_steiner(verts, count, ni, nv, nn)
                if sit >= 0.0:
                    si = int(sit)
                    t = sit - si
                    a, b = verts[si], verts[nexti(si, count)]
                    steiner = (a[0] * (1.0 - t) + b[0] * t, a[1] * (1.0 - t) + b[1] * t)
                    sub1 = (si - ni + count) % count + 1
                    sub2 = count - (si - ni + count) % count
                    scratch = [verts[(ni + i) % count] for i in range(sub1)] + [steiner]
                    decomp(scratch + [(math.nan, math.nan)] * 8, sub1 + 1)
                    scratch = [verts[(si + 1 + i) % count] for i in range(sub2)] + [steiner]
                    decomp(scratch + [(math.nan, math.nan)] * 8, sub2 + 1)
                    return
        parts.append(list(hull) + [hull[0]])

    pts = [tuple(v) for v in closed_polyline]
    decomp(pts, len(pts) - 1)
    return parts


# ---------------------------------------------------------------------------
# geom.py / entities.py formulas
def rect_verts(w, h):
    return [(w / 2, h / 2), (-w / 2, h / 2), (-w / 2, -h / 2), (w / 2, -h / 2)]


def make_finger_vertices(upper_arm_len, forearm_len, thickness, side_sign):
    """entities.py:193-214"""
    up_shift = upper_arm_len / 2
    upper = rect_verts(thickness, upper_arm_len)
    fore = rect_verts(thickness, forearm_len)
    upper_start = (side_sign * thickness / 2, upper_arm_len / 2)
    off_unrot = (-side_sign * thickness / 2, forearm_len / 2)
    rot_angle = side_sign * math.pi / 8
    r = rotated(off_unrot, rot_angle)
    ft = [upper_start[0] + r[0], upper_start[1] + r[1]]
    ft[1] += up_shift
    fore_t = []
    for v in fore:
        q = rotated(v, rot_angle)
        fore_t.append((q[0] + ft[0], q[1] + ft[1]))
    upper_t = [(v[0], v[1] + up_shift) for v in upper]
    return upper_t, fore_t


def regular_poly_side_length(n_sides, rad):
    """geom.py:18-22"""
    p_n = math.pi / n_sides
    return 2 * rad * math.sqrt(p_n * crtan(p_n))


def regular_poly_verts(n_sides, side_length):
    """geom.py:35-46"""
    step = 2 * math.pi / n_sides
    radius = side_length / (2 * crsin(math.pi / n_sides))
    return [rotated((0, radius), i * step) for i in range(n_sides)]


def star_verts(n_points, out_rad, in_rad):
    """geom.py:49-63"""
    out = []
    for i in range(n_points):
        out.append(rotated((0, out_rad), i * 2 * math.pi / n_points))
        out.append(rotated((0, in_rad), (2 * i + 1) * math.pi / n_points))
    return out


def make_circle_pts(radius, res, trig=None):
    """render.py:27-32.  trig = (cos, sin) replaces the correctly rounded pair (tests inject the
    reference's libm values to show that is the only difference)."""
    cos, sin = trig or (crcos, crsin)
    pts = []
    for i in range(res):
        ang = 2 * math.pi * i / res
        pts.append((cos(ang) * radius, sin(ang) * radius))
    return pts


def make_rect_pts(width, height):
    """render.py:13-24"""
    rad_h, rad_w = height / 2, width / 2
    return [(-rad_w, rad_h), (rad_w, rad_h), (rad_w, -rad_h), (-rad_w, -rad_h)]


# ---------------------------------------------------------------------------
# render.py Transform (numpy arithmetic)
def transform_trs(translation=(0.0, 0.0), rotation=0.0, scale=(1.0, 1.0), trig=None):
    cos, sin = trig or (crcos, crsin)
    c, s = cos(rotation), sin(rotation)
    T = np.asarray([[1.0, 0.0, translation[0]], [0.0, 1.0, translation[1]], [0.0, 0.0, 1.0]])
    R = np.asarray([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])
    S = np.asarray([[scale[0], 0.0, 0.0], [0.0, scale[1], 0.0], [0.0, 0.0, 1.0]])
    return T @ R @ S


def pygame_transform(height=384):
    """render.py:329-330: Transform(scale=(1,-1)).post_multiply(Transform(translation=(0, H)))"""
    return transform_trs(translation=(0, height)) @ transform_trs(scale=(1.0, -1.0))


def allo_view(res=384):
    """base_env.py:318-322 + render.py:339-347"""
    left, right, bottom, top = -1 * 1.02, 1 * 1.02, -1 * 1.02, 1 * 1.02
    sx, sy = res / (right - left), res / (top - bottom)
    cam = transform_trs(scale=(sx, sy), translation=(-left * sx, -bottom * sy))
    return pygame_transform(res) @ cam


def ego_view(rx, ry, ra, res=384, trig=None):
    """base_env.py:309-316 + render.py:290-304, 349-371"""
    world_h = world_w = 2 * 1.02
    sx, sy = res / world_w, res / world_h
    scale = transform_trs(scale=(sx, sy))
    tr1 = transform_trs(translation=(world_w * 0.5, world_h * 0.15))
    rot = transform_trs(rotation=-ra, trig=trig)
    tr2 = transform_trs(translation=(-rx, -ry))
    m = scale @ (tr1 @ (rot @ tr2))
    return pygame_transform(res) @ m


# ---------------------------------------------------------------------------
# palette (style.py)
def _rgb(r, g, b):
    return (r / 255.0, g / 255.0, b / 255.0)


def _darken(rgb):
    h, l, s = colorsys.rgb_to_hls(*rgb)
    return colorsys.hls_to_rgb(h, max(0, l * 0.9), s)


def _lighten(rgb, times=1):
    h, l, s = colorsys.rgb_to_hls(*rgb)
    mult = 1.4 ** times
    return colorsys.hls_to_rgb(h, 1 - (1 - l) / mult, s)


COLOURS_RGB = {
    "blue": _lighten(_rgb(0x3B, 0x7E, 0xA1), 1.7),
    "yellow": _lighten(_rgb(0xFD, 0xB5, 0x15), 1.7),
    "red": _lighten(_rgb(0xEE, 0x1F, 0x60), 1.7),
    "green": _lighten(_rgb(0x85, 0x94, 0x38), 1.7),
    "grey": _rgb(162, 163, 175),
}


def to_u8(rgb):
    """render.py:146-149 Geom.convert_color: round(rgb * 255)"""
    return tuple(int(v) for v in np.round(np.asarray(rgb) * 255))


def palette():
    out = {}
    for name in ["red", "green", "blue", "yellow", "grey"]:
        c = COLOURS_RGB[name]
        out[name] = [to_u8(c), to_u8(_darken(c)), to_u8(_lighten(c, 2)), to_u8(_lighten(c, 4))]
    return out


# ---------------------------------------------------------------------------
FPS = 8
ROBOT_RAD = 0.2
ROBOT_MASS = 1.0
SHAPE_RAD = ROBOT_RAD * 0.6
SHAPE_MASS = 0.5
ROBOT_LINE_THICKNESS = 0.01
SHAPE_LINE_THICKNESS = 0.015


def robot_tables():
    r = ROBOT_RAD
    thick, upper, lower = 0.25 * r, 1.1 * r, 0.7 * r
    outer, inner, inertia = [], [], []
    for side in (-1, 1):
        fv = make_finger_vertices(upper, lower, thick, side)
        iv = make_finger_vertices(upper - ROBOT_LINE_THICKNESS * 2, lower - ROBOT_LINE_THICKNESS * 2,
                                  thick - ROBOT_LINE_THICKNESS * 2, side)
        iv = [[(x, y + ROBOT_LINE_THICKNESS) for x, y in box] for box in iv]
        outer.append(fv)
        inner.append(iv)
        inertia.append(moment_for_poly(ROBOT_MASS / 8, list(fv[0]) + list(fv[1])))
    return outer, inner, inertia


def block_tables():
    """per shape type: physics polys (list of vertex lists, hull-ordered), mass, inertia, render polys"""
    size = SHAPE_RAD
    out = {}
    # SQUARE: create_box raw verts, radius 0.01 side, mass from the shape
    side = math.sqrt(math.pi) * size
    hw = hh = side / 2.0
    box = [(hw, -hh), (hw, hh), (-hw, hh), (-hw, -hh)]
    unit_i = moment_for_poly(1.0, box, (-0.0, -0.0))
    bm = 0.0
    msum = bm + SHAPE_MASS
    bi = 0.0 + (SHAPE_MASS * unit_i + 0.0 * (SHAPE_MASS * bm) / msum)
    out[SQUARE] = dict(polys=[(box, 0.01 * side)], mass=msum, inertia=bi,
                       render=[(make_rect_pts(side, side), OUTLINE_SOLID, RC_ENT_BASE, RC_ENT_DARK)])
    # CIRCLE
    out[CIRCLE] = dict(polys=[None], mass=SHAPE_MASS, inertia=moment_for_circle(SHAPE_MASS, 0, size),
                       render=[(make_circle_pts(size, 100), OUTLINE_SOLID, RC_ENT_BASE, RC_ENT_DARK)])
    # STAR
    out_rad = 1.3 * size
    in_rad = 0.5 * out_rad
    sv = star_verts(5, out_rad, in_rad)
    parts = convex_decomposition(sv + sv[:1])
    hull, _ = convex_hull(sv, 1e-5)
    inertia = moment_for_poly(SHAPE_MASS, hull + [hull[0]])
    ssv = star_verts(5, out_rad - SHAPE_LINE_THICKNESS, in_rad - SHAPE_LINE_THICKNESS)
    short_parts = convex_decomposition(ssv + ssv[:1])
    render = [(p, OUTLINE_NONE, RC_ENT_DARK, RC_ENT_DARK) for p in parts]
    render += [(p, OUTLINE_NONE, RC_ENT_BASE, RC_ENT_BASE) for p in short_parts]
    out[STAR] = dict(polys=[(convex_hull(p)[0], 0.0) for p in parts], mass=SHAPE_MASS, inertia=inertia,
                     render=render)
    # regular polygons
    for t, (factor, n) in {TRIANGLE: (0.8, 3), PENTAGON: (1.0, 5), HEXAGON: (1.0, 6), OCTAGON: (1.0, 8)}.items():
        sl = factor * regular_poly_side_length(n, size)
        pv = regular_poly_verts(n, sl)
        out[t] = dict(polys=[(convex_hull(pv)[0], 0.0)], mass=SHAPE_MASS, inertia=moment_for_poly(SHAPE_MASS, pv),
                      render=[(pv, OUTLINE_SOLID, RC_ENT_BASE, RC_ENT_DARK)])
    return out


def build_library():
    L = mg_library()
    dt = (1 / FPS) / 10
    L.dt = dt
    bias = 1.0 - math.pow(math.pow(1.0 - 0.1, 60.0), dt)
    L.collision_bias_coef = bias
    L.default_bias_coef = bias
    L.slop = 0.01
    r = ROBOT_RAD
    L.robot_radius = r
    L.robot_mass = ROBOT_MASS
    L.robot_inertia = moment_for_circle(ROBOT_MASS, 0, r)
    L.eye_mass = ROBOT_MASS / 10
    L.eye_inertia = moment_for_circle(ROBOT_MASS / 10, 0, r)
    L.finger_mass = ROBOT_MASS / 8
    moment = 1.0 / L.robot_inertia + 1.0 / L.eye_inertia
    L.spring_w_coef = 1.0 - math.exp(-3e-3 * dt * moment)
    outer, inner, finertia = robot_tables()
    polys = []  # (verts, radius)

    def add_poly(verts, radius):
        polys.append((verts, radius))
        return len(polys) - 1

    fpoly = []
    for k in range(2):
        L.finger_inertia[k] = finertia[k]
        side = -1 if k == 0 else 1
        L.finger_rel[k][0] = side * r * 0.45
        L.finger_rel[k][1] = r * 0.1
        for p in range(2):
            fpoly.append(add_poly(convex_hull(outer[k][p])[0], 0.0))
    for i in range(4):
        L.finger_poly[i] = fpoly[i]
    L.finger_lim[0][0], L.finger_lim[0][1] = -0.0, math.pi / 8
    L.finger_lim[1][0], L.finger_lim[1][1] = -math.pi / 8, 0.0
    L.finger_angle_off[0], L.finger_angle_off[1] = math.pi / 8, -math.pi / 8
    blocks = block_tables()
    for t in range(NUM_SHAPE_TYPES):
        b = blocks[t]
        L.block_nshapes[t] = len(b["polys"])
        for i, p in enumerate(b["polys"]):
            L.block_poly[t][i] = -1 if p is None else add_poly(p[0], p[1])
        L.block_mass[t] = b["mass"]
        L.block_inertia[t] = b["inertia"]
    L.block_circle_r = SHAPE_RAD
    assert len(polys) <= MAX_LIB_POLYS
    L.n_polys = len(polys)
    for i, (verts, radius) in enumerate(polys):
        assert len(verts) <= MAX_PVERTS
        L.poly_count[i] = len(verts)
        L.poly_r[i] = radius
        for j, (v, n) in enumerate(zip(verts, poly_planes(verts))):
            L.poly_v[i][j][0], L.poly_v[i][j][1] = v
            L.poly_n[i][j][0], L.poly_n[i][j][1] = n
    # ---- render library ----
    rpolys, rpts = [], []
    statics = [transform_trs(translation=(-1 + 2 / 2, -1 + 2 / 2)),           # arena centre_xform
               transform_trs(translation=(-1 * 0.4 * r, 0.3 * r)),              # eye base L
               transform_trs(translation=(1 * 0.4 * r, 0.3 * r)),               # eye base R
               transform_trs(translation=(0, r * 0.07))]                        # pupil offset

    def add_r(pts, outline, col, ocol, xfs):
        off = len(rpts)
        if pts is None:
            off = -1
            npts = 4
        else:
            rpts.extend(pts)
            npts = len(pts)
        rpolys.append((npts, off, outline, col, ocol, xfs))
        return len(rpolys) - 1

    L.arena_rpoly0 = add_r(make_rect_pts(2, 2), OUTLINE_SOLID, RC_WHITE, RC_GREY_BASE, [XF_STATIC0 + 0])
    L.arena_nrpoly = 1
    L.goal_rpoly0 = add_r(None, OUTLINE_DASHED, RC_ENT_LIGHT2, RC_ENT_BASE, [XF_MAIN])  # make_rect(w, h) per env
    L.goal_nrpoly = 1
    L.robot_rpoly0 = len(rpolys)
    for k in range(2):
        for p in range(2):
            add_r(convex_hull(outer[k][p])[0], OUTLINE_NONE, RC_GREY_BASE, RC_GREY_BASE, [XF_FINGER_L + k])
    for k in range(2):
        for p in range(2):
            add_r(inner[k][p], OUTLINE_NONE, RC_GREY_LIGHT4, RC_GREY_LIGHT4, [XF_FINGER_L + k])
    add_r(make_circle_pts(r, 100), OUTLINE_SOLID, RC_GREY_BASE, RC_GREY_DARK, [XF_MAIN])
    for k in range(2):
        add_r(make_circle_pts(0.2 * r, 100), OUTLINE_NONE, RC_WHITE, RC_WHITE, [XF_STATIC0 + 1 + k, XF_MAIN])
        add_r(make_circle_pts(0.12 * r, 100), OUTLINE_NONE, RC_PUPIL, RC_PUPIL,
              [XF_STATIC0 + 3, XF_PUPIL_L + k, XF_STATIC0 + 1 + k, XF_MAIN])
    L.robot_nrpoly = len(rpolys) - L.robot_rpoly0
    for t in range(NUM_SHAPE_TYPES):
        L.block_rpoly0[t] = len(rpolys)
        for pts, outline, col, ocol in blocks[t]["render"]:
            add_r(pts, outline, col, ocol, [XF_MAIN])
        L.block_nrpoly[t] = len(rpolys) - L.block_rpoly0[t]
    assert len(rpolys) <= MAX_RPOLYS and len(rpts) <= MAX_RPTS
    # the render kernel's outline layer holds one bit per entity (mg_render.h RenderSmem): at most one
    # outlined polygon per entity kind
    for r0, n in ([(L.arena_rpoly0, L.arena_nrpoly), (L.goal_rpoly0, L.goal_nrpoly), (L.robot_rpoly0, L.robot_nrpoly)]
                  + [(L.block_rpoly0[t], L.block_nrpoly[t]) for t in range(NUM_SHAPE_TYPES)]):
        assert sum(1 for i in range(r0, r0 + n) if rpolys[i][2] != OUTLINE_NONE) <= 1
    L.n_rpolys = len(rpolys)
    for i, (npts, off, outline, col, ocol, xfs) in enumerate(rpolys):
        rp = L.rpoly[i]
        rp.npts, rp.pts_off, rp.outline, rp.col_ref, rp.ocol_ref, rp.nxf = npts, off, outline, col, ocol, len(xfs)
        for j, x in enumerate(xfs):
            rp.xf[j] = x
    for i, (x, y) in enumerate(rpts):
        L.rpts[i][0], L.rpts[i][1] = x, y
    for i, m in enumerate(statics):
        for j, v in enumerate(m.ravel()):
            L.static_xf[i][j] = v
    for j, v in enumerate(allo_view().ravel()):
        L.allo_view[j] = v
    world = 2 * 1.02
    for name, m in (("ego_scale_m", transform_trs(scale=(384 / world, 384 / world))),
                    ("ego_tr1_m", transform_trs(translation=(world * 0.5, world * 0.15))),
                    ("pygame_m", pygame_transform())):
        arr = getattr(L, name)
        for j, v in enumerate(m.ravel()):
            arr[j] = v
    pal = palette()
    for ci, name in enumerate(["red", "green", "blue", "yellow", "grey"]):
        for k in range(4):
            for ch in range(3):
                L.palette[ci][k][ch] = pal[name][k][ch]
    for ch in range(3):
        L.white[ch] = 255
        L.pupil[ch] = to_u8((0.1, 0.1, 0.1))[ch]
        L.background[ch] = pal["grey"][3][ch]
    return L
