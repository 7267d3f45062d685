// mg_phys.h -- Chipmunk2D 7.0.x step semantics, one env per lane.
//
// Replaces base_env.BaseEnv._phys_steps_on_frame (base_env.py:248-255) and the
// pymunk Space.step it calls: position integration,
// shape caches, canonical broadphase (dynamic shape i vs walls, then vs
// dynamic j > i), GJK/EPA narrowphase with pymunk's contact clipping, arbiter
// cache with contact-hash warm starting and persistence 3, then 10 sequential
// impulse iterations over arbiters and constraints (Pivot, Gear, RotaryLimit,
// SimpleMotor, DampedRotarySpring).  Every expression keeps Chipmunk's
// operation order so results are bit-identical to the CPU oracle.
#pragma once
#include <float.h>
#include "mg_math.h"
#include "mg_state.h"

#define AT(p, i) (p)[(uint32_t)(i) * (uint32_t)S.N + (uint32_t)e]
#define CPA(k, c) S.cp[((uint32_t)(k) * (uint32_t)S.cons_cap + (uint32_t)(c)) * (uint32_t)S.N + (uint32_t)e]
#define ACON(k, f, a) S.acon[(((uint32_t)(k) * AC_NUM + (uint32_t)(f)) * (uint32_t)S.arb_cap + (uint32_t)(a)) * (uint32_t)S.N + (uint32_t)e]
#define AHASH(k, a) S.ahash[((uint32_t)(k) * (uint32_t)S.arb_cap + (uint32_t)(a)) * (uint32_t)S.N + (uint32_t)e]

struct V2 { double x, y; };
MG_DEV V2 v2(double x, double y) { return {x, y}; }
MG_DEV V2 vadd(V2 a, V2 b) { return {a.x + b.x, a.y + b.y}; }
MG_DEV V2 vsub(V2 a, V2 b) { return {a.x - b.x, a.y - b.y}; }
MG_DEV V2 vneg(V2 a) { return {-a.x, -a.y}; }
MG_DEV V2 vmult(V2 a, double s) { return {a.x * s, a.y * s}; }
MG_DEV double vdot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
MG_DEV double vcross(V2 a, V2 b) { return a.x * b.y - a.y * b.x; }
MG_DEV V2 vperp(V2 a) { return {-a.y, a.x}; }
MG_DEV V2 vrperp(V2 a) { return {a.y, -a.x}; }
MG_DEV V2 vrotate(V2 a, V2 b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
MG_DEV double vlengthsq(V2 a) { return vdot(a, a); }
MG_DEV double vlength(V2 a) { return sqrt(vdot(a, a)); }
MG_DEV V2 vnormalize(V2 a) { return vmult(a, 1.0 / (vlength(a) + DBL_MIN)); }
MG_DEV V2 vlerp(V2 a, V2 b, double t) { return vadd(vmult(a, 1.0 - t), vmult(b, t)); }
MG_DEV V2 vclamp(V2 v, double len) { return (vdot(v, v) > len * len) ? vmult(vnormalize(v), len) : v; }
MG_DEV double cpmax(double a, double b) { return (a > b) ? a : b; }
MG_DEV double cpmin(double a, double b) { return (a < b) ? a : b; }
MG_DEV double cpclamp(double f, double mn, double mx) { return cpmin(cpmax(f, mn), mx); }
MG_DEV double cpclamp01(double f) { return cpmax(0.0, cpmin(f, 1.0)); }
MG_DEV uint64_t hash_pair(uint64_t a, uint64_t b) { return (a * 3344921057ull) ^ (b * 3344921057ull); }

// arena walls (entities.py:510-522): static segments, radius 1, friction 0.8, end points
// {(-2,2)-(2,2), (2,2)-(2,-2), (2,-2)-(-2,-2), (-2,-2)-(-2,2)} (wall_a / wall_b below)

// --------------------------------------------------------------------------
// body helpers
MG_DEV void body_set_angle(const MGState &S, int e, int b, double a) {
    AT(S.ba, b) = a;
    if (a != AT(S.bacache, b)) { // transform depends only on the angle
        double s, c;
        mg_sincos(a, s, c);
        AT(S.brc, b) = c; AT(S.brs, b) = s; AT(S.bacache, b) = a;
    }
}

// Bodies whose rotation transform nothing reads: the robot's kinematic control body (its one joint,
// PivotJoint(control, body, (0, 0), (0, 0)) at entities.py:312-320, rotates a zero anchor, so any
// rotation gives the same r1) and its two eye bodies (no shapes; their DampedRotarySprings read angles,
// not transforms; the pupils are drawn from angle differences, entities.py:489-491).  Their angle is
// stored without the correctly rounded sincos: the cache (bacache) then no longer matches the angle and
// any reader that needs the transform recomputes it (render body_sincos).
MG_DEV bool body_rot_unused(const MGState &S, int e, int b) {
    const int r = S.robot_body0[e];
    return b > r && b <= r + 3;
}
MG_DEV void body_set_angle_step(const MGState &S, int e, int b, double a) {
    if (body_rot_unused(S, e, b)) AT(S.ba, b) = a;
    else body_set_angle(S, e, b, a);
}

// --------------------------------------------------------------------------
// world-space view of one shape (cpShape cache data)
enum { WS_CIRCLE = 0, WS_SEGMENT = 1, WS_POLY = 2 };
struct ShapeW {
    int type, count, body;
    uint64_t hashid;
    double r;
    V2 c;             // circle centre
    V2 a, b, n;       // segment
    V2 v[MG_MAX_PVERTS], pn[MG_MAX_PVERTS];
    double bbl, bbb, bbr, bbt;
};

// wall w's end points (as arithmetic on w: no constant-memory load on the narrowphase's path)
MG_DEV V2 wall_a(int w) { return v2(w == 0 || w == 3 ? -2.0 : 2.0, w >= 2 ? -2.0 : 2.0); }
MG_DEV V2 wall_b(int w) { return v2(w <= 1 ? 2.0 : -2.0, w == 1 || w == 2 ? -2.0 : 2.0); }
MG_DEV void load_wall(int w, ShapeW &sh) {
    sh.type = WS_SEGMENT; sh.count = 0; sh.body = -1; sh.hashid = (uint64_t)w; sh.r = 1.0;
    // identity transform of the (never positioned) static arena body: {1, 0, -0, 1, 0, 0}
    V2 a = wall_a(w), b = wall_b(w);
    sh.a = v2(1.0 * a.x + (-0.0) * a.y + 0.0, 0.0 * a.x + 1.0 * a.y + 0.0);
    sh.b = v2(1.0 * b.x + (-0.0) * b.y + 0.0, 0.0 * b.x + 1.0 * b.y + 0.0);
    V2 n = vrperp(vnormalize(vsub(b, a)));
    sh.n = v2(1.0 * n.x + (-0.0) * n.y, 0.0 * n.x + 1.0 * n.y);
    double l, r, bt, t;
    if (sh.a.x < sh.b.x) { l = sh.a.x; r = sh.b.x; } else { l = sh.b.x; r = sh.a.x; }
    if (sh.a.y < sh.b.y) { bt = sh.a.y; t = sh.b.y; } else { bt = sh.b.y; t = sh.a.y; }
    sh.bbl = l - 1.0; sh.bbb = bt - 1.0; sh.bbr = r + 1.0; sh.bbt = t + 1.0;
}

// dynamic shape slot k in world space using its body's current transform
MG_DEV void load_shape(const MGState &S, const mg_library *L, int e, int k, uint64_t hashid, ShapeW &sh) {
    int b = AT(S.sbody, k), p = AT(S.spoly, k);
    double c = AT(S.brc, b), s = AT(S.brs, b), px = AT(S.bpx, b), py = AT(S.bpy, b);
    sh.body = b; sh.hashid = hashid; sh.r = AT(S.sr, k);
    if (p < 0) {
        sh.type = WS_CIRCLE; sh.count = 0;
        sh.c = v2(c * 0.0 + (-s) * 0.0 + px, s * 0.0 + c * 0.0 + py);
        sh.bbl = sh.c.x - sh.r; sh.bbb = sh.c.y - sh.r; sh.bbr = sh.c.x + sh.r; sh.bbt = sh.c.y + sh.r;
    } else {
        sh.type = WS_POLY;
        int n = L->poly_count[p];
        sh.count = n;
        double l = INFINITY, r = -INFINITY, bb = INFINITY, t = -INFINITY;
        for (int i = 0; i < n; i++) {
            double vx = L->poly_v[p][i][0], vy = L->poly_v[p][i][1];
            double nx = L->poly_n[p][i][0], ny = L->poly_n[p][i][1];
            V2 v = v2(c * vx + (-s) * vy + px, s * vx + c * vy + py);
            sh.v[i] = v;
            sh.pn[i] = v2(c * nx + (-s) * ny, s * nx + c * ny);
            l = cpmin(l, v.x); r = cpmax(r, v.x); bb = cpmin(bb, v.y); t = cpmax(t, v.y);
        }
        sh.bbl = l - sh.r; sh.bbb = bb - sh.r; sh.bbr = r + sh.r; sh.bbt = t + sh.r;
    }
}

// goal sensor: static box (cpBoxShapeNew raw verts) at its body position
MG_DEV void load_goal(double gx, double gy, double w, double h, uint64_t hashid, ShapeW &sh) {
    double hw = w / 2.0, hh = h / 2.0;
    V2 vs[4] = {v2(hw, -hh), v2(hw, hh), v2(-hw, hh), v2(-hw, -hh)};
    sh.type = WS_POLY; sh.count = 4; sh.body = -1; sh.hashid = hashid; sh.r = 0.0;
    double l = INFINITY, r = -INFINITY, bb = INFINITY, t = -INFINITY;
    for (int i = 0; i < 4; i++) {
        V2 a = vs[(i + 3) % 4], b = vs[i];
        V2 n = vnormalize(vrperp(vsub(b, a)));
        V2 v = v2(1.0 * b.x + (-0.0) * b.y + gx, 0.0 * b.x + 1.0 * b.y + gy);
        sh.v[i] = v;
        sh.pn[i] = v2(1.0 * n.x + (-0.0) * n.y, 0.0 * n.x + 1.0 * n.y);
        l = cpmin(l, v.x); r = cpmax(r, v.x); bb = cpmin(bb, v.y); t = cpmax(t, v.y);
    }
    sh.bbl = l; sh.bbb = bb; sh.bbr = r; sh.bbt = t;
}

// the shape's cached BB (cpShapeCacheBB), computed as load_shape does but without materialising
// the world-space vertices
MG_DEV void shape_update_bb(const MGState &S, const mg_library *L, int e, int k) {
    const int b = AT(S.sbody, k), p = AT(S.spoly, k);
    const double c = AT(S.brc, b), s = AT(S.brs, b), px = AT(S.bpx, b), py = AT(S.bpy, b), r = AT(S.sr, k);
    double bl, bb, br, bt;
    if (p < 0) {
        const double cx = c * 0.0 + (-s) * 0.0 + px, cy = s * 0.0 + c * 0.0 + py;
        bl = cx - r; bb = cy - r; br = cx + r; bt = cy + r;
    } else {
        double l = INFINITY, rr = -INFINITY, lo = INFINITY, t = -INFINITY;
        const int n = L->poly_count[p];
        for (int i = 0; i < n; i++) {
            const double vx = L->poly_v[p][i][0], vy = L->poly_v[p][i][1];
            const double x = c * vx + (-s) * vy + px, y = s * vx + c * vy + py;
            l = cpmin(l, x); rr = cpmax(rr, x); lo = cpmin(lo, y); t = cpmax(t, y);
        }
        bl = l - r; bb = lo - r; br = rr + r; bt = t + r;
    }
    AT(S.sbbl, k) = bl; AT(S.sbbb, k) = bb; AT(S.sbbr, k) = br; AT(S.sbbt, k) = bt;
}

// BB of arena wall w (load_wall: segment a-b of radius 1)
MG_DEV void wall_bb(int w, double &l, double &b, double &r, double &t) {
    const V2 wa = wall_a(w), wb = wall_b(w);
    const double ax = wa.x, ay = wa.y, bx = wb.x, by = wb.y;
    l = (ax < bx ? ax : bx) - 1.0; r = (ax < bx ? bx : ax) + 1.0;
    b = (ay < by ? ay : by) - 1.0; t = (ay < by ? by : ay) + 1.0;
}

// --------------------------------------------------------------------------
// narrowphase (cpCollision.c): GJK / EPA / ContactPoints
struct MinkP { V2 a, b, ab; uint32_t id; };
struct Closest { V2 a, b, n; double d; };
struct Collision { int count; V2 n; V2 p1[2], p2[2]; uint64_t hash[2]; };

MG_DEV int poly_support_index(const ShapeW &sh, V2 n) {
    double mx = -INFINITY; int index = 0;
    for (int i = 0; i < sh.count; i++) {
        double d = vdot(sh.v[i], n);
        if (d > mx) { mx = d; index = i; }
    }
    return index;
}
MG_DEV void support_point(const ShapeW &sh, V2 n, V2 &p, int &idx) {
    if (sh.type == WS_CIRCLE) { p = sh.c; idx = 0; }
    else if (sh.type == WS_SEGMENT) {
        if (vdot(sh.a, n) > vdot(sh.b, n)) { p = sh.a; idx = 0; } else { p = sh.b; idx = 1; }
    } else { idx = poly_support_index(sh, n); p = sh.v[idx]; }
}
MG_DEV MinkP support(const ShapeW &s1, const ShapeW &s2, V2 n) {
    V2 pa, pb; int ia, ib;
    support_point(s1, vneg(n), pa, ia);
    support_point(s2, n, pb, ib);
    return {pa, pb, vsub(pb, pa), ((uint32_t)(ia & 0xFF) << 8) | (uint32_t)(ib & 0xFF)};
}
MG_DEV double closest_t(V2 a, V2 b) {
    V2 delta = vsub(b, a);
    return -cpclamp(vdot(delta, vadd(a, b)) / vlengthsq(delta), -1.0, 1.0);
}
MG_DEV V2 lerp_t(V2 a, V2 b, double t) {
    double ht = 0.5 * t;
    return vadd(vmult(a, 0.5 - ht), vmult(b, 0.5 + ht));
}
MG_DEV double closest_dist(V2 v0, V2 v1) { return vlengthsq(lerp_t(v0, v1, closest_t(v0, v1))); }
MG_DEV bool check_area(V2 v1, V2 v2_) { return (v1.x * v2_.y) > (v1.y * v2_.x); }

MG_DEV Closest closest_points_new(const MinkP &v0, const MinkP &v1) {
    double t = closest_t(v0.ab, v1.ab);
    V2 p = lerp_t(v0.ab, v1.ab, t);
    V2 pa = lerp_t(v0.a, v1.a, t), pb = lerp_t(v0.b, v1.b, t);
    V2 n = vnormalize(vrperp(vsub(v1.ab, v0.ab)));
    double d = vdot(n, p);
    if (d <= 0.0 || (-1.0 < t && t < 1.0)) return {pa, pb, n, d};
    double d2 = vlength(p);
    return {pa, pb, vmult(p, 1.0 / (d2 + DBL_MIN)), d2};
}

// EPA's polytope holds support-point ids (ia << 8 | ib) and rebuilds each Minkowski point from the two
// shapes when it is read: the same operands, so the same bits as storing the points (a 4-byte entry
// instead of a 56-byte one keeps the per-lane scratch small)
MG_DEV V2 shape_point(const ShapeW &sh, int idx) {
    return sh.type == WS_CIRCLE ? sh.c : sh.type == WS_SEGMENT ? (idx ? sh.b : sh.a) : sh.v[idx];
}
MG_DEV MinkP mink(const ShapeW &s1, const ShapeW &s2, uint32_t id) {
    const V2 pa = shape_point(s1, (int)((id >> 8) & 0xFF)), pb = shape_point(s2, (int)(id & 0xFF));
    return {pa, pb, vsub(pb, pa), id};
}

#define MG_EPA_MAX 40
MG_DEV Closest epa(const ShapeW &s1, const ShapeW &s2, MinkP v0, MinkP v1, MinkP v2_) {
    uint32_t hull[MG_EPA_MAX], hull2[MG_EPA_MAX];
    int count = 3;
    hull[0] = v0.id; hull[1] = v1.id; hull[2] = v2_.id;
    for (int iteration = 1;; iteration++) {
        int mini = 0;
        double minDist = INFINITY;
        for (int j = 0, i = count - 1; j < count; i = j, j++) {
            double d = closest_dist(mink(s1, s2, hull[i]).ab, mink(s1, s2, hull[j]).ab);
            if (d < minDist) { minDist = d; mini = i; }
        }
        MinkP w0 = mink(s1, s2, hull[mini]), w1 = mink(s1, s2, hull[(mini + 1) % count]);
        MinkP p = support(s1, s2, vperp(vsub(w1.ab, w0.ab)));
        bool duplicate = (p.id == w0.id || p.id == w1.id);
        if (!duplicate && check_area(w1.ab, p.ab) && iteration < 30 && count < MG_EPA_MAX - 1) {
            int count2 = 1;
            hull2[0] = p.id;
            for (int i = 0; i < count; i++) {
                int index = (mini + 1 + i) % count;
                V2 h0 = mink(s1, s2, hull2[count2 - 1]).ab, h1 = mink(s1, s2, hull[index]).ab;
                V2 h2 = (i + 1 < count ? mink(s1, s2, hull[(index + 1) % count]) : p).ab;
                if (check_area(vsub(h2, h0), vadd(vsub(h1, h0), vsub(h1, h2)))) hull2[count2++] = hull[index];
            }
            for (int i = 0; i < count2; i++) hull[i] = hull2[i];
            count = count2;
        } else {
            return closest_points_new(w0, w1);
        }
    }
}

MG_DEV Closest gjk(const ShapeW &s1, const ShapeW &s2) {
    V2 c1 = vlerp(v2(s1.bbl, s1.bbb), v2(s1.bbr, s1.bbt), 0.5);
    V2 c2 = vlerp(v2(s2.bbl, s2.bbb), v2(s2.bbr, s2.bbt), 0.5);
    V2 axis = vperp(vsub(c1, c2));
    MinkP v0 = support(s1, s2, axis), v1 = support(s1, s2, vneg(axis));
    int iteration = 1;
    for (;;) {
        if (iteration > 30) return closest_points_new(v0, v1);
        if (vcross(v1.ab, v0.ab) > 0.0) { MinkP t = v0; v0 = v1; v1 = t; continue; }
        double t = closest_t(v0.ab, v1.ab);
        V2 n = (-1.0 < t && t < 1.0 ? vperp(vsub(v1.ab, v0.ab)) : vneg(lerp_t(v0.ab, v1.ab, t)));
        MinkP p = support(s1, s2, n);
        if (vcross(vsub(v1.ab, p.ab), vadd(v1.ab, p.ab)) > 0.0 && vcross(vsub(v0.ab, p.ab), vadd(v0.ab, p.ab)) < 0.0)
            return epa(s1, s2, v0, p, v1);
        if (vdot(p.ab, n) <= cpmax(vdot(v0.ab, n), vdot(v1.ab, n))) return closest_points_new(v0, v1);
        if (closest_dist(v0.ab, p.ab) < closest_dist(p.ab, v1.ab)) v1 = p; else v0 = p;
        iteration++;
    }
}

struct Edge { V2 ap, bp; uint64_t ah, bh; double r; };
MG_DEV Edge support_edge_poly(const ShapeW &sh, V2 n) {
    int count = sh.count;
    int i1 = poly_support_index(sh, n);
    int i0 = (i1 - 1 + count) % count, i2 = (i1 + 1) % count;
    if (vdot(n, sh.pn[i1]) > vdot(n, sh.pn[i2]))
        return {sh.v[i0], sh.v[i1], hash_pair(sh.hashid, i0), hash_pair(sh.hashid, i1), sh.r};
    return {sh.v[i1], sh.v[i2], hash_pair(sh.hashid, i1), hash_pair(sh.hashid, i2), sh.r};
}
MG_DEV Edge support_edge_segment(const ShapeW &sh, V2 n) {
    if (vdot(sh.n, n) > 0.0) return {sh.a, sh.b, hash_pair(sh.hashid, 0), hash_pair(sh.hashid, 1), sh.r};
    return {sh.b, sh.a, hash_pair(sh.hashid, 1), hash_pair(sh.hashid, 0), sh.r};
}
MG_DEV void push_contact(Collision &c, V2 p1, V2 p2, uint64_t h) {
    // constant indices (a run-time index puts the whole Collision in per-lane scratch memory)
    if (c.count >= 2) return;
    if (c.count == 0) { c.p1[0] = p1; c.p2[0] = p2; c.hash[0] = h; }
    else { c.p1[1] = p1; c.p2[1] = p2; c.hash[1] = h; }
    c.count++;
}
MG_DEV void contact_points(const Edge &e1, const Edge &e2, const Closest &pts, Collision &info) {
    double mindist = e1.r + e2.r;
    if (pts.d <= mindist) {
        V2 n = info.n = pts.n;
        double d_e1_a = vcross(e1.ap, n), d_e1_b = vcross(e1.bp, n);
        double d_e2_a = vcross(e2.ap, n), d_e2_b = vcross(e2.bp, n);
        double e1_denom = 1.0 / (d_e1_b - d_e1_a + DBL_MIN);
        double e2_denom = 1.0 / (d_e2_b - d_e2_a + DBL_MIN);
        {
            V2 p1 = vadd(vmult(n, e1.r), vlerp(e1.ap, e1.bp, cpclamp01((d_e2_b - d_e1_a) * e1_denom)));
            V2 p2 = vadd(vmult(n, -e2.r), vlerp(e2.ap, e2.bp, cpclamp01((d_e1_a - d_e2_a) * e2_denom)));
            if (vdot(vsub(p2, p1), n) <= 0.0) push_contact(info, p1, p2, hash_pair(e1.ah, e2.bh));
        }
        {
            V2 p1 = vadd(vmult(n, e1.r), vlerp(e1.ap, e1.bp, cpclamp01((d_e2_a - d_e1_a) * e1_denom)));
            V2 p2 = vadd(vmult(n, -e2.r), vlerp(e2.ap, e2.bp, cpclamp01((d_e1_b - d_e2_a) * e2_denom)));
            if (vdot(vsub(p2, p1), n) <= 0.0) push_contact(info, p1, p2, hash_pair(e1.bh, e2.ah));
        }
    }
}

// cpCollide: (a, b) are swapped so type(a) <= type(b); returns swapped flag
#ifndef MG_COLLIDE_ATTR
#define MG_COLLIDE_ATTR MG_DEV
#endif
MG_COLLIDE_ATTR bool collide(const ShapeW &A, const ShapeW &B, Collision &info) {
    info.count = 0; info.n = v2(0, 0);
    bool sw = A.type > B.type;
    const ShapeW &a = sw ? B : A;
    const ShapeW &b = sw ? A : B;
    int code = a.type + b.type * 3;
    if (code == 0) { // circle-circle
        double mindist = a.r + b.r;
        V2 delta = vsub(b.c, a.c);
        double distsq = vlengthsq(delta);
        if (distsq < mindist * mindist) {
            double dist = sqrt(distsq);
            V2 n = info.n = (dist != 0.0 ? vmult(delta, 1.0 / dist) : v2(1.0, 0.0));
            push_contact(info, vadd(a.c, vmult(n, a.r)), vadd(b.c, vmult(n, -b.r)), 0);
        }
    } else if (code == 3) { // circle-segment
        V2 seg_delta = vsub(b.b, b.a);
        double ct = cpclamp01(vdot(seg_delta, vsub(a.c, b.a)) / vlengthsq(seg_delta));
        V2 closest = vadd(b.a, vmult(seg_delta, ct));
        double mindist = a.r + b.r;
        V2 delta = vsub(closest, a.c);
        double distsq = vlengthsq(delta);
        if (distsq < mindist * mindist) {
            double dist = sqrt(distsq);
            V2 n = info.n = (dist != 0.0 ? vmult(delta, 1.0 / dist) : b.n);
            push_contact(info, vadd(a.c, vmult(n, a.r)), vadd(closest, vmult(n, -b.r)), 0);
        }
    } else if (code >= 6) { // circle-poly (6), segment-poly (7), poly-poly (8): one GJK / EPA for the three,
                            // so the narrowphase inlines it once
        Closest pts = gjk(a, b);
        if (code == 6) {
            if (pts.d <= a.r + b.r) {
                V2 n = info.n = pts.n;
                push_contact(info, vadd(pts.a, vmult(n, a.r)), vadd(pts.b, vmult(n, -b.r)), 0);
            }
        } else if (pts.d - a.r - b.r <= 0.0) {
            const Edge ea = code == 7 ? support_edge_segment(a, pts.n) : support_edge_poly(a, pts.n);
            contact_points(ea, support_edge_poly(b, vneg(pts.n)), pts, info);
        }
    }
    return sw;
}

// Exact skip of collide() for shape pairs that are certainly apart.  For convex polygon A, edge k's
// outward normal n_k (cpPolyShape plane k: the edge ending at vertex k) gives A's largest projection at
// vertex k; if every point of B (polygon vertices, or the circle's centre) projects more than
// rA + rB + 1e-9 beyond it, the shapes are farther apart than their radii.  GJK then ends with a
// distance above rA + rB (its estimate never undercuts the true distance, and 1e-9 is far above its
// rounding), so collide() returns no contact and touches no arbiter: skipping it changes nothing.
// A conservative test -- false means "run collide()".  World points as load_shape computes them.
MG_DEV bool sat_poly_against(const mg_library *L, int pa, double ca, double sa, double pxa, double pya, int pb,
                             double cb, double sb, double pxb, double pyb, double gap) {
    const int na = L->poly_count[pa], nb = pb >= 0 ? L->poly_count[pb] : 1;
    V2 wb[MG_MAX_PVERTS];
#pragma unroll
    for (int j = 0; j < MG_MAX_PVERTS; j++) {
        const double vx = (pb >= 0 && j < nb) ? L->poly_v[pb][j][0] : 0.0;
        const double vy = (pb >= 0 && j < nb) ? L->poly_v[pb][j][1] : 0.0;
        wb[j] = v2(cb * vx + (-sb) * vy + pxb, sb * vx + cb * vy + pyb);
    }
#pragma unroll
    for (int k = 0; k < MG_MAX_PVERTS; k++) {
        if (k >= na) break;
        const double nx = L->poly_n[pa][k][0], ny = L->poly_n[pa][k][1];
        const double vx = L->poly_v[pa][k][0], vy = L->poly_v[pa][k][1];
        const V2 n = v2(ca * nx + (-sa) * ny, sa * nx + ca * ny);
        const double da = vdot(n, v2(ca * vx + (-sa) * vy + pxa, sa * vx + ca * vy + pya));
        double mb = INFINITY;
#pragma unroll
        for (int j = 0; j < MG_MAX_PVERTS; j++)
            if (j < nb) mb = cpmin(mb, vdot(n, wb[j]));
        if (mb - da > gap) return true;
    }
    return false;
}
MG_DEV bool surely_apart(const MGState &S, const mg_library *L, int e, int i, int j) {
    const int pi = AT(S.spoly, i), pj = AT(S.spoly, j);
    if (pi < 0 && pj < 0) return false;   // circle-circle: collide() is cheaper than the test
    const int bi = AT(S.sbody, i), bj = AT(S.sbody, j);
    const double gap = AT(S.sr, i) + AT(S.sr, j) + 1e-9;
    const double ci = AT(S.brc, bi), si = AT(S.brs, bi), xi = AT(S.bpx, bi), yi = AT(S.bpy, bi);
    const double cj = AT(S.brc, bj), sj = AT(S.brs, bj), xj = AT(S.bpx, bj), yj = AT(S.bpy, bj);
    if (pi >= 0 && sat_poly_against(L, pi, ci, si, xi, yi, pj, cj, sj, xj, yj, gap)) return true;
    if (pj >= 0 && sat_poly_against(L, pj, cj, sj, xj, yj, pi, ci, si, xi, yi, gap)) return true;
    return false;
}

MG_DEV bool bb_intersects(const ShapeW &a, const ShapeW &b) {
    return (a.bbl <= b.bbr && b.bbl <= a.bbr && a.bbb <= b.bbt && b.bbb <= a.bbt);
}
