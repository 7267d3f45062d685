/*
 * scene.c -- MAGICAL entities, tasks, reset randomisation and scoring, restated.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Follows: entities.py:193-491 (Robot), :498-533 (ArenaBoundaries),
 * :580-754 (Shape), :762-868 (GoalRegion); geom.py:13-63 (vertex formulas),
 * :116-384 (pm_randomise_pose / pm_randomise_all_poses / randomise_hw /
 * pm_shift_bodies); base_env.py:49-57,190-246 (PhysicsVariables, reset);
 * benchmarks/move_to_region.py:30-94, move_to_corner.py:125-171,
 * cluster.py:67-216, match_regions.py:44-213; render.py:13-134 (geoms,
 * Transform); style.py (palette).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include "oscene.h"

static inline vec2 v2(double x, double y) { vec2 r = {x, y}; return r; }

/* palette: round(255 * rgb) of style.py COLOURS_RGB, darken_rgb, lighten_rgb(x,2),
 * lighten_rgb(x,4); pinned against magical/style.py in tests/golden */
const uint8_t O_PALETTE[5][4][3] = {
    {{245, 129, 165}, {243, 94, 141}, {250, 190, 209}, {253, 222, 232}}, /* red */
    {{195, 208, 130}, {183, 198, 105}, {224, 231, 191}, {239, 243, 222}}, /* green */
    {{135, 185, 211}, {110, 170, 202}, {194, 219, 233}, {224, 237, 244}}, /* blue */
    {{254, 213, 123}, {254, 201, 86}, {254, 234, 188}, {255, 244, 221}},  /* yellow */
    {{162, 163, 175}, {144, 145, 159}, {208, 208, 214}, {231, 231, 234}}, /* grey */
};
static const uint8_t WHITE[3] = {255, 255, 255};
static const uint8_t PUPIL[3] = {26, 26, 26};

/* constants (base_env.py:60-76, entities.py) */
#define ROBOT_RAD 0.2
#define ROBOT_MASS 1.0
#define SHAPE_MASS 0.5
#define SHAPE_LINE_THICKNESS 0.015
#define ROBOT_LINE_THICKNESS 0.01
static double shape_rad(void) { return ROBOT_RAD * 0.6; }

/* ---------------- numpy 3x3 arithmetic (render.py Transform) -------------- */
/* numpy float64 matmul (OpenBLAS dgemm) evaluates each element as the FMA chain
 * fma(a2, b2, fma(a1, b1, a0*b0)) -- measured in this container, pinned in
 * tests/golden. */
void o_mat3_mul(const double *a, const double *b, double *out) {
    double t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            t[i * 3 + j] = fma(a[i * 3 + 2], b[6 + j], fma(a[i * 3 + 1], b[3 + j], a[i * 3 + 0] * b[j]));
    memcpy(out, t, sizeof(t));
}

void o_transform_trs(double tx, double ty, double rot, double sx, double sy, double *out) {
    double c = o_crcos(rot), s = o_crsin(rot);
    double T[9] = {1.0, 0.0, tx, 0.0, 1.0, ty, 0.0, 0.0, 1.0};
    double R[9] = {c, -s, 0.0, s, c, 0.0, 0.0, 0.0, 1.0};
    double S[9] = {sx, 0.0, 0.0, 0.0, sy, 0.0, 0.0, 0.0, 1.0};
    double TR[9];
    o_mat3_mul(T, R, TR);
    o_mat3_mul(TR, S, out);
}

/* Viewer.pygame_transform = T(0, H) @ S(1, -1)  (render.py:329-330) */
static void pygame_xform(double *out) {
    double S[9], T[9];
    o_transform_trs(0.0, 0.0, 0.0, 1.0, -1.0, S);
    o_transform_trs(0.0, (double)O_RES, 0.0, 1.0, 1.0, T);
    o_mat3_mul(T, S, out);
}

/* Viewer.set_bounds(-1.02, 1.02, -1.02, 1.02)  (base_env.py:318-322, render.py:339-347) */
void o_allo_view(double *out) {
    double left = -1 * 1.02, right = 1 * 1.02, bottom = -1 * 1.02, top = 1 * 1.02;
    double sx = (double)O_RES / (right - left), sy = (double)O_RES / (top - bottom);
    double cam[9], P[9];
    o_transform_trs(-left * sx, -bottom * sy, 0.0, sx, sy, cam);
    pygame_xform(P);
    o_mat3_mul(P, cam, out);
}

/* Viewer.set_cam_follow + ego_cam_matrix (base_env.py:309-316, render.py:290-371) */
void o_ego_view(double rx, double ry, double ra, double *out) {
    double world_h = 2 * 1.02, world_w = 2 * 1.02;
    double sx = (double)O_RES / world_w, sy = (double)O_RES / world_h;
    double scale[9], tr1[9], rot[9], tr2[9], m1[9], m2[9], m3[9], P[9];
    o_transform_trs(0.0, 0.0, 0.0, sx, sy, scale);
    o_transform_trs(world_w * 0.5, world_h * 0.15, 0.0, 1.0, 1.0, tr1);
    o_transform_trs(0.0, 0.0, -ra, 1.0, 1.0, rot);
    o_transform_trs(-rx, -ry, 0.0, 1.0, 1.0, tr2);
    o_mat3_mul(rot, tr2, m1);
    o_mat3_mul(tr1, m1, m2);
    o_mat3_mul(scale, m2, m3);
    pygame_xform(P);
    o_mat3_mul(P, m3, out);
}

/* ---------------- vertex formulas (geom.py, entities.py) ----------------- */
/* pymunk Vec2d.rotated: (x cos - y sin, x sin + y cos) */
static vec2 rotated(vec2 v, double ang) {
    double c = o_crcos(ang), s = o_crsin(ang);
    return v2(v.x * c - v.y * s, v.x * s + v.y * c);
}

/* geom.py:101-108 rect_verts */
static void rect_verts(double w, double h, vec2 out[4]) {
    out[0] = v2(w / 2, h / 2);
    out[1] = v2(-w / 2, h / 2);
    out[2] = v2(-w / 2, -h / 2);
    out[3] = v2(w / 2, -h / 2);
}

/* entities.py:193-214 make_finger_vertices */
void o_finger_verts(double upper, double fore, double thick, int side, vec2 up_out[4], vec2 fore_out[4]) {
    double up_shift = upper / 2;
    vec2 ua[4], fa[4];
    rect_verts(thick, upper, ua);
    rect_verts(thick, fore, fa);
    vec2 upper_start = v2(side * thick / 2, upper / 2);
    vec2 off_unrot = v2(-side * thick / 2, fore / 2);
    double rot_angle = side * M_PI / 8;
    vec2 r = rotated(off_unrot, rot_angle);
    vec2 ft = v2(upper_start.x + r.x, upper_start.y + r.y);
    ft.y += up_shift;
    for (int i = 0; i < 4; i++) {
        vec2 q = rotated(fa[i], rot_angle);
        fore_out[i] = v2(q.x + ft.x, q.y + ft.y);
    }
    for (int i = 0; i < 4; i++) up_out[i] = v2(ua[i].x, ua[i].y + up_shift);
}

/* geom.py:13-22 */
static double regular_poly_circumrad(int n, double side) { return side / (2 * o_crsin(M_PI / n)); }
static double circ_rad_to_side_length(int n, double rad) {
    double p_n = M_PI / n;
    return 2 * rad * sqrt(p_n * o_crtan(p_n));
}
/* geom.py:35-46 */
static void regular_poly_verts(int n, double side, vec2 *out) {
    double step = 2 * M_PI / n;
    double radius = regular_poly_circumrad(n, side);
    for (int i = 0; i < n; i++) out[i] = rotated(v2(0, radius), i * step);
}
/* geom.py:49-63 */
static void star_verts(int npts, double out_rad, double in_rad, vec2 *out) {
    for (int i = 0; i < npts; i++) {
        out[2 * i] = rotated(v2(0, out_rad), i * 2 * M_PI / npts);
        out[2 * i + 1] = rotated(v2(0, in_rad), (2 * i + 1) * M_PI / npts);
    }
}

/* cpMomentForPoly */
double o_moment_for_poly(double m, int count, const vec2 *verts, vec2 offset, double r) {
    (void)r;
    double sum1 = 0.0, sum2 = 0.0;
    for (int i = 0; i < count; i++) {
        vec2 v1 = v2(verts[i].x + offset.x, verts[i].y + offset.y);
        vec2 w = verts[(i + 1) % count];
        vec2 v2_ = v2(w.x + offset.x, w.y + offset.y);
        double a = v2_.x * v1.y - v2_.y * v1.x;
        double b = (v1.x * v1.x + v1.y * v1.y) + (v1.x * v2_.x + v1.y * v2_.y) + (v2_.x * v2_.x + v2_.y * v2_.y);
        sum1 += a * b;
        sum2 += a;
    }
    return (m * sum1) / (6.0 * sum2);
}
/* cpMomentForCircle */
static double moment_for_circle(double m, double r1, double r2) {
    return m * (0.5 * (r1 * r1 + r2 * r2) + (0.0 * 0.0 + 0.0 * 0.0));
}

/* ---- cpPolylineConvexDecomposition_BETA (cpPolyline.c, Chipmunk 7) ---- */
typedef struct { int i; double d; vec2 v, n; } Notch;
static int nexti(int i, int count) { return (i + 1) % count; }

static double find_steiner(int count, const vec2 *verts, Notch notch) {
    double mn = INFINITY, feature = -1.0;
    for (int i = 1; i < count - 1; i++) {
        int index = (notch.i + i) % count;
        vec2 a = verts[index], b = verts[nexti(index, count)];
        double thing_a = notch.n.x * (a.y - notch.v.y) - notch.n.y * (a.x - notch.v.x);
        double thing_b = notch.n.x * (b.y - notch.v.y) - notch.n.y * (b.x - notch.v.x);
        if (thing_a * thing_b <= 0.0) {
            double t = thing_a / (thing_a - thing_b);
            vec2 l = v2(a.x * (1.0 - t) + b.x * t, a.y * (1.0 - t) + b.y * t);
            double dist = notch.n.x * (l.x - notch.v.x) + notch.n.y * (l.y - notch.v.y);
            if (dist >= 0.0 && dist <= mn) { mn = dist; feature = index + t; }
        }
    }
    return feature;
}

static Notch deepest_notch(int count, const vec2 *verts, int hull_count, const vec2 *hull, int first) {
    Notch notch;
    memset(&notch, 0, sizeof(notch));
    int j = nexti(first, count);
    for (int i = 0; i < hull_count; i++) {
        vec2 a = hull[i], b = hull[nexti(i, hull_count)];
        vec2 d = v2(a.x - b.x, a.y - b.y);
        vec2 rp = v2(d.y, -d.x);
        double len = sqrt(rp.x * rp.x + rp.y * rp.y);
        double inv = 1.0 / (len + DBL_MIN);
        vec2 n = v2(rp.x * inv, rp.y * inv);
        double dd = n.x * a.x + n.y * a.y;
        vec2 v = verts[j];
        while (!(v.x == b.x && v.y == b.y)) {
            double depth = (n.x * v.x + n.y * v.y) - dd;
            if (depth > notch.d) { notch.d = depth; notch.i = j; notch.v = v; notch.n = n; }
            j = nexti(j, count);
            v = verts[j];
        }
        j = nexti(j, count);
    }
    return notch;
}

typedef struct { vec2 *out; int *counts; int nparts, max_parts, nverts; } PartSet;

static void approx_decomp(const vec2 *verts, int count, double tol, PartSet *set) {
    int first;
    vec2 hull[64];
    int hull_count = o_convex_hull(count, verts, hull, &first, 0.0);
    if (hull_count != count) {
        Notch notch = deepest_notch(count, verts, hull_count, hull, first);
        if (notch.d > tol) {
            double steiner_it = find_steiner(count, verts, notch);
            if (steiner_it >= 0.0) {
                int si = (int)steiner_it;
                double t = steiner_it - si;
                vec2 a = verts[si], b = verts[nexti(si, count)];
                vec2 steiner = v2(a.x * (1.0 - t) + b.x * t, a.y * (1.0 - t) + b.y * t);
                int sub1 = (si - notch.i + count) % count + 1;
                int sub2 = count - (si - notch.i + count) % count;
                vec2 scratch[64];
                /* Chipmunk reads verts[count] when the cut lands at t = 1 of the last
                 * edge; that slot is never written in recursive calls: poison it */
                for (int i = 0; i < 64; i++) scratch[i] = v2(NAN, NAN);
                for (int i = 0; i < sub1; i++) scratch[i] = verts[(notch.i + i) % count];
                scratch[sub1] = steiner;
                approx_decomp(scratch, sub1 + 1, tol, set);
                for (int i = 0; i < sub2; i++) scratch[i] = verts[(si + 1 + i) % count];
                scratch[sub2] = steiner;
                approx_decomp(scratch, sub2 + 1, tol, set);
                return;
            }
        }
    }
    if (set->nparts >= set->max_parts) return;
    for (int i = 0; i < hull_count; i++) set->out[set->nverts + i] = hull[i];
    set->out[set->nverts + hull_count] = hull[0];
    set->counts[set->nparts++] = hull_count + 1;
    set->nverts += hull_count + 1;
}

int o_star_decomposition(double out_rad, double in_rad, vec2 *out, int *counts, int max_parts) {
    vec2 sv[10];
    star_verts(5, out_rad, in_rad, sv);
    PartSet set = {out, counts, 0, max_parts, 0};
    /* closed polyline star + star[:1]; decomposition runs on count - 1 verts
     * (the closing duplicate stays readable at index 10, as in pymunk) */
    vec2 closed[11];
    memcpy(closed, sv, sizeof(sv));
    closed[10] = sv[0];
    approx_decomp(closed, 10, 0.0, &set);
    return set.nparts;
}

/* ---------------- transforms / geoms ------------------------------------- */
static int add_xf(OEnv *e) {
    int i = e->nxf++;
    o_transform_trs(0.0, 0.0, 0.0, 1.0, 1.0, e->xf[i].m);
    return i;
}
static int add_static_xf(OEnv *e, double tx, double ty) {
    int i = e->nxf++;
    o_transform_trs(tx, ty, 0.0, 1.0, 1.0, e->xf[i].m);
    return i;
}
static OGeom *add_geom(OEnv *e, int npts, const vec2 *pts, int outline, const uint8_t *col, const uint8_t *ocol) {
    if (e->ngeoms >= O_MAX_GEOMS) { /* table overflow: reported by oenv_reset/step, last slot reused */
        e->space.overflow = 1;
        e->ngeoms = O_MAX_GEOMS - 1;
    }
    OGeom *g = &e->geoms[e->ngeoms++];
    memset(g, 0, sizeof(*g));
    g->npts = npts;
    memcpy(g->pts, pts, sizeof(vec2) * (size_t)npts);
    g->outline = outline;
    memcpy(g->col, col, 3);
    if (ocol) memcpy(g->ocol, ocol, 3);
    return g;
}
static void geom_xf(OGeom *g, int xf) { g->xf[g->nxf++] = xf; }

/* render.py:13-36 */
static int make_rect_pts(double w, double h, vec2 *pts) {
    double rad_h = h / 2, rad_w = w / 2;
    pts[0] = v2(-rad_w, rad_h);
    pts[1] = v2(rad_w, rad_h);
    pts[2] = v2(rad_w, -rad_h);
    pts[3] = v2(-rad_w, -rad_h);
    return 4;
}
static int make_circle_pts(double radius, int res, vec2 *pts) {
    for (int i = 0; i < res; i++) {
        double ang = 2 * M_PI * i / res;
        pts[i] = v2(o_crcos(ang) * radius, o_crsin(ang) * radius);
    }
    return res;
}

/* ---------------- entities ---------------------------------------------- */
static OEntity *new_ent(OEnv *e, int kind) {
    OEntity *en = &e->ents[e->nents++];
    memset(en, 0, sizeof(*en));
    en->kind = kind;
    en->body0 = e->space.nbodies;
    en->shape0 = e->space.nshapes;
    en->xf_main = -1;
    return en;
}
static void end_ent(OEnv *e, OEntity *en) {
    en->nbodies = e->space.nbodies - en->body0;
    en->nshapes = e->space.nshapes - en->shape0;
    for (int i = en->shape0; i < e->space.nshapes; i++) e->space.shapes[i].entity = (int)(en - e->ents);
}

/* entities.py:498-533 */
static void add_arena(OEnv *e) {
    OEntity *en = new_ent(e, ENT_ARENA);
    double l = -1, r = 1, t = 1, b = -1, rad = 1;
    vec2 pts[4] = {v2(l - rad, t + rad), v2(r + rad, t + rad), v2(r + rad, b - rad), v2(l - rad, b - rad)};
    for (int i = 0; i < 4; i++) {
        int si = ophys_add_segment(&e->space, pts[i], pts[(i + 1) % 4], rad);
        e->space.shapes[si].u = 0.8;
    }
    end_ent(e, en);
    vec2 rp[4];
    double width = r - l, height = t - b;
    make_rect_pts(width, height, rp);
    OGeom *g = add_geom(e, 4, rp, OUTLINE_SOLID, WHITE, O_PALETTE[COL_GREY][0]);
    geom_xf(g, add_static_xf(e, l + width / 2, b + height / 2));
}

/* entities.py:762-801 */
static void add_goal(OEnv *e, double x, double y, double h, double w, int colour) {
    OEntity *en = new_ent(e, ENT_GOAL);
    en->gx = x; en->gy = y; en->gh = h; en->gw = w; en->colour = colour;
    vec2 pos = v2(x + w / 2, y - h / 2);
    int si = ophys_add_static_box(&e->space, pos, w, h);
    e->space.shapes[si].sensor = 1;
    en->pos = pos; en->angle = 0.0;
    end_ent(e, en);
    vec2 rp[4];
    make_rect_pts(w, h, rp);
    OGeom *g = add_geom(e, 4, rp, OUTLINE_DASHED, O_PALETTE[colour][2], O_PALETTE[colour][0]);
    en->xf_main = add_xf(e);
    geom_xf(g, en->xf_main);
    e->goal = (int)(en - e->ents);
}

/* entities.py:238-433 */
static void add_robot(OEnv *e, vec2 init_pos, double init_angle) {
    OSpace *s = &e->space;
    OEntity *en = new_ent(e, ENT_ROBOT);
    en->pos = init_pos; en->angle = init_angle;
    double radius = ROBOT_RAD, mass = ROBOT_MASS;
    double inertia = moment_for_circle(mass, 0, radius);
    int body = ophys_add_body(s, BODY_DYNAMIC, mass, inertia, init_pos, init_angle);
    int control = ophys_add_body(s, BODY_KINEMATIC, 0, 0, init_pos, init_angle);
    int c = ophys_add_pivot2(s, control, body, v2(0, 0), v2(0, 0));
    s->cons[c].maxBias = 0;
    s->cons[c].maxForce = e->pv[0];
    c = ophys_add_gear(s, control, body, 0.0, 1.0);
    s->cons[c].errorBias = 0.0;
    s->cons[c].maxBias = 2.5;
    s->cons[c].maxForce = e->pv[1];
    for (int side = -1; side <= 1; side += 2) {
        double eye_mass = mass / 10;
        double eye_inertia = moment_for_circle(eye_mass, 0, radius);
        int eye = ophys_add_body(s, BODY_DYNAMIC, eye_mass, eye_inertia, v2(0, 0), init_angle);
        c = ophys_add_spring(s, body, eye, 0, 0.1, 3e-3);
        s->cons[c].maxBias = 3.0;
        s->cons[c].maxForce = 0.001;
    }
    double f_thick = 0.25 * radius, f_upper = 1.1 * radius, f_lower = 0.7 * radius;
    vec2 fverts[2][2][4];
    vec2 finner[2][2][4];
    int fingers[2];
    const double limit_outer = M_PI / 8, limit_inner = 0.0;
    for (int k = 0; k < 2; k++) {
        int side = k == 0 ? -1 : 1;
        o_finger_verts(f_upper, f_lower, f_thick, side, fverts[k][0], fverts[k][1]);
        o_finger_verts(f_upper - ROBOT_LINE_THICKNESS * 2, f_lower - ROBOT_LINE_THICKNESS * 2,
                       f_thick - ROBOT_LINE_THICKNESS * 2, side, finner[k][0], finner[k][1]);
        for (int p = 0; p < 2; p++)
            for (int i = 0; i < 4; i++) finner[k][p][i].y = finner[k][p][i].y + ROBOT_LINE_THICKNESS;
        double lower, upper;
        if (side < 0) { lower = -limit_inner; upper = limit_outer; }
        else { lower = -limit_outer; upper = limit_inner; }
        double finger_mass = mass / 8;
        vec2 all8[8];
        memcpy(all8, fverts[k][0], sizeof(vec2) * 4);
        memcpy(all8 + 4, fverts[k][1], sizeof(vec2) * 4);
        double finger_inertia = o_moment_for_poly(finger_mass, 8, all8, v2(0, 0), 0);
        double fa = side < 0 ? init_angle + upper : init_angle + lower;
        vec2 rel = v2(side * radius * 0.45, radius * 0.1);
        vec2 relr = rotated(rel, init_angle);
        vec2 bp = s->bodies[body].p;
        vec2 fp = v2(bp.x + relr.x, bp.y + relr.y);
        int fb = ophys_add_body(s, BODY_DYNAMIC, finger_mass, finger_inertia, fp, fa);
        fingers[k] = fb;
        c = ophys_add_pivot1(s, body, fb, s->bodies[fb].p);
        s->cons[c].errorBias = 0.0;
        c = ophys_add_rotlimit(s, body, fb, lower, upper);
        s->cons[c].errorBias = 0.0;
        c = ophys_add_motor(s, body, fb, 0.0);
        s->cons[c].rate = 0.0;
        s->cons[c].maxBias = 0.0;
        s->cons[c].maxForce = e->pv[2];
    }
    int si = ophys_add_circle(s, body, radius, v2(0, 0));
    s->shapes[si].group = 1;
    s->shapes[si].u = 0.5;
    int fshape[2][2];
    for (int k = 0; k < 2; k++) {
        for (int p = 0; p < 2; p++) {
            si = ophys_add_poly(s, fingers[k], 4, fverts[k][p], 0.0, 0);
            s->shapes[si].group = 1;
            s->shapes[si].u = 5.0;
            fshape[k][p] = si;
        }
    }
    end_ent(e, en);
    /* graphics */
    const uint8_t *grey = O_PALETTE[COL_GREY][0], *dgrey = O_PALETTE[COL_GREY][1], *lgrey = O_PALETTE[COL_GREY][3];
    int fxf[2];
    for (int k = 0; k < 2; k++) fxf[k] = add_xf(e);
    for (int k = 0; k < 2; k++)
        for (int p = 0; p < 2; p++) {
            const OShape *sh = &s->shapes[fshape[k][p]];
            OGeom *g = add_geom(e, sh->count, sh->v, OUTLINE_NONE, grey, NULL);
            geom_xf(g, fxf[k]);
        }
    for (int k = 0; k < 2; k++)
        for (int p = 0; p < 2; p++) {
            OGeom *g = add_geom(e, 4, finner[k][p], OUTLINE_NONE, lgrey, NULL);
            geom_xf(g, fxf[k]);
        }
    int rxf = add_xf(e);
    vec2 pts[O_MAX_PTS];
    int n = make_circle_pts(radius, 100, pts);
    OGeom *g = add_geom(e, n, pts, OUTLINE_SOLID, grey, dgrey);
    geom_xf(g, rxf);
    int pxf[2];
    for (int k = 0; k < 2; k++) {
        int x_sign = k == 0 ? -1 : 1;
        n = make_circle_pts(0.2 * radius, 100, pts);
        OGeom *eye = add_geom(e, n, pts, OUTLINE_NONE, WHITE, NULL);
        int eb = add_static_xf(e, x_sign * 0.4 * radius, 0.3 * radius);
        geom_xf(eye, eb);
        geom_xf(eye, rxf);
        n = make_circle_pts(0.12 * radius, 100, pts);
        OGeom *pupil = add_geom(e, n, pts, OUTLINE_NONE, PUPIL, NULL);
        pxf[k] = add_xf(e);
        geom_xf(pupil, add_static_xf(e, 0, radius * 0.07));
        geom_xf(pupil, pxf[k]);
        geom_xf(pupil, eb);
        geom_xf(pupil, rxf);
    }
    en->xf_main = rxf;
    en->xf_aux[0] = fxf[0]; en->xf_aux[1] = fxf[1];
    en->xf_aux[2] = pxf[0]; en->xf_aux[3] = pxf[1];
    e->robot = (int)(en - e->ents);
}

/* entities.py:580-754 */
static void add_block(OEnv *e, int type, int colour, vec2 pos, double angle, int role) {
    OSpace *s = &e->space;
    OEntity *en = new_ent(e, ENT_BLOCK);
    en->type = type; en->colour = colour; en->pos = pos; en->angle = angle; en->role = role;
    double size = shape_rad(), mass = SHAPE_MASS;
    int body = -1;
    int shape_ids[16], nsh = 0;
    double side_len = 0;
    vec2 poly[8];
    int npoly = 0;
    vec2 parts[64]; int part_counts[8]; int nparts = 0;
    double star_out = 0, star_in = 0;
    if (type == SHAPE_SQUARE) {
        body = ophys_add_body(s, BODY_DYNAMIC, 1, 1, pos, angle); /* mass from the shape below */
        side_len = sqrt(M_PI) * size;
        double hw = side_len / 2.0, hh = side_len / 2.0;
        vec2 bv[4] = {v2(hw, -hh), v2(hw, hh), v2(-hw, hh), v2(-hw, -hh)};
        int si = ophys_add_poly(s, body, 4, bv, 0.01 * side_len, 1);
        shape_ids[nsh++] = si;
        /* shape.mass = 0.5 -> cpBodyAccumulateMassFromShapes (cog 0, i = m * unit moment) */
        vec2 neg_centroid = v2(-0.0, -0.0);
        double unit_i = o_moment_for_poly(1.0, 4, bv, neg_centroid, 0.01 * side_len);
        double bm = 0.0, bi = 0.0;
        double msum = bm + mass;
        bi += mass * unit_i + 0.0 * (mass * bm) / msum;
        bm = msum;
        OBody *b = &s->bodies[body];
        b->m = bm; b->i = bi; b->m_inv = 1.0 / bm; b->i_inv = 1.0 / bi;
    } else if (type == SHAPE_CIRCLE) {
        double inertia = moment_for_circle(mass, 0, size);
        body = ophys_add_body(s, BODY_DYNAMIC, mass, inertia, pos, angle);
        shape_ids[nsh++] = ophys_add_circle(s, body, size, v2(0, 0));
    } else if (type == SHAPE_STAR) {
        star_out = 1.3 * size;
        star_in = 0.5 * star_out;
        nparts = o_star_decomposition(star_out, star_in, parts, part_counts, 8);
        vec2 sv[10], hull[11];
        star_verts(5, star_out, star_in, sv);
        int hc = o_convex_hull(10, sv, hull, NULL, 1e-5);
        hull[hc] = hull[0];
        double inertia = o_moment_for_poly(mass, hc + 1, hull, v2(0, 0), 0);
        body = ophys_add_body(s, BODY_DYNAMIC, mass, inertia, pos, angle);
        uint32_t group = 1000 + (uint32_t)(++e->star_groups);
        int off = 0;
        for (int p = 0; p < nparts; p++) {
            int si = ophys_add_poly(s, body, part_counts[p], parts + off, 0.0, 0);
            s->shapes[si].group = group;
            shape_ids[nsh++] = si;
            off += part_counts[p];
        }
    } else {
        double factor = 1.0;
        int nsides = 5;
        if (type == SHAPE_TRIANGLE) { factor = 0.8; nsides = 3; }
        else if (type == SHAPE_PENTAGON) { nsides = 5; }
        else if (type == SHAPE_HEXAGON) { nsides = 6; }
        else if (type == SHAPE_OCTAGON) { nsides = 8; }
        side_len = factor * circ_rad_to_side_length(nsides, size);
        regular_poly_verts(nsides, side_len, poly);
        npoly = nsides;
        double inertia = o_moment_for_poly(mass, nsides, poly, v2(0, 0), 0);
        body = ophys_add_body(s, BODY_DYNAMIC, mass, inertia, pos, angle);
        shape_ids[nsh++] = ophys_add_poly(s, body, nsides, poly, 0.0, 0);
    }
    for (int i = 0; i < nsh; i++) s->shapes[shape_ids[i]].u = 0.5;
    int c = ophys_add_pivot2(s, -1, body, v2(0, 0), v2(0, 0));
    s->cons[c].maxBias = 0;
    s->cons[c].maxForce = e->pv[3];
    c = ophys_add_gear(s, -1, body, 0.0, 1.0);
    s->cons[c].maxBias = 0;
    s->cons[c].maxForce = e->pv[4];
    end_ent(e, en);
    /* graphics */
    const uint8_t *col = O_PALETTE[colour][0], *dcol = O_PALETTE[colour][1];
    en->xf_main = add_xf(e);
    vec2 pts[O_MAX_PTS];
    if (type == SHAPE_SQUARE) {
        int n = make_rect_pts(side_len, side_len, pts);
        geom_xf(add_geom(e, n, pts, OUTLINE_SOLID, col, dcol), en->xf_main);
    } else if (type == SHAPE_CIRCLE) {
        int n = make_circle_pts(size, 100, pts);
        geom_xf(add_geom(e, n, pts, OUTLINE_SOLID, col, dcol), en->xf_main);
    } else if (type == SHAPE_STAR) {
        vec2 sparts[64]; int scounts[8];
        int nsp = o_star_decomposition(star_out - SHAPE_LINE_THICKNESS, star_in - SHAPE_LINE_THICKNESS, sparts, scounts, 8);
        int off = 0;
        for (int p = 0; p < nparts; p++) {
            geom_xf(add_geom(e, part_counts[p], parts + off, OUTLINE_NONE, dcol, NULL), en->xf_main);
            off += part_counts[p];
        }
        off = 0;
        for (int p = 0; p < nsp; p++) {
            geom_xf(add_geom(e, scounts[p], sparts + off, OUTLINE_NONE, col, NULL), en->xf_main);
            off += scounts[p];
        }
    } else {
        geom_xf(add_geom(e, npoly, poly, OUTLINE_SOLID, col, dcol), en->xf_main);
    }
}

/* ---------------- pose randomisation (geom.py:116-384) ------------------- */
static void ent_bodies(OEnv *e, const OEntity *en, int *ids, int *n) {
    *n = 0;
    if (en->kind == ENT_GOAL) { ids[(*n)++] = -1; return; }
    for (int i = 0; i < en->nbodies; i++) ids[(*n)++] = en->body0 + i;
}

static vec2 body_pos(OEnv *e, const OEntity *en, int bi) {
    if (bi < 0) return e->space.shapes[en->shape0].sp;
    return e->space.bodies[bi].p;
}
static double body_angle(OEnv *e, int bi) { return bi < 0 ? 0.0 : e->space.bodies[bi].a; }

static void reindex_entity(OEnv *e, const OEntity *en) {
    for (int i = 0; i < en->nshapes; i++) ophys_shape_update(&e->space, en->shape0 + i);
}

/* geom.py:362-384 pm_shift_bodies */
static void shift_bodies(OEnv *e, OEntity *en, vec2 position, double angle) {
    int ids[8], n;
    ent_bodies(e, en, ids, &n);
    double root_angle = body_angle(e, ids[0]);
    vec2 root_pos = body_pos(e, en, ids[0]);
    for (int k = 0; k < n; k++) {
        int bi = ids[k];
        if (bi < 0) {
            /* static goal body: rand_rot is always False for goals */
            double lad = 0.0 - root_angle; (void)lad;
            vec2 d = v2(e->space.shapes[en->shape0].sp.x - root_pos.x, e->space.shapes[en->shape0].sp.y - root_pos.y);
            vec2 r = rotated(d, angle - root_angle);
            e->space.shapes[en->shape0].sp = v2(position.x + r.x, position.y + r.y);
            continue;
        }
        OBody *b = &e->space.bodies[bi];
        double local_angle_delta = b->a - root_angle;
        vec2 local_pos_delta = v2(b->p.x - root_pos.x, b->p.y - root_pos.y);
        ophys_body_set_angle(&e->space, bi, angle + local_angle_delta);
        vec2 r = rotated(local_pos_delta, angle - root_angle);
        ophys_body_set_position(&e->space, bi, v2(position.x + r.x, position.y + r.y));
    }
    reindex_entity(e, en);
}

static void set_ent_categories(OEnv *e, const OEntity *en, uint32_t cat) {
    for (int i = 0; i < en->nshapes; i++) e->space.shapes[en->shape0 + i].categories = cat;
}

/* returns 0 on success, -1 on PlacementError */
static int randomise_pose(OEnv *e, OEntity *en, int rand_pos, int rand_rot, double pos_limit, double rot_limit,
                          const uint8_t *ign) {
    int ids[8], n;
    ent_bodies(e, en, ids, &n);
    double orig_angle = body_angle(e, ids[0]);
    vec2 orig_pos = body_pos(e, en, ids[0]);
    /* saved state for PlacementError rollback */
    vec2 saved_p[8]; double saved_a[8]; vec2 saved_sp = v2(0, 0);
    for (int k = 0; k < n; k++) {
        if (ids[k] >= 0) { saved_p[k] = e->space.bodies[ids[k]].p; saved_a[k] = e->space.bodies[ids[k]].a; }
        else saved_sp = e->space.shapes[en->shape0].sp;
    }
    double al = -1, ar = 1, ab = -1, at = 1;
    double xlo = al, xhi = ar, ylo = ab, yhi = at;
    if (pos_limit >= 0) {
        xlo = fmax(al, orig_pos.x - pos_limit); xhi = fmin(ar, orig_pos.x + pos_limit);
        ylo = fmax(ab, orig_pos.y - pos_limit); yhi = fmin(at, orig_pos.y + pos_limit);
        /* python max/min keep the first argument on ties; values are equal either way */
    }
    double rmin = -M_PI, rmax = M_PI;
    if (rot_limit >= 0) { rmin = orig_angle - rot_limit; rmax = orig_angle + rot_limit; }
    for (int tries = 0; tries < e->max_tries; tries++) {
        vec2 npos = orig_pos;
        if (rand_pos) {
            double x = o_mt_uniform(&e->rng, xlo, xhi);
            double y = o_mt_uniform(&e->rng, ylo, yhi);
            npos = v2(x, y);
        }
        double nang = rand_rot ? o_mt_uniform(&e->rng, rmin, rmax) : orig_angle;
        shift_bodies(e, en, npos, nang);
        int reject = 0;
        for (int i = 0; i < en->nshapes && !reject; i++)
            if (ophys_shape_query_any_ign(&e->space, en->shape0 + i, ign)) reject = 1;
        if (!reject) return 0;
    }
    for (int k = 0; k < n; k++) {
        if (ids[k] >= 0) {
            ophys_body_set_angle(&e->space, ids[k], saved_a[k]);
            ophys_body_set_position(&e->space, ids[k], saved_p[k]);
        } else e->space.shapes[en->shape0].sp = saved_sp;
    }
    reindex_entity(e, en);
    return -1;
}

/* geom.py:281-341 */
static void randomise_all_poses_ign(OEnv *e, const int *ents, int n, const int *rand_rot, double pos_limit,
                                    const double *rot_limits, const uint8_t *ign) {
    for (int retry = 0; retry < 10; retry++) {
        uint32_t saved[O_MAX_ENTS];
        for (int k = 0; k < n; k++) {
            saved[k] = e->space.shapes[e->ents[ents[k]].shape0].categories;
            set_ent_categories(e, &e->ents[ents[k]], 0);
        }
        int failed = 0;
        for (int k = 0; k < n; k++) {
            OEntity *en = &e->ents[ents[k]];
            set_ent_categories(e, en, saved[k]);
            if (randomise_pose(e, en, 1, rand_rot[k], pos_limit, rot_limits[k], ign) != 0) { failed = 1; break; }
        }
        if (!failed) return;
        e->placement_retries++; /* test instrumentation: failed whole-layout retries of this reset */
    }
    e->placement_error = 1;
}

static void randomise_all_poses(OEnv *e, const int *ents, int n, const int *rand_rot, double pos_limit,
                                const double *rot_limits) {
    randomise_all_poses_ign(e, ents, n, rand_rot, pos_limit, rot_limits, NULL);
}

/* ignore set of an entity's shapes (ignore_shapes=entity.shapes) */
static void ign_add(uint8_t *ign, const OEntity *en) {
    for (int i = 0; i < en->nshapes; i++) ign[en->shape0 + i] = 1;
}

/* geom.py:344-359 */
static void randomise_hw(OEnv *e, double mn, double mx, double ch, double cw, double linf, double *h, double *w) {
    double lo0 = mn, lo1 = mn, hi0 = mx, hi1 = mx;
    if (linf >= 0) {
        lo0 = fmax(lo0, ch - linf); lo1 = fmax(lo1, cw - linf);
        hi0 = fmin(hi0, ch + linf); hi1 = fmin(hi1, cw + linf);
    }
    *h = o_mt_uniform(&e->rng, lo0, hi0);
    *w = o_mt_uniform(&e->rng, lo1, hi1);
}

/* ---------------- tasks --------------------------------------------------- */
static const int SHAPE_COLOURS[4] = {COL_RED, COL_GREEN, COL_BLUE, COL_YELLOW};
static const int SHAPE_TYPES[4] = {SHAPE_SQUARE, SHAPE_PENTAGON, SHAPE_STAR, SHAPE_CIRCLE};
#define JITTER_POS_BOUND (1 * 0.05 / 2.0)
#define JITTER_ROT_BOUND (0.05 * M_PI)
#define JITTER_TARGET_BOUND (0.05 * (0.8 - 0.5) / 2)

static void reset_move_to_region(OEnv *e) {
    int f = e->flags;
    double gx = -0.62, gy = -0.17, gh = 0.76, gw = 0.75;
    if (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) {
        double bound = (f & RAND_LAYOUT_MINOR) ? JITTER_TARGET_BOUND : -1;
        randomise_hw(e, 0.5, 0.8, gh, gw, bound, &gh, &gw);
    }
    int colour = COL_BLUE;
    if (f & RAND_COLOUR) colour = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
    add_goal(e, gx, gy, gh, gw, colour);
    int goal = e->nents - 1;
    add_robot(e, v2(0.058, 0.53), -2.13);
    int robot = e->nents - 1;
    if (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) {
        int ents[2] = {goal, robot}, rr[2] = {0, 1};
        double rl[2] = {-1, -1};
        double pl = -1;
        if (f & RAND_LAYOUT_MINOR) { pl = JITTER_POS_BOUND; rl[1] = JITTER_ROT_BOUND; }
        randomise_all_poses(e, ents, 2, rr, pl, rl);
    }
}

static void reset_move_to_corner(OEnv *e) {
    int f = e->flags;
    double rx = o_mt_double(&e->rng), ry = o_mt_double(&e->rng);
    add_robot(e, v2(rx, ry), 0.55 * M_PI);
    int robot = e->nents - 1;
    int colour = COL_RED, type = SHAPE_SQUARE;
    if (f & RAND_COLOUR) colour = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
    if (f & RAND_SHAPE_TYPE) type = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
    add_block(e, type, colour, v2(0.1, -0.65), 0.13 * M_PI, 0);
    int shape = e->nents - 1;
    if (f & RAND_LAYOUT_MINOR) {
        int ents[2] = {robot, shape}, rr[2] = {1, 1};
        double rl[2] = {JITTER_ROT_BOUND, JITTER_ROT_BOUND};
        randomise_all_poses(e, ents, 2, rr, JITTER_POS_BOUND, rl);
    }
}

/* cluster.py:219-291 defaults */
static const int CC_COLOURS[8] = {COL_BLUE, COL_BLUE, COL_BLUE, COL_GREEN, COL_GREEN, COL_RED, COL_YELLOW, COL_YELLOW};
static const int CC_TYPES[8] = {SHAPE_CIRCLE, SHAPE_STAR, SHAPE_SQUARE, SHAPE_PENTAGON, SHAPE_PENTAGON,
                                SHAPE_SQUARE, SHAPE_STAR, SHAPE_PENTAGON};
static const double CC_POSES[8][3] = {{-0.5147, 0.14149, -0.38871}, {-0.1347, -0.71414, 1.0533},
                                      {-0.74247, -0.097592, 1.1571}, {-0.077363, -0.42964, -0.64379},
                                      {0.51978, 0.1853, -1.1762},    {-0.5278, -0.21642, 2.9356},
                                      {-0.54039, 0.48292, 0.072818}, {-0.16761, 0.64303, -2.3255}};
static const double CC_ROBOT[3] = {0.71692, -0.34374, 0.83693};
static const int CS_COLOURS[8] = {COL_YELLOW, COL_BLUE, COL_RED, COL_RED, COL_GREEN, COL_YELLOW, COL_BLUE, COL_GREEN};
static const int CS_TYPES[8] = {SHAPE_SQUARE, SHAPE_PENTAGON, SHAPE_PENTAGON, SHAPE_PENTAGON,
                                SHAPE_CIRCLE, SHAPE_STAR, SHAPE_STAR, SHAPE_CIRCLE};
static const double CS_POSES[8][3] = {{-0.414, 0.297, -1.731}, {0.068, 0.705, 2.184},  {0.821, 0.220, 0.650},
                                      {-0.461, -0.749, -2.673}, {0.867, -0.149, -2.215}, {-0.785, -0.140, -0.405},
                                      {-0.305, -0.226, 1.341},  {0.758, -0.708, -2.140}};
static const double CS_ROBOT[3] = {0.286, -0.202, -1.878};

static void reset_cluster(OEnv *e, int by_type) {
    int f = e->flags;
    const int *dcol = by_type ? CS_COLOURS : CC_COLOURS;
    const int *dtyp = by_type ? CS_TYPES : CC_TYPES;
    const double(*dpose)[3] = by_type ? CS_POSES : CC_POSES;
    const double *rp = by_type ? CS_ROBOT : CC_ROBOT;
    int n = 8;
    double poses[16][3];
    if (f & RAND_SHAPE_COUNT) {
        n = (int)o_mt_randint(&e->rng, 7, 10 + 1);
        for (int i = 0; i < n; i++) poses[i][0] = poses[i][1] = poses[i][2] = 0.0;
    } else {
        for (int i = 0; i < n; i++) memcpy(poses[i], dpose[i], sizeof(poses[i]));
    }
    int cols[16], types[16];
    if (f & RAND_COLOUR) {
        for (int i = 0; i < 4; i++) cols[i] = SHAPE_COLOURS[i];
        for (int i = 4; i < n; i++) cols[i] = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
        for (int i = n - 1; i >= 1; i--) {
            int j = (int)o_mt_interval(&e->rng, (uint64_t)i);
            int t = cols[i]; cols[i] = cols[j]; cols[j] = t;
        }
    } else memcpy(cols, dcol, sizeof(int) * 8);
    if (f & RAND_SHAPE_TYPE) {
        for (int i = 0; i < 4; i++) types[i] = SHAPE_TYPES[i];
        for (int i = 4; i < n; i++) types[i] = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
        for (int i = n - 1; i >= 1; i--) {
            int j = (int)o_mt_interval(&e->rng, (uint64_t)i);
            int t = types[i]; types[i] = types[j]; types[j] = t;
        }
    } else memcpy(types, dtyp, sizeof(int) * 8);
    int first_block = e->nents;
    for (int i = 0; i < n; i++) add_block(e, types[i], cols[i], v2(poses[i][0], poses[i][1]), poses[i][2], 0);
    add_robot(e, v2(rp[0], rp[1]), rp[2]);
    if (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) {
        int ents[16], rr[16]; double rl[16];
        double pl = (f & RAND_LAYOUT_FULL) ? -1 : JITTER_POS_BOUND;
        ents[0] = e->robot;
        for (int i = 0; i < n; i++) ents[1 + i] = first_block + i;
        for (int i = 0; i <= n; i++) { rr[i] = 1; rl[i] = (f & RAND_LAYOUT_FULL) ? -1 : JITTER_ROT_BOUND; }
        randomise_all_poses(e, ents, n + 1, rr, pl, rl);
    }
}

static void reset_match_regions(OEnv *e) {
    int f = e->flags;
    int target_colour = COL_GREEN;
    if (f & RAND_COLOUR) target_colour = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
    int dcols[3], nd = 0;
    for (int i = 0; i < 4; i++) if (SHAPE_COLOURS[i] != target_colour) dcols[nd++] = SHAPE_COLOURS[i];
    double th = 0.7, tw = 0.6, tx = 0.1, ty = 0.7;
    if (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) {
        double bound = (f & RAND_LAYOUT_MINOR) ? JITTER_TARGET_BOUND : -1;
        randomise_hw(e, 0.5, 0.8, th, tw, bound, &th, &tw);
    }
    add_goal(e, tx, ty, th, tw, target_colour);
    int sensor = e->nents - 1;
    int dtt[2] = {SHAPE_STAR, SHAPE_SQUARE};
    int ddt[3][2] = {{0, 0}, {SHAPE_PENTAGON, 0}, {SHAPE_CIRCLE, SHAPE_PENTAGON}};
    int ddc[3] = {0, 1, 2};
    double dtp[2][3] = {{0.8, -0.7, 2.37}, {-0.68, 0.72, 1.28}};
    double ddp[3][2][3] = {{{0}}, {{-0.05, -0.2, -1.09}}, {{-0.75, -0.55, 2.78}, {0.3, -0.82, -1.15}}};
    int tcount = 2, dcount[3] = {0, 1, 2};
    if (f & RAND_SHAPE_COUNT) {
        tcount = (int)o_mt_randint(&e->rng, 1, 2 + 1);
        for (int i = 0; i < 3; i++) dcount[i] = (int)o_mt_randint(&e->rng, 0, 2 + 1);
    } else {
        for (int i = 0; i < 3; i++) dcount[i] = ddc[i];
    }
    int ttypes[2], dtypes[3][2];
    if (f & RAND_SHAPE_TYPE) {
        for (int i = 0; i < tcount; i++) ttypes[i] = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
        for (int c = 0; c < 3; c++)
            for (int i = 0; i < dcount[c]; i++) dtypes[c][i] = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
    } else {
        memcpy(ttypes, dtt, sizeof(ttypes));
        memcpy(dtypes, ddt, sizeof(dtypes));
    }
    int full = (f & RAND_LAYOUT_FULL) != 0;
    int first_block = e->nents;
    for (int i = 0; i < tcount; i++) {
        double x = full ? 0 : dtp[i][0], y = full ? 0 : dtp[i][1], a = full ? 0 : dtp[i][2];
        add_block(e, ttypes[i], target_colour, v2(x, y), a, 1);
    }
    for (int c = 0; c < 3; c++)
        for (int i = 0; i < dcount[c]; i++) {
            double x = full ? 0 : ddp[c][i][0], y = full ? 0 : ddp[c][i][1], a = full ? 0 : ddp[c][i][2];
            add_block(e, dtypes[c][i], dcols[c], v2(x, y), a, 2);
        }
    int nblocks = e->nents - first_block;
    add_robot(e, v2(-0.5, 0.1), -M_PI * 1.2);
    if (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) {
        int ents[16], rr[16]; double rl[16];
        int n = 0;
        ents[n++] = sensor;
        ents[n++] = e->robot;
        for (int i = 0; i < nblocks; i++) ents[n++] = first_block + i;
        double pl = (f & RAND_LAYOUT_MINOR) ? JITTER_POS_BOUND : -1;
        for (int i = 0; i < n; i++) {
            rr[i] = i == 0 ? 0 : 1;
            rl[i] = (f & RAND_LAYOUT_MINOR) ? JITTER_ROT_BOUND : -1;
        }
        randomise_all_poses(e, ents, n, rr, pl, rl);
    }
}

/* make_line.py:13-27 defaults, :86-132 on_reset */
static const int ML_COLOURS[4] = {COL_BLUE, COL_YELLOW, COL_RED, COL_GREEN};
static const int ML_TYPES[4] = {SHAPE_STAR, SHAPE_CIRCLE, SHAPE_STAR, SHAPE_PENTAGON};
static const double ML_POSES[4][3] = {{0.790, -0.820, -0.721}, {-0.177, 0.383, -1.733},
                                      {-0.051, -0.128, 2.696}, {-0.292, -0.745, -0.159}};
static const double ML_ROBOT[3] = {0.702, -0.255, 0.347};

static void reset_make_line(OEnv *e) {
    int f = e->flags;
    int n = 4;
    double poses[4][3];
    memcpy(poses, ML_POSES, sizeof(poses));
    if (f & RAND_SHAPE_COUNT) { /* rng.randint(MIN_BLOCKS, MAX_BLOCKS + 1); block_poses[:1] * n */
        n = (int)o_mt_randint(&e->rng, 3, 4 + 1);
        for (int i = 0; i < n; i++) memcpy(poses[i], ML_POSES[0], sizeof(poses[i]));
    }
    int cols[4], types[4];
    memcpy(cols, ML_COLOURS, sizeof(cols));
    memcpy(types, ML_TYPES, sizeof(types));
    /* rng.choice(list, size=n) = randint(0, len, size=n) */
    if (f & RAND_COLOUR) for (int i = 0; i < n; i++) cols[i] = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
    if (f & RAND_SHAPE_TYPE) for (int i = 0; i < n; i++) types[i] = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
    int first_block = e->nents;
    for (int i = 0; i < n; i++) add_block(e, types[i], cols[i], v2(poses[i][0], poses[i][1]), poses[i][2], 0);
    add_robot(e, v2(ML_ROBOT[0], ML_ROBOT[1]), ML_ROBOT[2]);
    if (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) { /* all_ents = (robot, *blocks), rand_rot everywhere */
        int ents[8], rr[8]; double rl[8];
        int minor = (f & RAND_LAYOUT_MINOR) != 0;
        ents[0] = e->robot;
        for (int i = 0; i < n; i++) ents[1 + i] = first_block + i;
        for (int i = 0; i <= n; i++) { rr[i] = 1; rl[i] = minor ? JITTER_ROT_BOUND : -1; }
        randomise_all_poses(e, ents, n + 1, rr, minor ? JITTER_POS_BOUND : -1, rl);
    }
}

/* find_dupe.py:7-37 defaults, :62-199 on_reset */
static const int FD_OUT_TYPES[6] = {SHAPE_PENTAGON, SHAPE_CIRCLE, SHAPE_CIRCLE, SHAPE_SQUARE, SHAPE_STAR, SHAPE_PENTAGON};
static const int FD_OUT_COLOURS[6] = {COL_GREEN, COL_RED, COL_RED, COL_YELLOW, COL_BLUE, COL_YELLOW};
static const double FD_OUT_POSES[6][3] = {{-0.066751, 0.7552, -2.9266}, {-0.05195, 0.31468, 1.5418},
                                          {0.57528, -0.46865, -2.2141},  {0.40594, -0.74977, 0.24582},
                                          {0.45254, 0.3681, -1.0834},    {0.76849, -0.10652, 0.10028}};

static void reset_find_dupe(OEnv *e) {
    int f = e->flags;
    const int layout = (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) != 0, minor = (f & RAND_LAYOUT_MINOR) != 0;
    int qcol = COL_YELLOW, qtype = SHAPE_PENTAGON;
    int cols[8], types[8];
    memcpy(cols, FD_OUT_COLOURS, sizeof(FD_OUT_COLOURS));
    memcpy(types, FD_OUT_TYPES, sizeof(FD_OUT_TYPES));
    int n_out = 6;
    if (f & RAND_SHAPE_COUNT) n_out = (int)o_mt_randint(&e->rng, 1, 5 + 1) + 1;
    int nd = n_out - 1;
    if (f & RAND_COLOUR) {
        qcol = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
        for (int i = 0; i < nd; i++) cols[i] = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
        cols[nd] = qcol;
    }
    if (f & RAND_SHAPE_TYPE) {
        qtype = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
        for (int i = 0; i < nd; i++) types[i] = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
        types[nd] = qtype;
    }
    double tx = -0.72, ty = -0.22, th = 0.67, tw = 0.72;
    if (layout) randomise_hw(e, 0.5, 0.8, th, tw, minor ? JITTER_TARGET_BOUND : -1, &th, &tw);
    add_goal(e, tx, ty, th, tw, qcol);
    int sensor = e->nents - 1;
    int first = e->nents;
    for (int i = 0; i < n_out; i++) {
        const int cnt = (f & RAND_SHAPE_COUNT) != 0; /* [((0, 0), 0)] * n_out */
        double x = cnt ? 0 : FD_OUT_POSES[i][0], y = cnt ? 0 : FD_OUT_POSES[i][1], a = cnt ? 0 : FD_OUT_POSES[i][2];
        /* role 1: in the target set (same colour and shape as the query), 2: distractor */
        add_block(e, types[i], cols[i], v2(x, y), a, (cols[i] == qcol && types[i] == qtype) ? 1 : 2);
    }
    add_block(e, qtype, qcol, v2(-0.33, -0.49), -0.51, 1); /* the query block */
    int query = e->nents - 1;
    add_robot(e, v2(-0.57, 0.25), 3.83);
    if (layout) {
        int ents[16], rr[16]; double rl[16]; int n = 0;
        ents[n++] = sensor; ents[n++] = e->robot;
        for (int i = 0; i < n_out; i++) ents[n++] = first + i;
        for (int i = 0; i < n; i++) { rr[i] = i != 0; rl[i] = minor ? JITTER_ROT_BOUND : -1; }
        uint8_t ign[O_MAX_SHAPES] = {0};
        ign_add(ign, &e->ents[query]);
        randomise_all_poses_ign(e, ents, n, rr, minor ? JITTER_POS_BOUND : -1, rl, ign);
        if (e->placement_error) return;
        /* the query block last, mostly inside the (placed) sensor region */
        double lim = fmin(th, tw) / 2 - shape_rad() / 2;
        lim = lim > 0 ? lim : 0;
        if (minor) lim = fmin(JITTER_POS_BOUND, lim);
        OEntity *q = &e->ents[query];
        shift_bodies(e, q, e->space.shapes[e->ents[sensor].shape0].sp, e->space.bodies[q->body0].a);
        uint8_t ign2[O_MAX_SHAPES] = {0};
        ign_add(ign2, &e->ents[sensor]);
        if (randomise_pose(e, q, 1, 1, lim, minor ? JITTER_ROT_BOUND : -1, ign2) != 0) e->placement_error = 1;
    }
}

/* fix_colour.py:12-41 defaults, :67-176 on_reset */
static const int FC_BLOCK_COLOURS[3] = {COL_GREEN, COL_GREEN, COL_BLUE};
static const int FC_BLOCK_TYPES[3] = {SHAPE_PENTAGON, SHAPE_SQUARE, SHAPE_PENTAGON};
static const double FC_BLOCK_POSES[3][3] = {{0.289, 0.030, 0.307}, {0.133, -0.561, 1.699}, {-0.336, 0.000, -1.529}};
static const double FC_REGIONS[3][4] = {{-0.032, 0.348, 0.427, 0.468}, {0.019, -0.391, 0.460, 0.458},
                                        {-0.681, 0.196, 0.498, 0.418}};
static const int FC_REGION_COLOURS[3] = {COL_GREEN, COL_GREEN, COL_RED};

static void reset_fix_colour(OEnv *e) {
    int f = e->flags;
    const int layout = (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) != 0, minor = (f & RAND_LAYOUT_MINOR) != 0;
    int n = 3;
    double poses[3][3], regions[3][4];
    memcpy(poses, FC_BLOCK_POSES, sizeof(poses));
    memcpy(regions, FC_REGIONS, sizeof(regions));
    if (f & RAND_SHAPE_COUNT) {
        n = (int)o_mt_randint(&e->rng, 2, 3 + 1);
        for (int i = 0; i < n; i++) { memcpy(poses[i], FC_BLOCK_POSES[0], sizeof(poses[i])); memcpy(regions[i], FC_REGIONS[0], sizeof(regions[i])); }
    }
    int rcols[3], bcols[3], types[3];
    memcpy(rcols, FC_REGION_COLOURS, sizeof(rcols));
    memcpy(bcols, FC_BLOCK_COLOURS, sizeof(bcols));
    memcpy(types, FC_BLOCK_TYPES, sizeof(types));
    if (f & RAND_COLOUR) {
        for (int i = 0; i < n; i++) rcols[i] = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
        for (int i = 0; i < n; i++) bcols[i] = rcols[i];
        int odd = (int)o_mt_randint(&e->rng, 0, n);
        int nc = (int)o_mt_randint(&e->rng, 0, 4 - 1);
        if (SHAPE_COLOURS[nc] == bcols[odd]) nc++;
        bcols[odd] = SHAPE_COLOURS[nc];
    }
    if (f & RAND_SHAPE_TYPE) for (int i = 0; i < n; i++) types[i] = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
    if (layout)
        for (int i = 0; i < n; i++)
            randomise_hw(e, 0.4, 0.5, regions[i][2], regions[i][3], minor ? JITTER_TARGET_BOUND : -1, &regions[i][2],
                         &regions[i][3]);
    int first_sensor = e->nents;
    for (int i = 0; i < n; i++) add_goal(e, regions[i][0], regions[i][1], regions[i][2], regions[i][3], rcols[i]);
    int first_block = e->nents;
    /* role 1: the block matches its region's colour (must stay), 2: the odd one out (must leave) */
    for (int i = 0; i < n; i++)
        add_block(e, types[i], bcols[i], v2(poses[i][0], poses[i][1]), poses[i][2], bcols[i] == rcols[i] ? 1 : 2);
    add_robot(e, v2(0.368, 0.586), 0.718);
    if (layout) {
        int ents[8], rr[8]; double rl[8]; int m = 0;
        for (int i = 0; i < n; i++) ents[m++] = first_sensor + i;
        ents[m++] = e->robot;
        for (int i = 0; i < m; i++) { rr[i] = i == n; rl[i] = minor ? JITTER_ROT_BOUND : -1; }
        uint8_t ign[O_MAX_SHAPES] = {0};
        for (int i = 0; i < n; i++) ign_add(ign, &e->ents[first_block + i]);
        randomise_all_poses_ign(e, ents, m, rr, minor ? JITTER_POS_BOUND : -1, rl, ign);
        if (e->placement_error) return;
        for (int i = 0; i < n; i++) {
            OEntity *b = &e->ents[first_block + i];
            shift_bodies(e, b, e->space.shapes[e->ents[first_sensor + i].shape0].sp, e->space.bodies[b->body0].a);
        }
        for (int i = 0; i < n; i++) {
            double lim = fmin(regions[i][2], regions[i][3]) / 2 - shape_rad();
            lim = lim > 0 ? lim : 0;
            if (minor) lim = fmin(JITTER_POS_BOUND, lim);
            uint8_t ign2[O_MAX_SHAPES] = {0};
            ign_add(ign2, &e->ents[first_sensor + i]);
            if (randomise_pose(e, &e->ents[first_block + i], 1, 1, lim, minor ? JITTER_ROT_BOUND : -1, ign2) != 0) {
                e->placement_error = 1;
                return;
            }
        }
    }
}

/* pick_and_place.py:30-85 */
static void reset_pick_and_place(OEnv *e) {
    int f = e->flags;
    add_robot(e, v2(0.0, 0.0), 0.55 * M_PI); /* added first: arena, robot, shapes */
    int cols[3], types[3], first = e->nents;
    for (int i = 0; i < 3; i++) { /* per shape: colour draw, then type draw (rng.choice of one element) */
        cols[i] = COL_RED; types[i] = SHAPE_SQUARE;
        if (f & RAND_COLOUR) cols[i] = SHAPE_COLOURS[o_mt_randint(&e->rng, 0, 4)];
        if (f & RAND_SHAPE_TYPE) types[i] = SHAPE_TYPES[o_mt_randint(&e->rng, 0, 4)];
    }
    for (int i = 0; i < 3; i++) add_block(e, types[i], cols[i], v2(0.1, -0.65), 0.13 * M_PI, 0);
    for (int k = 0; k < 4; k++) {
        if (SHAPE_TYPES[k] == types[0]) e->target_type_id = k;
        if (SHAPE_COLOURS[k] == cols[0]) e->target_colour_id = k;
    }
    double tx = o_mt_double(&e->rng), ty = o_mt_double(&e->rng); /* rng.rand(2) * 2 - 1 */
    e->target_pos = v2(tx * 2 - 1, ty * 2 - 1);
    int valid[3], nv = 0;
    for (int i = 0; i < 3; i++) if (types[i] == types[0] && cols[i] == cols[0]) valid[nv++] = first + i;
    e->target_ent = valid[o_mt_randint(&e->rng, 0, nv)]; /* rng.choice(valid_target_shapes) */
    if (f & (RAND_LAYOUT_MINOR | RAND_LAYOUT_FULL)) { /* rand_poses: unrestricted */
        int ents[4] = {e->robot, first, first + 1, first + 2}, rr[4] = {1, 1, 1, 1};
        double rl[4] = {-1, -1, -1, -1};
        randomise_all_poses(e, ents, 4, rr, -1, rl);
    }
}

void oscene_reset(OEnv *e) {
    e->episode_steps = 0;
    e->nents = 0; e->ngeoms = 0; e->nxf = 0; e->robot = -1; e->goal = -1; e->star_groups = 0;
    ophys_init(&e->space);
    /* PhysicsVariables (base_env.py:49-57, 210-215; phys_vars.py:512-537) */
    static const double PV_DEF[5] = {3, 1, 4, 1.5, 0.1};
    static const double PV_LO[5] = {2.2, 0.7, 2.5, 1.0, 0.07};
    static const double PV_HI[5] = {3.5, 1.5, 4.5, 1.8, 0.15};
    for (int i = 0; i < 5; i++)
        e->pv[i] = (e->flags & RAND_DYNAMICS) ? o_mt_uniform(&e->rng, PV_LO[i], PV_HI[i]) : PV_DEF[i];
    add_arena(e);
    switch (e->task) {
    case TASK_MOVE_TO_REGION: reset_move_to_region(e); break;
    case TASK_MOVE_TO_CORNER: reset_move_to_corner(e); break;
    case TASK_CLUSTER_COLOUR: reset_cluster(e, 0); break;
    case TASK_CLUSTER_SHAPE: reset_cluster(e, 1); break;
    case TASK_MATCH_REGIONS: reset_match_regions(e); break;
    case TASK_MAKE_LINE: reset_make_line(e); break;
    case TASK_FIND_DUPE: reset_find_dupe(e); break;
    case TASK_FIX_COLOUR: reset_fix_colour(e); break;
    case TASK_PICK_AND_PLACE: reset_pick_and_place(e); break;
    }
    /* Robot.__init__ control state (entities.py:219-228, 287) */
    e->rel_turn = 0.0;
    e->target_speed = 0.0;
    e->target_finger = 0.0;
}

/* ---------------- robot control (entities.py:435-476) -------------------- */
/* ACTION_NUMS_FLAGS_NAMES (entities.py:162-182): ud 0 none 1 up 2 down; lr 0/4 left/8 right; grip 16 open/32 close */
void oscene_set_action(OEnv *e, int action) {
    static const int UD[18] = {0, 1, 2, 0, 1, 2, 0, 1, 2, 0, 1, 2, 0, 1, 2, 0, 1, 2};
    static const int LR[18] = {0, 0, 0, 4, 4, 4, 8, 8, 8, 0, 0, 0, 4, 4, 4, 8, 8, 8};
    int flags = UD[action] | LR[action] | (action < 9 ? 16 : 32);
    double radius = ROBOT_RAD;
    e->rel_turn = 0.0;
    e->target_speed = 0.0;
    if (flags & 1) e->target_speed += 4.0 * radius;
    if (flags & 2) e->target_speed -= 3.0 * radius;
    if ((flags & 1) && (flags & 2)) e->target_speed = 0.0;
    if (flags & 4) e->rel_turn += 1.5;
    if (flags & 8) e->rel_turn -= 1.5;
    if (flags & 16) e->target_finger = M_PI / 8;
    else if (flags & 32) e->target_finger = -0.0;
}

/* the decoded control targets of one action (target_speed, rel_turn_angle, target_finger_angle) */
void o_action_decode(int action, double out[3]) {
    OEnv *e = (OEnv *)calloc(1, sizeof(OEnv));
    oscene_set_action(e, action);
    out[0] = e->target_speed; out[1] = e->rel_turn; out[2] = e->target_finger;
    free(e);
}

void oscene_robot_update(OEnv *e) {
    OEntity *r = &e->ents[e->robot];
    OSpace *s = &e->space;
    OBody *body = &s->bodies[r->body0];
    int control = r->body0 + 1;
    ophys_body_set_angle(s, control, body->a + e->rel_turn);
    double c = body->rc, sn = body->rs;
    double ts = e->target_speed;
    s->bodies[control].v = v2(c * 0.0 - sn * ts, c * ts + sn * 0.0);
    /* motors are constraints 6 and 9 of the robot (pivot, gear, 2 springs, then per finger pivot, limit, motor) */
    int cons0 = -1;
    for (int i = 0; i < s->ncons; i++) if (s->cons[i].a == control) { cons0 = i; break; }
    for (int k = 0; k < 2; k++) {
        int side = k == 0 ? -1 : 1;
        OBody *fb = &s->bodies[r->body0 + 4 + k];
        double rel_angle = fb->a - body->a;
        double angle_error = rel_angle + side * e->target_finger;
        double x = angle_error * 10;
        double tr = (x < 1) ? x : 1;       /* min(1, x) */
        tr = (tr > -1) ? tr : -1;          /* max(-1, .) */
        if (fabs(tr) < 1e-4) tr = 0.0;
        s->cons[cons0 + 6 + 3 * k].rate = tr;
    }
}

/* ---------------- pre_draw (entities.py:478-491, 751-754, 865-868) -------- */
void oscene_pre_draw(OEnv *e) {
    OSpace *s = &e->space;
    for (int i = 0; i < e->nents; i++) {
        OEntity *en = &e->ents[i];
        if (en->kind == ENT_ROBOT) {
            OBody *b = &s->bodies[en->body0];
            o_transform_trs(b->p.x, b->p.y, b->a, 1.0, 1.0, e->xf[en->xf_main].m);
            for (int k = 0; k < 2; k++) {
                OBody *fb = &s->bodies[en->body0 + 4 + k];
                o_transform_trs(fb->p.x, fb->p.y, fb->a, 1.0, 1.0, e->xf[en->xf_aux[k]].m);
                OBody *eb = &s->bodies[en->body0 + 2 + k];
                o_transform_trs(0.0, 0.0, eb->a - b->a, 1.0, 1.0, e->xf[en->xf_aux[2 + k]].m);
            }
        } else if (en->kind == ENT_BLOCK) {
            OBody *b = &s->bodies[en->body0];
            o_transform_trs(b->p.x, b->p.y, b->a, 1.0, 1.0, e->xf[en->xf_main].m);
        } else if (en->kind == ENT_GOAL) {
            vec2 p = s->shapes[en->shape0].sp;
            o_transform_trs(p.x, p.y, 0.0, 1.0, 1.0, e->xf[en->xf_main].m);
        }
    }
}

/* ---------------- scoring ---------------------------------------------- */
static double score_move_to_region(OEnv *e) {
    OEntity *g = &e->ents[e->goal];
    const OShape *gs = &e->space.shapes[g->shape0];
    double dist = ophys_poly_point_query(gs, e->space.bodies[e->ents[e->robot].body0].p);
    return dist <= 0 ? 1.0 : 0.0;
}

/* move_to_corner.py:67-77: the ROBOT's distance to the top-left corner (fork quirk: not the block's) */
double o_score_move_to_corner(double rx, double ry) {
    double dx = -1.0 - rx, dy = 1.0 - ry;
    double dist = sqrt(fma(dy, dy, dx * dx)); /* np.linalg.norm -> BLAS ddot */
    double succeed = sqrt(2.0) / 2, furthest = sqrt(2.0);
    double drange = furthest - succeed;
    double v = furthest - dist;
    double score = (v > 0.0 ? v : 0.0) / drange;
    return score < 1.0 ? score : 1.0;
}

static double score_move_to_corner(OEnv *e) {
    vec2 p = e->space.bodies[e->ents[e->robot].body0].p;
    return o_score_move_to_corner(p.x, p.y);
}

/* cluster.py:166-216 on block positions: val[i] = the rank of block i's characteristic value among the
 * values present (np.unique order), blocks in entity (insertion) order */
double o_cluster_score(int nblocks, const int *val, const double *x, const double *y) {
    int present[4] = {0, 0, 0, 0};
    for (int i = 0; i < nblocks; i++) present[val[i]] = 1;
    int nvals = 0;
    for (int k = 0; k < 4; k++) nvals += present[k];
    double cx[4], cy[4];
    for (int c = 0; c < nvals; c++) {
        double sx = 0, sy = 0; int cnt = 0;
        for (int i = 0; i < nblocks; i++) {
            if (val[i] != c) continue;
            if (cnt == 0) { sx = x[i]; sy = y[i]; } else { sx += x[i]; sy += y[i]; }
            cnt++;
        }
        cx[c] = sx / cnt; cy[c] = sy / cnt;
    }
    int n_blocks = 0, n_correct = 0;
    for (int c = 0; c < nvals; c++) {
        for (int i = 0; i < nblocks; i++) {
            if (val[i] != c) continue;
            n_blocks++;
            double sse[4];
            for (int k = 0; k < nvals; k++) {
                double dx = x[i] - cx[k], dy = y[i] - cy[k];
                sse[k] = dx * dx + dy * dy;
            }
            double true_sse = sse[c], nearest_bad = INFINITY;
            for (int k = 0; k < nvals; k++) if (k != c && sse[k] < nearest_bad) nearest_bad = sse[k];
            double margin = 2.0 * true_sse;
            n_correct += (sqrt(true_sse) < sqrt(nearest_bad) - margin);
        }
    }
    double frac = (double)n_correct / (n_blocks > 1 ? n_blocks : 1);
    double v = frac - 0.75;
    return (v > 0 ? v : 0) / (1 - 0.75);
}

static double score_cluster(OEnv *e, int by_type) {
    /* characteristic values: np.unique sorts the str-enum values */
    static const int COLOUR_ORDER[4] = {COL_BLUE, COL_GREEN, COL_RED, COL_YELLOW};
    static const int TYPE_ORDER[4] = {SHAPE_CIRCLE, SHAPE_PENTAGON, SHAPE_SQUARE, SHAPE_STAR};
    const int *order = by_type ? TYPE_ORDER : COLOUR_ORDER;
    int rank_of[4] = {-1, -1, -1, -1}, nvals = 0;
    for (int k = 0; k < 4; k++) {
        for (int i = 0; i < e->nents; i++) {
            OEntity *en = &e->ents[i];
            if (en->kind != ENT_BLOCK) continue;
            if ((by_type ? en->type : en->colour) == order[k]) { rank_of[k] = nvals++; break; }
        }
    }
    int val[O_MAX_ENTS], nb = 0;
    double x[O_MAX_ENTS], y[O_MAX_ENTS];
    for (int i = 0; i < e->nents; i++) {
        OEntity *en = &e->ents[i];
        if (en->kind != ENT_BLOCK) continue;
        const int v = by_type ? en->type : en->colour;
        int k = 0;
        while (order[k] != v) k++;
        val[nb] = rank_of[k];
        x[nb] = e->space.bodies[en->body0].p.x; y[nb] = e->space.bodies[en->body0].p.y;
        nb++;
    }
    return o_cluster_score(nb, val, x, y);
}

/* entities.py:803-863 get_overlapping_ents(com_overlap=True) of goal entity gi over the block
 * entities: in[i] = 1 if every shape of block i overlaps the goal and has its body's position
 * inside the goal's BB */
static void goal_overlap_blocks(OEnv *e, int gi, int *in) {
    OSpace *s = &e->space;
    int gsi = e->ents[gi].shape0;
    ophys_shape_update(s, gsi);
    const OShape *gs = &s->shapes[gsi];
    int overlap[O_MAX_SHAPES] = {0};
    for (int j = 0; j < s->nshapes; j++) {
        if (j == gsi) continue;
        OShape *b = &s->shapes[j];
        if (!(gs->bb_l <= b->bb_r && b->bb_l <= gs->bb_r && gs->bb_b <= b->bb_t && b->bb_b <= gs->bb_t)) continue;
        if ((gs->group != 0 && gs->group == b->group) || (gs->categories & b->mask) == 0 ||
            (b->categories & gs->mask) == 0) continue;
        OCollision info; int sw;
        if (ophys_collide(s, gsi, j, &info, &sw) > 0) {
            /* com_overlap: goal_bb.contains_vect(shape.body.position) */
            vec2 p = b->body >= 0 ? s->bodies[b->body].p : b->sp;
            if (gs->bb_l <= p.x && gs->bb_r >= p.x && gs->bb_b <= p.y && gs->bb_t >= p.y) overlap[j] = 1;
        }
    }
    for (int i = 0; i < e->nents; i++) {
        OEntity *en = &e->ents[i];
        in[i] = 0;
        if (en->kind != ENT_BLOCK) continue;
        int any = 0, all = 1;
        for (int k = 0; k < en->nshapes; k++) {
            if (overlap[en->shape0 + k]) any = 1; else all = 0;
        }
        in[i] = any && all;
    }
}

static double score_match_regions(OEnv *e) {
    int in[O_MAX_ENTS];
    goal_overlap_blocks(e, e->goal, in);
    int n_t = 0, n_d = 0, n_in = 0, total_t = 0;
    for (int i = 0; i < e->nents; i++) {
        OEntity *en = &e->ents[i];
        if (en->kind != ENT_BLOCK) continue;
        if (en->role == 1) total_t++;
        if (in[i]) {
            n_in++;
            if (en->role == 1) n_t++;
            else n_d++;
        }
    }
    double frac = (double)n_t / total_t;
    double contamination = n_in == 0 ? 0.0 : (double)n_d / n_in;
    return frac * (1 - contamination);
}

/* find_dupe.py:202-216 */
static double score_find_dupe(OEnv *e) {
    int in[O_MAX_ENTS];
    goal_overlap_blocks(e, e->goal, in);
    int n_t = 0, n_d = 0, n_in = 0;
    for (int i = 0; i < e->nents; i++) {
        if (!in[i]) continue;
        n_in++;
        if (e->ents[i].role == 1) n_t++; else n_d++;
    }
    double have_two = n_t >= 2 ? 1.0 : 0.0;
    double contamination = n_in == 0 ? 0.0 : (double)n_d / n_in;
    return have_two * (1 - contamination);
}

/* fix_colour.py:181-192: region i (i-th goal) must hold exactly block i if that block matches its
 * colour (role 1), and nothing otherwise */
static double score_fix_colour(OEnv *e) {
    int goals[8], blocks[8], ng = 0, nb = 0;
    for (int i = 0; i < e->nents; i++) {
        if (e->ents[i].kind == ENT_GOAL) goals[ng++] = i;
        if (e->ents[i].kind == ENT_BLOCK) blocks[nb++] = i;
    }
    for (int r = 0; r < ng; r++) {
        int in[O_MAX_ENTS];
        goal_overlap_blocks(e, goals[r], in);
        int cnt = 0;
        for (int i = 0; i < e->nents; i++) cnt += in[i];
        int want = e->ents[blocks[r]].role == 1;
        if (want ? (cnt != 1 || !in[blocks[r]]) : cnt != 0) return 0.0;
    }
    return 1.0;
}

/* make_line.py:33-74 longest_line, in this image's numpy arithmetic: np.linalg.norm of one
 * 2-vector = sqrt(ddot) = sqrt(fma(y, y, x * x)); offs @ unit[:, None] (OpenBLAS gemv) =
 * fma(x, ux, y * uy); np.linalg.norm(..., axis=1) = sqrt(x * x + y * y) */
int o_longest_line(const double *px, const double *py, int n, double inlier_dist, double max_sep) {
    int best = n < 1 ? n : 1;
    for (int i = 0; i < n - 1; i++)
        for (int j = i + 1; j < n; j++) {
            double ox[16], oy[16], proj[16], inl[16];
            for (int k = 0; k < n; k++) { ox[k] = px[k] - px[i]; oy[k] = py[k] - py[i]; }
            const double nrm = sqrt(fma(oy[j], oy[j], ox[j] * ox[j]));
            const double ux = ox[j] / nrm, uy = oy[j] / nrm;
            int ni = 0;
            for (int k = 0; k < n; k++) {
                proj[k] = fma(ox[k], ux, oy[k] * uy);
                const double dx = ox[k] - proj[k] * ux, dy = oy[k] - proj[k] * uy;
                if (sqrt(dx * dx + dy * dy) <= inlier_dist) inl[ni++] = proj[k];
            }
            if (ni <= best) continue;
            for (int a = 1; a < ni; a++) { /* sort */
                double v = inl[a]; int b = a - 1;
                while (b >= 0 && inl[b] > v) { inl[b + 1] = inl[b]; b--; }
                inl[b + 1] = v;
            }
            int run = 0, max_run = 0; /* longest run of separations <= max_sep */
            for (int k = 0; k + 1 < ni; k++) {
                if (fabs(inl[k + 1] - inl[k]) <= max_sep) { run++; if (run > max_run) max_run = run; }
                else run = 0;
            }
            if (max_run + 1 > best) best = max_run + 1;
        }
    return best;
}

/* make_line.py:140-152 */
static double score_make_line(OEnv *e) {
    double px[16], py[16];
    int n = 0;
    for (int i = 0; i < e->nents; i++) {
        OEntity *en = &e->ents[i];
        if (en->kind != ENT_BLOCK) continue;
        vec2 p = e->space.bodies[en->body0].p;
        px[n] = p.x; py[n] = p.y; n++;
    }
    const double rad = shape_rad();
    int line_len = o_longest_line(px, py, n, rad * 1.5, rad * 3.5);
    int min_len = n - 2 > 2 ? n - 2 : 2;
    int d = line_len - min_len;
    return (double)(d > 0 ? d : 0) / (double)(n - min_len);
}

/* norm of a 2-vector as np.linalg.norm computes it (sqrt of BLAS ddot) */
static double np_norm2(double x, double y) { return sqrt(fma(y, y, x * x)); }

/* pick_and_place.py:87-101 (every valid shape is scored with self.target_shape: one value) */
static double score_pick_and_place(OEnv *e) {
    vec2 p = e->space.bodies[e->ents[e->target_ent].body0].p;
    double dist = np_norm2(e->target_pos.x - p.x, e->target_pos.y - p.y);
    double succeed = shape_rad(), furthest = sqrt(2.0);
    double drange = furthest - succeed;
    double v = furthest - dist;
    double score = (v > 0.0 ? v : 0.0) / drange;
    return score < 1.0 ? score : 1.0;
}

/* debug_shaped_reward: move_to_corner.py:85-100, pick_and_place.py:114-124 */
double oscene_debug_reward(OEnv *e) {
    vec2 r = e->space.bodies[e->ents[e->robot].body0].p;
    if (e->task == TASK_PICK_AND_PLACE) {
        vec2 p = e->space.bodies[e->ents[e->target_ent].body0].p;
        double s2t = np_norm2(p.x - e->target_pos.x, p.y - e->target_pos.y);
        double r2s = np_norm2(r.x - p.x, r.y - p.y);
        double shaping = -s2t / 5 - (r2s > shape_rad() ? r2s : shape_rad()) / 10;
        return shaping + score_pick_and_place(e);
    }
    int shape = -1; /* MoveToCorner: the block */
    for (int i = 0; i < e->nents; i++) if (e->ents[i].kind == ENT_BLOCK) { shape = i; break; }
    vec2 p = e->space.bodies[e->ents[shape].body0].p;
    return o_shaped_move_to_corner(r.x, r.y, p.x, p.y);
}

/* move_to_corner.py:86-100 debug_shaped_reward on (robot, block) positions */
double o_shaped_move_to_corner(double rx, double ry, double sx, double sy) {
    double s2c = np_norm2(sx - 0.0, sy - 1.0);
    double r2s = np_norm2(rx - sx, ry - sy);
    double shaping = -s2c / 5 - (r2s > 0.2 ? r2s : 0.2) / 20;
    return shaping + o_score_move_to_corner(rx, ry);
}

double oscene_score(OEnv *e) {
    switch (e->task) {
    case TASK_MOVE_TO_REGION: return score_move_to_region(e);
    case TASK_MOVE_TO_CORNER: return score_move_to_corner(e);
    case TASK_CLUSTER_COLOUR: return score_cluster(e, 0);
    case TASK_CLUSTER_SHAPE: return score_cluster(e, 1);
    case TASK_MATCH_REGIONS: return score_match_regions(e);
    case TASK_MAKE_LINE: return score_make_line(e);
    case TASK_FIND_DUPE: return score_find_dupe(e);
    case TASK_FIX_COLOUR: return score_fix_colour(e);
    case TASK_PICK_AND_PLACE: return score_pick_and_place(e);
    }
    return 0.0;
}

/* ---------------- reference control-flow fixtures ------------------------
 * tests/golden/make_ref_fixtures.py executes the reference's OWN reset code (task on_reset, geom.py
 * pm_randomise_all_poses / pm_randomise_pose / pm_shift_bodies) over a stand-in pymunk Space whose
 * entities, poses, shape filters and shape queries are these: the entity builders and the collision test
 * of this oracle, driven in the order the reference code calls them.  TEST INFRASTRUCTURE ONLY. */
OEnv *osc_create(int task, int flags) {
    OEnv *e = (OEnv *)calloc(1, sizeof(OEnv));
    e->task = task; e->flags = flags; e->max_tries = 10000;
    e->robot = -1; e->goal = -1;
    ophys_init(&e->space);
    static const double PV_DEF[5] = {3, 1, 4, 1.5, 0.1};
    for (int i = 0; i < 5; i++) e->pv[i] = PV_DEF[i];  /* joint forces only: no effect on poses at reset */
    return e;
}
void osc_destroy(OEnv *e) { free(e); }
int osc_add_arena(OEnv *e) { add_arena(e); return e->nents - 1; }
int osc_add_goal(OEnv *e, double x, double y, double h, double w, int colour) {
    add_goal(e, x, y, h, w, colour); return e->nents - 1;
}
int osc_add_robot(OEnv *e, double x, double y, double angle) { add_robot(e, v2(x, y), angle); return e->nents - 1; }
int osc_add_block(OEnv *e, int type, int colour, double x, double y, double angle) {
    add_block(e, type, colour, v2(x, y), angle, 0); return e->nents - 1;
}
/* kind, body0, nbodies (goal: 1, its static body), shape0, nshapes */
void osc_entity(const OEnv *e, int ent, int out[5]) {
    const OEntity *en = &e->ents[ent];
    out[0] = en->kind; out[1] = en->body0; out[2] = en->kind == ENT_GOAL ? 1 : en->nbodies;
    out[3] = en->shape0; out[4] = en->nshapes;
}
/* pose of the k-th body of an entity (the goal's static body: its shape's static position, angle 0) */
void osc_get_pose(OEnv *e, int ent, int k, double out[3]) {
    const OEntity *en = &e->ents[ent];
    if (en->kind == ENT_GOAL) { vec2 p = e->space.shapes[en->shape0].sp; out[0] = p.x; out[1] = p.y; out[2] = 0.0; return; }
    const OBody *b = &e->space.bodies[en->body0 + k];
    out[0] = b->p.x; out[1] = b->p.y; out[2] = b->a;
}
/* pymunk Body.position / Body.angle setters (cpBodySetPosition / cpBodySetAngle) */
void osc_set_position(OEnv *e, int ent, int k, double x, double y) {
    const OEntity *en = &e->ents[ent];
    if (en->kind == ENT_GOAL) { e->space.shapes[en->shape0].sp = v2(x, y); return; }
    ophys_body_set_position(&e->space, en->body0 + k, v2(x, y));
}
void osc_set_angle(OEnv *e, int ent, int k, double a) {
    const OEntity *en = &e->ents[ent];
    if (en->kind == ENT_GOAL) return;   /* static goal body: rand_rot is always False for it */
    ophys_body_set_angle(&e->space, en->body0 + k, a);
}
/* Space.reindex_shapes_for_body of every body of the entity */
void osc_reindex(OEnv *e, int ent) { reindex_entity(e, &e->ents[ent]); }
void osc_get_filter(const OEnv *e, int sh, uint32_t out[3]) {
    const OShape *s = &e->space.shapes[sh];
    out[0] = s->group; out[1] = s->categories; out[2] = s->mask;
}
void osc_set_filter(OEnv *e, int sh, uint32_t group, uint32_t categories, uint32_t mask) {
    OShape *s = &e->space.shapes[sh];
    s->group = group; s->categories = categories; s->mask = mask;
}
/* Space.shape_query(shape): the shapes that collide with it (each once, in shape order) */
int osc_shape_query(OEnv *e, int sh, int *hits, int max) {
    int n = 0;
    uint8_t ign[O_MAX_SHAPES];
    memset(ign, 0, sizeof(ign));
    while (n < max && ophys_shape_query_any_ign(&e->space, sh, ign)) {
        /* find the first hit not yet reported: query with every earlier hit ignored */
        int found = -1;
        for (int j = 0; j < e->space.nshapes && found < 0; j++) {
            if (ign[j] || j == sh) continue;
            uint8_t only[O_MAX_SHAPES];
            for (int k = 0; k < e->space.nshapes; k++) only[k] = (k != j);
            if (ophys_shape_query_any_ign(&e->space, sh, only)) found = j;
        }
        if (found < 0) break;
        hits[n++] = found;
        ign[found] = 1;
    }
    return n;
}
/* the env's numpy-legacy MT19937 state (RandomState.get_state()[1:3]) */
void oenv_get_rng(const OEnv *e, uint32_t key[624], int *pos) {
    memcpy(key, e->rng.key, sizeof(e->rng.key));
    *pos = e->rng.pos;
}
/* body index of a shape (-1: a static body) */
int osc_shape_body(const OEnv *e, int sh) { return e->space.shapes[sh].body; }
