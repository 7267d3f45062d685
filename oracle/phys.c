/*
 * phys.c -- Chipmunk2D 7.0.x semantics (as bundled in pymunk 5.6), restated.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Reference call sites: base_env.py:206-208 (Space, collision_slop 0.01,
 * iterations 10), base_env.py:248-255 (10 x space.step(1/fps/10)),
 * entities.py:238-433 / 507-533 / 610-749 / 783-801 (bodies, shapes, joints),
 * geom.py:116-384 (shape_query rejection sampling).  Upstream semantics are
 * SURVEY.md Appendix A; the one deliberate deviation is the broadphase/arbiter
 * order (Chipmunk uses BBTree traversal order, history dependent): here pairs
 * are visited canonically -- for each dynamic shape i in add order: every static
 * shape in add order, then every dynamic shape j > i -- and GJK always starts
 * from the bounding-box-centre axis (collision id 0).
 */
#include <math.h>
#include <string.h>
#include <float.h>
#include "ophys.h"

/* ---------------- cpVect helpers (chipmunk_private.h / cpVect.h) -------- */
static inline vec2 v2(double x, double y) { vec2 r = {x, y}; return r; }
static inline vec2 vadd(vec2 a, vec2 b) { return v2(a.x + b.x, a.y + b.y); }
static inline vec2 vsub(vec2 a, vec2 b) { return v2(a.x - b.x, a.y - b.y); }
static inline vec2 vneg(vec2 a) { return v2(-a.x, -a.y); }
static inline vec2 vmult(vec2 a, double s) { return v2(a.x * s, a.y * s); }
static inline double vdot(vec2 a, vec2 b) { return a.x * b.x + a.y * b.y; }
static inline double vcross(vec2 a, vec2 b) { return a.x * b.y - a.y * b.x; }
static inline vec2 vperp(vec2 a) { return v2(-a.y, a.x); }
static inline vec2 vrperp(vec2 a) { return v2(a.y, -a.x); }
static inline vec2 vrotate(vec2 a, vec2 b) { return v2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
static inline double vlengthsq(vec2 a) { return vdot(a, a); }
static inline double vlength(vec2 a) { return sqrt(vdot(a, a)); }
static inline vec2 vnormalize(vec2 a) { return vmult(a, 1.0 / (vlength(a) + DBL_MIN)); }
static inline vec2 vlerp(vec2 a, vec2 b, double t) { return vadd(vmult(a, 1.0 - t), vmult(b, t)); }
static inline int veql(vec2 a, vec2 b) { return a.x == b.x && a.y == b.y; }
static inline vec2 vclamp(vec2 v, double len) {
    return (vdot(v, v) > len * len) ? vmult(vnormalize(v), len) : v;
}
static inline double fmax_cp(double a, double b) { return (a > b) ? a : b; }
static inline double fmin_cp(double a, double b) { return (a < b) ? a : b; }
static inline double fclamp(double f, double mn, double mx) { return fmin_cp(fmax_cp(f, mn), mx); }
static inline double fclamp01(double f) { return fmax_cp(0.0, fmin_cp(f, 1.0)); }

#define HASH_COEF 3344921057ull
#define HASH_PAIR(A, B) (((uint64_t)(A) * HASH_COEF) ^ ((uint64_t)(B) * HASH_COEF))

/* body transform: {a=c, b=s, c=-s, d=c, tx=p.x, ty=p.y} (cog = 0) */
static inline vec2 xform_point(double c, double s, vec2 p, vec2 v) {
    return v2(c * v.x + (-s) * v.y + p.x, s * v.x + c * v.y + p.y);
}
static inline vec2 xform_vect(double c, double s, vec2 v) {
    return v2(c * v.x + (-s) * v.y, s * v.x + c * v.y);
}

/* ---------------- bodies ------------------------------------------------ */
void ophys_init(OSpace *s) {
    memset(s, 0, sizeof(*s));
    s->collision_slop = 0.01;                 /* base_env.py:207 */
    s->collision_bias = pow(1.0 - 0.1, 60.0); /* cpSpaceInit default */
    s->iterations = 10;                       /* base_env.py:208 */
}

static void body_set_transform(OBody *b) {
    b->rc = o_crcos(b->a);
    b->rs = o_crsin(b->a);
}

int ophys_add_body(OSpace *s, int type, double m, double i, vec2 p, double a) {
    if (s->nbodies >= O_MAX_BODIES) { s->overflow = 1; return -1; }
    OBody *b = &s->bodies[s->nbodies];
    memset(b, 0, sizeof(*b));
    b->type = type;
    if (type == BODY_DYNAMIC) {
        b->m = m; b->m_inv = 1.0 / m;
        b->i = i; b->i_inv = 1.0 / i;
    } else {
        b->m = b->i = INFINITY;
        b->m_inv = b->i_inv = 0.0;
    }
    b->p = p;
    b->a = a;
    body_set_transform(b);
    return s->nbodies++;
}

void ophys_body_set_angle(OSpace *s, int bi, double a) {
    OBody *b = &s->bodies[bi];
    b->a = a;
    body_set_transform(b);
}

void ophys_body_set_position(OSpace *s, int bi, vec2 p) {
    /* cpBodySetPosition: p = T(cog) + position, cog = 0 */
    OBody *b = &s->bodies[bi];
    b->p = vadd(xform_vect(b->rc, b->rs, v2(0.0, 0.0)), p);
}

/* ---------------- shapes ------------------------------------------------ */
static OShape *new_shape(OSpace *s, int type, int body) {
    if (s->nshapes >= O_MAX_SHAPES) { s->overflow = 1; return NULL; }
    OShape *sh = &s->shapes[s->nshapes];
    memset(sh, 0, sizeof(*sh));
    sh->type = type;
    sh->body = body;
    sh->categories = 0xffffffffu;
    sh->mask = 0xffffffffu;
    sh->hashid = (uint64_t)s->nshapes; /* cpSpace shapeIDCounter: one per added shape */
    sh->entity = -1;
    return sh;
}

static void shape_xform(const OSpace *s, const OShape *sh, double *c, double *sn, vec2 *p) {
    if (sh->body >= 0) {
        const OBody *b = &s->bodies[sh->body];
        *c = b->rc; *sn = b->rs; *p = b->p;
    } else {
        *c = 1.0; *sn = 0.0; *p = sh->sp;
    }
}

void ophys_shape_update(OSpace *s, int si) {
    OShape *sh = &s->shapes[si];
    double c, sn; vec2 p;
    shape_xform(s, sh, &c, &sn, &p);
    if (sh->type == SH_CIRCLE) {
        sh->tc = xform_point(c, sn, p, sh->c);
        sh->bb_l = sh->tc.x - sh->r; sh->bb_b = sh->tc.y - sh->r;
        sh->bb_r = sh->tc.x + sh->r; sh->bb_t = sh->tc.y + sh->r;
    } else if (sh->type == SH_SEGMENT) {
        sh->ta = xform_point(c, sn, p, sh->a);
        sh->tb = xform_point(c, sn, p, sh->b);
        sh->tn = xform_vect(c, sn, sh->n);
        double l, r, b, t;
        if (sh->ta.x < sh->tb.x) { l = sh->ta.x; r = sh->tb.x; } else { l = sh->tb.x; r = sh->ta.x; }
        if (sh->ta.y < sh->tb.y) { b = sh->ta.y; t = sh->tb.y; } else { b = sh->tb.y; t = sh->ta.y; }
        sh->bb_l = l - sh->r; sh->bb_b = b - sh->r; sh->bb_r = r + sh->r; sh->bb_t = t + sh->r;
    } else {
        double l = INFINITY, r = -INFINITY, b = INFINITY, t = -INFINITY;
        for (int i = 0; i < sh->count; i++) {
            vec2 v = xform_point(c, sn, p, sh->v[i]);
            vec2 n = xform_vect(c, sn, sh->pn[i]);
            sh->tv[i] = v; sh->tpn[i] = n;
            l = fmin_cp(l, v.x); r = fmax_cp(r, v.x);
            b = fmin_cp(b, v.y); t = fmax_cp(t, v.y);
        }
        sh->bb_l = l - sh->r; sh->bb_b = b - sh->r; sh->bb_r = r + sh->r; sh->bb_t = t + sh->r;
    }
}

int ophys_add_circle(OSpace *s, int body, double r, vec2 offset) {
    OShape *sh = new_shape(s, SH_CIRCLE, body);
    if (!sh) return -1;
    sh->c = offset; sh->r = r;
    ophys_shape_update(s, s->nshapes);
    return s->nshapes++;
}

int ophys_add_segment(OSpace *s, vec2 a, vec2 b, double r) {
    /* static arena body (never positioned): identity transform */
    OShape *sh = new_shape(s, SH_SEGMENT, -1);
    if (!sh) return -1;
    sh->a = a; sh->b = b; sh->r = r;
    sh->n = vrperp(vnormalize(vsub(b, a)));
    sh->sp = v2(0.0, 0.0);
    ophys_shape_update(s, s->nshapes);
    return s->nshapes++;
}

/* cpLoopIndexes + QuickHull (cpPolyline.c / chipmunk.c cpConvexHull) */
static void loop_indexes(const vec2 *verts, int count, int *start, int *end) {
    *start = *end = 0;
    vec2 mn = verts[0], mx = mn;
    for (int i = 1; i < count; i++) {
        vec2 v = verts[i];
        if (v.x < mn.x || (v.x == mn.x && v.y < mn.y)) { mn = v; *start = i; }
        else if (v.x > mx.x || (v.x == mx.x && v.y > mx.y)) { mx = v; *end = i; }
    }
}
#define SWAPV(a, b) do { vec2 _t = (a); (a) = (b); (b) = _t; } while (0)
static int qhull_partition(vec2 *verts, int count, vec2 a, vec2 b, double tol) {
    if (count == 0) return 0;
    double mx = 0; int pivot = 0;
    vec2 delta = vsub(b, a);
    double valueTol = tol * vlength(delta);
    int head = 0;
    for (int tail = count - 1; head <= tail;) {
        double value = vcross(vsub(verts[head], a), delta);
        if (value > valueTol) {
            if (value > mx) { mx = value; pivot = head; }
            head++;
        } else {
            SWAPV(verts[head], verts[tail]);
            tail--;
        }
    }
    if (pivot != 0) SWAPV(verts[0], verts[pivot]);
    return head;
}
static int qhull_reduce(double tol, vec2 *verts, int count, vec2 a, vec2 pivot, vec2 b, vec2 *result) {
    if (count < 0) return 0;
    if (count == 0) { result[0] = pivot; return 1; }
    int left_count = qhull_partition(verts, count, a, pivot, tol);
    int index = qhull_reduce(tol, verts + 1, left_count - 1, a, verts[0], pivot, result);
    result[index++] = pivot;
    int right_count = qhull_partition(verts + left_count, count - left_count, pivot, b, tol);
    return index + qhull_reduce(tol, verts + left_count + 1, right_count - 1, pivot, verts[left_count], b, result + index);
}
int o_convex_hull(int count, const vec2 *verts, vec2 *result, int *first, double tol) {
    if (verts != result) memcpy(result, verts, (size_t)count * sizeof(vec2));
    int start, end;
    loop_indexes(verts, count, &start, &end);
    if (start == end) { if (first) *first = 0; return 1; }
    SWAPV(result[0], result[start]);
    SWAPV(result[1], result[end == 0 ? start : end]);
    vec2 a = result[0], b = result[1];
    if (first) *first = start;
    return qhull_reduce(tol, result + 2, count - 2, a, b, a, result + 1) + 1;
}

static void poly_set_verts(OShape *sh, int count, const vec2 *verts) {
    sh->count = count;
    for (int i = 0; i < count; i++) {
        vec2 a = verts[(i - 1 + count) % count], b = verts[i];
        sh->v[i] = b;
        sh->pn[i] = vnormalize(vrperp(vsub(b, a)));
    }
}

int ophys_add_poly(OSpace *s, int body, int count, const vec2 *verts, double r, int raw) {
    OShape *sh = new_shape(s, SH_POLY, body);
    if (!sh) return -1;
    vec2 hull[O_MAX_VERTS * 2];
    int n = count;
    if (raw) {
        memcpy(hull, verts, (size_t)count * sizeof(vec2));
    } else {
        /* cpPolyShapeInit: transform by identity {1,0,0,1,0,0} then hull */
        for (int i = 0; i < count; i++)
            hull[i] = v2(1.0 * verts[i].x + 0.0 * verts[i].y + 0.0, 0.0 * verts[i].x + 1.0 * verts[i].y + 0.0);
        n = o_convex_hull(count, hull, hull, NULL, 0.0);
    }
    if (n > O_MAX_VERTS) { s->overflow = 1; n = O_MAX_VERTS; }
    poly_set_verts(sh, n, hull);
    sh->r = r;
    ophys_shape_update(s, s->nshapes);
    return s->nshapes++;
}

int ophys_add_static_box(OSpace *s, vec2 pos, double w, double h) {
    /* cpBoxShapeNew(static body at pos, w, h, 0): raw verts (r,b),(r,t),(l,t),(l,b) */
    double hw = w / 2.0, hh = h / 2.0;
    vec2 verts[4] = {v2(hw, -hh), v2(hw, hh), v2(-hw, hh), v2(-hw, -hh)};
    OShape *sh = new_shape(s, SH_POLY, -1);
    if (!sh) return -1;
    poly_set_verts(sh, 4, verts);
    sh->r = 0.0;
    sh->sp = pos;
    ophys_shape_update(s, s->nshapes);
    return s->nshapes++;
}

/* ---------------- constraints ------------------------------------------- */
static OCons *new_cons(OSpace *s, int type, int a, int b) {
    if (s->ncons >= O_MAX_CONS) { s->overflow = 1; return NULL; }
    OCons *c = &s->cons[s->ncons];
    memset(c, 0, sizeof(*c));
    c->type = type; c->a = a; c->b = b;
    c->maxForce = INFINITY;
    c->maxBias = INFINITY;
    c->errorBias = pow(1.0 - 0.1, 60.0);
    return c;
}

static void body_xf(const OSpace *s, int bi, double *c, double *sn, vec2 *p) {
    if (bi >= 0) { *c = s->bodies[bi].rc; *sn = s->bodies[bi].rs; *p = s->bodies[bi].p; }
    else { *c = 1.0; *sn = 0.0; *p = v2(0.0, 0.0); }
}

int ophys_add_pivot2(OSpace *s, int a, int b, vec2 anchorA, vec2 anchorB) {
    OCons *c = new_cons(s, C_PIVOT, a, b);
    if (!c) return -1;
    c->anchorA = anchorA; c->anchorB = anchorB;
    return s->ncons++;
}

/* cpBodyWorldToLocal via cpTransformRigidInverse */
static vec2 world_to_local(const OSpace *s, int bi, vec2 pt) {
    double c, sn; vec2 p;
    body_xf(s, bi, &c, &sn, &p);
    double ta = c, tb = sn, tc = -sn, td = c, tx = p.x, ty = p.y;
    double ia = td, ic = -tc, itx = tc * ty - tx * td;
    double ib = -tb, id = ta, ity = tx * tb - ta * ty;
    return v2(ia * pt.x + ic * pt.y + itx, ib * pt.x + id * pt.y + ity);
}

int ophys_add_pivot1(OSpace *s, int a, int b, vec2 pivot) {
    vec2 aa = world_to_local(s, a, pivot), bb = world_to_local(s, b, pivot);
    return ophys_add_pivot2(s, a, b, aa, bb);
}

int ophys_add_gear(OSpace *s, int a, int b, double phase, double ratio) {
    OCons *c = new_cons(s, C_GEAR, a, b);
    if (!c) return -1;
    c->phase = phase; c->ratio = ratio; c->ratio_inv = 1.0 / ratio;
    return s->ncons++;
}

int ophys_add_rotlimit(OSpace *s, int a, int b, double mn, double mx) {
    OCons *c = new_cons(s, C_ROTLIMIT, a, b);
    if (!c) return -1;
    c->min = mn; c->max = mx;
    return s->ncons++;
}

int ophys_add_motor(OSpace *s, int a, int b, double rate) {
    OCons *c = new_cons(s, C_MOTOR, a, b);
    if (!c) return -1;
    c->rate = rate;
    return s->ncons++;
}

int ophys_add_spring(OSpace *s, int a, int b, double rest, double k, double damp) {
    OCons *c = new_cons(s, C_SPRING, a, b);
    if (!c) return -1;
    c->restAngle = rest; c->stiffness = k; c->damping = damp;
    return s->ncons++;
}

/* static body pseudo-state: m_inv = i_inv = 0, v = w = 0 */
typedef struct { vec2 *v, *vb; double *w, *wb; double m_inv, i_inv; vec2 p; double a; } BRef;
static vec2 g_zero_v, g_zero_vb;
static double g_zero_w, g_zero_wb;
static BRef bref(OSpace *s, int bi) {
    BRef r;
    if (bi >= 0) {
        OBody *b = &s->bodies[bi];
        r.v = &b->v; r.vb = &b->v_bias; r.w = &b->w; r.wb = &b->w_bias;
        r.m_inv = b->m_inv; r.i_inv = b->i_inv; r.p = b->p; r.a = b->a;
    } else {
        g_zero_v = v2(0, 0); g_zero_vb = v2(0, 0); g_zero_w = 0; g_zero_wb = 0;
        r.v = &g_zero_v; r.vb = &g_zero_vb; r.w = &g_zero_w; r.wb = &g_zero_wb;
        r.m_inv = 0.0; r.i_inv = 0.0; r.p = v2(0, 0); r.a = 0.0;
    }
    return r;
}

static inline void apply_impulse(BRef *b, vec2 j, vec2 r) {
    *b->v = vadd(*b->v, vmult(j, b->m_inv));
    *b->w += b->i_inv * vcross(r, j);
}
static inline void apply_impulses(BRef *a, BRef *b, vec2 r1, vec2 r2, vec2 j) {
    apply_impulse(a, vneg(j), r1);
    apply_impulse(b, j, r2);
}
static inline void apply_bias_impulse(BRef *b, vec2 j, vec2 r) {
    *b->vb = vadd(*b->vb, vmult(j, b->m_inv));
    *b->wb += b->i_inv * vcross(r, j);
}
static inline void apply_bias_impulses(BRef *a, BRef *b, vec2 r1, vec2 r2, vec2 j) {
    apply_bias_impulse(a, vneg(j), r1);
    apply_bias_impulse(b, j, r2);
}
static inline vec2 relative_velocity(BRef *a, BRef *b, vec2 r1, vec2 r2) {
    vec2 v1 = vadd(*a->v, vmult(vperp(r1), *a->w));
    vec2 v2_ = vadd(*b->v, vmult(vperp(r2), *b->w));
    return vsub(v2_, v1);
}
static inline double k_scalar_body(const BRef *b, vec2 r, vec2 n) {
    double rcn = vcross(r, n);
    return b->m_inv + b->i_inv * rcn * rcn;
}
static inline double k_scalar(const BRef *a, const BRef *b, vec2 r1, vec2 r2, vec2 n) {
    return k_scalar_body(a, r1, n) + k_scalar_body(b, r2, n);
}
static inline double bias_coef(double errorBias, double dt) { return 1.0 - pow(errorBias, dt); }

static void cons_prestep(OSpace *s, OCons *c, double dt) {
    BRef a = bref(s, c->a), b = bref(s, c->b);
    switch (c->type) {
    case C_PIVOT: {
        double ac, as, bc, bs; vec2 ap, bp;
        body_xf(s, c->a, &ac, &as, &ap);
        body_xf(s, c->b, &bc, &bs, &bp);
        c->r1 = xform_vect(ac, as, vsub(c->anchorA, v2(0.0, 0.0)));
        c->r2 = xform_vect(bc, bs, vsub(c->anchorB, v2(0.0, 0.0)));
        /* k_tensor */
        double m_sum = a.m_inv + b.m_inv;
        double k11 = m_sum, k12 = 0.0, k21 = 0.0, k22 = m_sum;
        double r1xsq = c->r1.x * c->r1.x * a.i_inv;
        double r1ysq = c->r1.y * c->r1.y * a.i_inv;
        double r1nxy = -c->r1.x * c->r1.y * a.i_inv;
        k11 += r1ysq; k12 += r1nxy; k21 += r1nxy; k22 += r1xsq;
        double r2xsq = c->r2.x * c->r2.x * b.i_inv;
        double r2ysq = c->r2.y * c->r2.y * b.i_inv;
        double r2nxy = -c->r2.x * c->r2.y * b.i_inv;
        k11 += r2ysq; k12 += r2nxy; k21 += r2nxy; k22 += r2xsq;
        double det = k11 * k22 - k12 * k21;
        double det_inv = 1.0 / det;
        c->k11 = k22 * det_inv; c->k12 = -k12 * det_inv;
        c->k21 = -k21 * det_inv; c->k22 = k11 * det_inv;
        vec2 delta = vsub(vadd(b.p, c->r2), vadd(a.p, c->r1));
        c->biasv = vclamp(vmult(delta, -bias_coef(c->errorBias, dt) / dt), c->maxBias);
        break;
    }
    case C_GEAR: {
        c->iSum = 1.0 / (a.i_inv * c->ratio_inv + c->ratio * b.i_inv);
        double maxBias = c->maxBias;
        c->bias = fclamp(-bias_coef(c->errorBias, dt) * (b.a * c->ratio - a.a - c->phase) / dt, -maxBias, maxBias);
        break;
    }
    case C_ROTLIMIT: {
        double dist = b.a - a.a, pdist = 0.0;
        if (dist > c->max) pdist = c->max - dist;
        else if (dist < c->min) pdist = c->min - dist;
        c->iSum = 1.0 / (a.i_inv + b.i_inv);
        double maxBias = c->maxBias;
        c->bias = fclamp(-bias_coef(c->errorBias, dt) * pdist / dt, -maxBias, maxBias);
        if (!c->bias) c->jAcc = 0.0;
        break;
    }
    case C_MOTOR:
        c->iSum = 1.0 / (a.i_inv + b.i_inv);
        break;
    case C_SPRING: {
        double moment = a.i_inv + b.i_inv;
        c->iSum = 1.0 / moment;
        c->w_coef = 1.0 - exp(-c->damping * dt * moment);
        c->target_wrn = 0.0;
        double j_spring = ((a.a - b.a) - c->restAngle) * c->stiffness * dt;
        c->jAcc = j_spring;
        *a.w -= j_spring * a.i_inv;
        *b.w += j_spring * b.i_inv;
        break;
    }
    }
}

static void cons_apply_cached(OSpace *s, OCons *c, double dt_coef) {
    BRef a = bref(s, c->a), b = bref(s, c->b);
    switch (c->type) {
    case C_PIVOT:
        apply_impulses(&a, &b, c->r1, c->r2, vmult(c->jAccv, dt_coef));
        break;
    case C_GEAR: {
        double j = c->jAcc * dt_coef;
        *a.w -= j * a.i_inv * c->ratio_inv;
        *b.w += j * b.i_inv;
        break;
    }
    case C_ROTLIMIT:
    case C_MOTOR: {
        double j = c->jAcc * dt_coef;
        *a.w -= j * a.i_inv;
        *b.w += j * b.i_inv;
        break;
    }
    case C_SPRING:
        break;
    }
}

static void cons_apply(OSpace *s, OCons *c, double dt) {
    BRef a = bref(s, c->a), b = bref(s, c->b);
    switch (c->type) {
    case C_PIVOT: {
        vec2 r1 = c->r1, r2 = c->r2;
        vec2 vr = relative_velocity(&a, &b, r1, r2);
        vec2 d = vsub(c->biasv, vr);
        vec2 j = v2(d.x * c->k11 + d.y * c->k12, d.x * c->k21 + d.y * c->k22);
        vec2 jOld = c->jAccv;
        c->jAccv = vclamp(vadd(c->jAccv, j), c->maxForce * dt);
        j = vsub(c->jAccv, jOld);
        apply_impulses(&a, &b, c->r1, c->r2, j);
        break;
    }
    case C_GEAR: {
        double wr = *b.w * c->ratio - *a.w;
        double jMax = c->maxForce * dt;
        double j = (c->bias - wr) * c->iSum;
        double jOld = c->jAcc;
        c->jAcc = fclamp(jOld + j, -jMax, jMax);
        j = c->jAcc - jOld;
        *a.w -= j * a.i_inv * c->ratio_inv;
        *b.w += j * b.i_inv;
        break;
    }
    case C_ROTLIMIT: {
        if (!c->bias) return;
        double wr = *b.w - *a.w;
        double jMax = c->maxForce * dt;
        double j = -(c->bias + wr) * c->iSum;
        double jOld = c->jAcc;
        if (c->bias < 0.0) c->jAcc = fclamp(jOld + j, 0.0, jMax);
        else c->jAcc = fclamp(jOld + j, -jMax, 0.0);
        j = c->jAcc - jOld;
        *a.w -= j * a.i_inv;
        *b.w += j * b.i_inv;
        break;
    }
    case C_MOTOR: {
        double wr = *b.w - *a.w + c->rate;
        double jMax = c->maxForce * dt;
        double j = -wr * c->iSum;
        double jOld = c->jAcc;
        c->jAcc = fclamp(jOld + j, -jMax, jMax);
        j = c->jAcc - jOld;
        *a.w -= j * a.i_inv;
        *b.w += j * b.i_inv;
        break;
    }
    case C_SPRING: {
        double wrn = *a.w - *b.w;
        double w_damp = (c->target_wrn - wrn) * c->w_coef;
        c->target_wrn = wrn + w_damp;
        double j_damp = w_damp * c->iSum;
        c->jAcc += j_damp;
        *a.w += j_damp * a.i_inv;
        *b.w -= j_damp * b.i_inv;
        break;
    }
    }
}

/* ---------------- narrowphase (cpCollision.c) --------------------------- */
typedef struct { vec2 p; int index; } SupportPoint;
typedef struct { vec2 a, b, ab; uint32_t id; } MinkowskiPoint;
typedef struct { const OShape *s1, *s2; } SupportCtx;

static int poly_support_index(const OShape *sh, vec2 n) {
    double mx = -INFINITY; int index = 0;
    for (int i = 0; i < sh->count; i++) {
        double d = vdot(sh->tv[i], n);
        if (d > mx) { mx = d; index = i; }
    }
    return index;
}
static SupportPoint support_point(const OShape *sh, vec2 n) {
    SupportPoint sp;
    if (sh->type == SH_CIRCLE) { sp.p = sh->tc; sp.index = 0; }
    else if (sh->type == SH_SEGMENT) {
        if (vdot(sh->ta, n) > vdot(sh->tb, n)) { sp.p = sh->ta; sp.index = 0; }
        else { sp.p = sh->tb; sp.index = 1; }
    } else {
        int i = poly_support_index(sh, n);
        sp.p = sh->tv[i]; sp.index = i;
    }
    return sp;
}
static MinkowskiPoint mink_new(SupportPoint a, SupportPoint b) {
    MinkowskiPoint m = {a.p, b.p, vsub(b.p, a.p), ((uint32_t)(a.index & 0xFF) << 8) | (uint32_t)(b.index & 0xFF)};
    return m;
}
static MinkowskiPoint support(const SupportCtx *ctx, vec2 n) {
    SupportPoint a = support_point(ctx->s1, vneg(n));
    SupportPoint b = support_point(ctx->s2, n);
    return mink_new(a, b);
}
static inline double closest_t(vec2 a, vec2 b) {
    vec2 delta = vsub(b, a);
    return -fclamp(vdot(delta, vadd(a, b)) / vlengthsq(delta), -1.0, 1.0);
}
static inline vec2 lerp_t(vec2 a, vec2 b, double t) {
    double ht = 0.5 * t;
    return vadd(vmult(a, 0.5 - ht), vmult(b, 0.5 + ht));
}
static inline double closest_dist(vec2 v0, vec2 v1) { return vlengthsq(lerp_t(v0, v1, closest_t(v0, v1))); }
static inline int check_area(vec2 v1, vec2 v2_) { return (v1.x * v2_.y) > (v1.y * v2_.x); }

static OClosest closest_points_new(MinkowskiPoint v0, MinkowskiPoint v1) {
    double t = closest_t(v0.ab, v1.ab);
    vec2 p = lerp_t(v0.ab, v1.ab, t);
    vec2 pa = lerp_t(v0.a, v1.a, t);
    vec2 pb = lerp_t(v0.b, v1.b, t);
    vec2 delta = vsub(v1.ab, v0.ab);
    vec2 n = vnormalize(vrperp(delta));
    double d = vdot(n, p);
    OClosest r;
    if (d <= 0.0 || (-1.0 < t && t < 1.0)) {
        r.a = pa; r.b = pb; r.n = n; r.d = d;
    } else {
        double d2 = vlength(p);
        vec2 n2 = vmult(p, 1.0 / (d2 + DBL_MIN));
        r.a = pa; r.b = pb; r.n = n2; r.d = d2;
    }
    return r;
}

#define MAX_GJK_ITERATIONS 30
#define MAX_EPA_ITERATIONS 30

/* number of EPA runs so far (the known-answer tests check which path a configuration takes) */
long ophys_epa_runs = 0;

static OClosest epa(const SupportCtx *ctx, MinkowskiPoint v0, MinkowskiPoint v1, MinkowskiPoint v2_) {
    MinkowskiPoint hull[64], hull2[64];
    int count = 3;
    ophys_epa_runs++;
    hull[0] = v0; hull[1] = v1; hull[2] = v2_;
    for (int iteration = 1;; iteration++) {
        int mini = 0;
        double minDist = INFINITY;
        for (int j = 0, i = count - 1; j < count; i = j, j++) {
            double d = closest_dist(hull[i].ab, hull[j].ab);
            if (d < minDist) { minDist = d; mini = i; }
        }
        MinkowskiPoint w0 = hull[mini];
        MinkowskiPoint w1 = hull[(mini + 1) % count];
        MinkowskiPoint p = support(ctx, vperp(vsub(w1.ab, w0.ab)));
        int duplicate = (p.id == w0.id || p.id == w1.id);
        if (!duplicate && check_area(w1.ab, p.ab) && iteration < MAX_EPA_ITERATIONS && count < 63) {
            int count2 = 1;
            hull2[0] = p;
            for (int i = 0; i < count; i++) {
                int index = (mini + 1 + i) % count;
                vec2 h0 = hull2[count2 - 1].ab;
                vec2 h1 = hull[index].ab;
                vec2 h2 = (i + 1 < count ? hull[(index + 1) % count] : p).ab;
                if (check_area(vsub(h2, h0), vadd(vsub(h1, h0), vsub(h1, h2)))) {
                    hull2[count2] = hull[index];
                    count2++;
                }
            }
            memcpy(hull, hull2, (size_t)count2 * sizeof(MinkowskiPoint));
            count = count2;
        } else {
            return closest_points_new(w0, w1);
        }
    }
}

static OClosest gjk_recurse(const SupportCtx *ctx, MinkowskiPoint v0, MinkowskiPoint v1, int iteration) {
    for (;;) {
        if (iteration > MAX_GJK_ITERATIONS) return closest_points_new(v0, v1);
        if (vcross(v1.ab, v0.ab) > 0.0) {
            MinkowskiPoint t = v0; v0 = v1; v1 = t;
            continue;
        }
        double t = closest_t(v0.ab, v1.ab);
        vec2 n = (-1.0 < t && t < 1.0 ? vperp(vsub(v1.ab, v0.ab)) : vneg(lerp_t(v0.ab, v1.ab, t)));
        MinkowskiPoint p = support(ctx, n);
        if (vcross(vsub(v1.ab, p.ab), vadd(v1.ab, p.ab)) > 0.0 &&
            vcross(vsub(v0.ab, p.ab), vadd(v0.ab, p.ab)) < 0.0) {
            return epa(ctx, v0, p, v1);
        }
        if (vdot(p.ab, n) <= fmax_cp(vdot(v0.ab, n), vdot(v1.ab, n))) {
            return closest_points_new(v0, v1);
        }
        if (closest_dist(v0.ab, p.ab) < closest_dist(p.ab, v1.ab)) { v1 = p; }
        else { v0 = p; }
        iteration++;
    }
}

static inline vec2 bb_center(const OShape *s) {
    return vlerp(v2(s->bb_l, s->bb_b), v2(s->bb_r, s->bb_t), 0.5);
}

static OClosest gjk(const SupportCtx *ctx) {
    vec2 axis = vperp(vsub(bb_center(ctx->s1), bb_center(ctx->s2)));
    MinkowskiPoint v0 = support(ctx, axis);
    MinkowskiPoint v1 = support(ctx, vneg(axis));
    return gjk_recurse(ctx, v0, v1, 1);
}

typedef struct { vec2 ap, bp; uint64_t ah, bh; double r; vec2 n; } Edge;

static Edge support_edge_poly(const OShape *sh, vec2 n) {
    int count = sh->count;
    int i1 = poly_support_index(sh, n);
    int i0 = (i1 - 1 + count) % count;
    int i2 = (i1 + 1) % count;
    uint64_t hid = sh->hashid;
    Edge e;
    if (vdot(n, sh->tpn[i1]) > vdot(n, sh->tpn[i2])) {
        e.ap = sh->tv[i0]; e.ah = HASH_PAIR(hid, i0);
        e.bp = sh->tv[i1]; e.bh = HASH_PAIR(hid, i1);
        e.r = sh->r; e.n = sh->tpn[i1];
    } else {
        e.ap = sh->tv[i1]; e.ah = HASH_PAIR(hid, i1);
        e.bp = sh->tv[i2]; e.bh = HASH_PAIR(hid, i2);
        e.r = sh->r; e.n = sh->tpn[i2];
    }
    return e;
}
static Edge support_edge_segment(const OShape *sh, vec2 n) {
    uint64_t hid = sh->hashid;
    Edge e;
    if (vdot(sh->tn, n) > 0.0) {
        e.ap = sh->ta; e.ah = HASH_PAIR(hid, 0); e.bp = sh->tb; e.bh = HASH_PAIR(hid, 1);
        e.r = sh->r; e.n = sh->tn;
    } else {
        e.ap = sh->tb; e.ah = HASH_PAIR(hid, 1); e.bp = sh->ta; e.bh = HASH_PAIR(hid, 0);
        e.r = sh->r; e.n = vneg(sh->tn);
    }
    return e;
}

static void push_contact(OCollision *info, vec2 p1, vec2 p2, uint64_t hash) {
    if (info->count >= 2) return;
    info->p1[info->count] = p1; info->p2[info->count] = p2; info->hash[info->count] = hash;
    info->count++;
}

static void contact_points(Edge e1, Edge e2, OClosest points, OCollision *info) {
    double mindist = e1.r + e2.r;
    if (points.d <= mindist) {
        vec2 n = info->n = points.n;
        double d_e1_a = vcross(e1.ap, n), d_e1_b = vcross(e1.bp, n);
        double d_e2_a = vcross(e2.ap, n), d_e2_b = vcross(e2.bp, n);
        double e1_denom = 1.0 / (d_e1_b - d_e1_a + DBL_MIN);
        double e2_denom = 1.0 / (d_e2_b - d_e2_a + DBL_MIN);
        {
            vec2 p1 = vadd(vmult(n, e1.r), vlerp(e1.ap, e1.bp, fclamp01((d_e2_b - d_e1_a) * e1_denom)));
            vec2 p2 = vadd(vmult(n, -e2.r), vlerp(e2.ap, e2.bp, fclamp01((d_e1_a - d_e2_a) * e2_denom)));
            double dist = vdot(vsub(p2, p1), n);
            if (dist <= 0.0) push_contact(info, p1, p2, HASH_PAIR(e1.ah, e2.bh));
        }
        {
            vec2 p1 = vadd(vmult(n, e1.r), vlerp(e1.ap, e1.bp, fclamp01((d_e2_a - d_e1_a) * e1_denom)));
            vec2 p2 = vadd(vmult(n, -e2.r), vlerp(e2.ap, e2.bp, fclamp01((d_e1_b - d_e2_a) * e2_denom)));
            double dist = vdot(vsub(p2, p1), n);
            if (dist <= 0.0) push_contact(info, p1, p2, HASH_PAIR(e1.bh, e2.ah));
        }
    }
}

static void circle_to_circle(const OShape *c1, const OShape *c2, OCollision *info) {
    double mindist = c1->r + c2->r;
    vec2 delta = vsub(c2->tc, c1->tc);
    double distsq = vlengthsq(delta);
    if (distsq < mindist * mindist) {
        double dist = sqrt(distsq);
        vec2 n = info->n = (dist ? vmult(delta, 1.0 / dist) : v2(1.0, 0.0));
        push_contact(info, vadd(c1->tc, vmult(n, c1->r)), vadd(c2->tc, vmult(n, -c2->r)), 0);
    }
}

static void circle_to_segment(const OShape *circle, const OShape *seg, OCollision *info) {
    vec2 seg_a = seg->ta, seg_b = seg->tb, center = circle->tc;
    vec2 seg_delta = vsub(seg_b, seg_a);
    double closest_t_ = fclamp01(vdot(seg_delta, vsub(center, seg_a)) / vlengthsq(seg_delta));
    vec2 closest = vadd(seg_a, vmult(seg_delta, closest_t_));
    double mindist = circle->r + seg->r;
    vec2 delta = vsub(closest, center);
    double distsq = vlengthsq(delta);
    if (distsq < mindist * mindist) {
        double dist = sqrt(distsq);
        vec2 n = info->n = (dist ? vmult(delta, 1.0 / dist) : seg->tn);
        /* endcap tangents are zero: rejection test always passes */
        push_contact(info, vadd(center, vmult(n, circle->r)), vadd(closest, vmult(n, -seg->r)), 0);
    }
}

static void segment_to_poly(const OShape *seg, const OShape *poly, OCollision *info) {
    SupportCtx ctx = {seg, poly};
    OClosest points = gjk(&ctx);
    vec2 n = points.n;
    (void)n;
    if (points.d - seg->r - poly->r <= 0.0) {
        contact_points(support_edge_segment(seg, n), support_edge_poly(poly, vneg(n)), points, info);
    }
}

static void circle_to_poly(const OShape *circle, const OShape *poly, OCollision *info) {
    SupportCtx ctx = {circle, poly};
    OClosest points = gjk(&ctx);
    if (points.d <= circle->r + poly->r) {
        vec2 n = info->n = points.n;
        push_contact(info, vadd(points.a, vmult(n, circle->r)), vadd(points.b, vmult(n, -poly->r)), 0);
    }
}

static void poly_to_poly(const OShape *p1, const OShape *p2, OCollision *info) {
    SupportCtx ctx = {p1, p2};
    OClosest points = gjk(&ctx);
    if (points.d - p1->r - p2->r <= 0.0) {
        contact_points(support_edge_poly(p1, points.n), support_edge_poly(p2, vneg(points.n)), points, info);
    }
}

/* cpCollide: type-ordered dispatch; returns count, *swapped when (a,b) reversed */
int ophys_collide(OSpace *s, int ia, int ib, OCollision *info, int *swapped) {
    const OShape *a = &s->shapes[ia], *b = &s->shapes[ib];
    info->count = 0;
    info->n = v2(0, 0);
    *swapped = 0;
    if (a->type > b->type) { const OShape *t = a; a = b; b = t; *swapped = 1; }
    int code = a->type + b->type * 3;
    switch (code) {
    case 0: circle_to_circle(a, b, info); break;
    case 3: circle_to_segment(a, b, info); break;
    case 6: circle_to_poly(a, b, info); break;
    case 7: segment_to_poly(a, b, info); break;
    case 8: poly_to_poly(a, b, info); break;
    default: break; /* segment-segment never occurs (all segments static) */
    }
    return info->count;
}

static int filter_reject(const OShape *a, const OShape *b) {
    return (a->group != 0 && a->group == b->group) || (a->categories & b->mask) == 0 ||
           (b->categories & a->mask) == 0;
}
static int bb_intersects(const OShape *a, const OShape *b) {
    return (a->bb_l <= b->bb_r && b->bb_l <= a->bb_r && a->bb_b <= b->bb_t && b->bb_b <= a->bb_t);
}
static int is_static_shape(const OShape *sh) { return sh->body < 0; }

/* ---------------- arbiters ---------------------------------------------- */
static int find_arbiter(OSpace *s, int lo, int hi) {
    for (int i = 0; i < O_MAX_ARB; i++)
        if (s->arbs[i].used && s->arbs[i].key_lo == lo && s->arbs[i].key_hi == hi) return i;
    return -1;
}
static int new_arbiter(OSpace *s, int lo, int hi) {
    for (int i = 0; i < O_MAX_ARB; i++) {
        if (!s->arbs[i].used) {
            OArbiter *arb = &s->arbs[i];
            memset(arb, 0, sizeof(*arb));
            arb->used = 1; arb->key_lo = lo; arb->key_hi = hi;
            arb->state = ARB_FIRST;
            arb->stamp = 0;
            return i;
        }
    }
    s->overflow = 1;
    return -1;
}

static void collide_shapes(OSpace *s, int ia, int ib) {
    OShape *a = &s->shapes[ia], *b = &s->shapes[ib];
    /* QueryReject */
    if (!bb_intersects(a, b)) return;
    if (a->body >= 0 && a->body == b->body) return;
    if (filter_reject(a, b)) return;
    OCollision info;
    int sw;
    if (!ophys_collide(s, ia, ib, &info, &sw)) return;
    int sa = sw ? ib : ia, sb = sw ? ia : ib;
    int lo = ia < ib ? ia : ib, hi = ia < ib ? ib : ia;
    int ai = find_arbiter(s, lo, hi);
    if (ai < 0) ai = new_arbiter(s, lo, hi);
    if (ai < 0) return;
    OArbiter *arb = &s->arbs[ai];
    const OShape *A = &s->shapes[sa], *B = &s->shapes[sb];
    /* cpArbiterUpdate */
    OContact con[2];
    vec2 pa = A->body >= 0 ? s->bodies[A->body].p : A->sp;
    vec2 pb = B->body >= 0 ? s->bodies[B->body].p : B->sp;
    for (int i = 0; i < info.count; i++) {
        memset(&con[i], 0, sizeof(OContact));
        con[i].r1 = vsub(info.p1[i], pa);
        con[i].r2 = vsub(info.p2[i], pb);
        con[i].hash = info.hash[i];
        con[i].jnAcc = con[i].jtAcc = 0.0;
        for (int j = 0; j < arb->count; j++) {
            if (con[i].hash == arb->con[j].hash) {
                con[i].jnAcc = arb->con[j].jnAcc;
                con[i].jtAcc = arb->con[j].jtAcc;
            }
        }
    }
    arb->sa = sa; arb->sb = sb;
    for (int i = 0; i < info.count; i++) arb->con[i] = con[i];
    arb->count = info.count;
    arb->n = info.n;
    arb->e = 0.0 * 0.0; /* elasticity default 0 */
    arb->u = A->u * B->u;
    {
        vec2 svr = vsub(v2(0.0, 0.0), v2(0.0, 0.0));
        arb->surface_vr = vsub(svr, vmult(info.n, vdot(svr, info.n)));
    }
    if (arb->state == ARB_CACHED) arb->state = ARB_FIRST;
    /* sensors never reach the solver (they are skipped before collide_shapes) */
    if (s->nactive < O_MAX_ARB) s->active[s->nactive++] = ai;
    else s->overflow = 1;
    arb->stamp = s->stamp;
}

static void arbiter_prestep(OSpace *s, OArbiter *arb, double dt, double slop, double bias) {
    const OShape *A = &s->shapes[arb->sa], *B = &s->shapes[arb->sb];
    BRef a = bref(s, A->body), b = bref(s, B->body);
    vec2 n = arb->n;
    vec2 body_delta = vsub(b.p, a.p);
    for (int i = 0; i < arb->count; i++) {
        OContact *con = &arb->con[i];
        con->nMass = 1.0 / k_scalar(&a, &b, con->r1, con->r2, n);
        con->tMass = 1.0 / k_scalar(&a, &b, con->r1, con->r2, vperp(n));
        double dist = vdot(vadd(vsub(con->r2, con->r1), body_delta), n);
        con->bias = -bias * fmin_cp(0.0, dist + slop) / dt;
        con->jBias = 0.0;
        con->bounce = vdot(relative_velocity(&a, &b, con->r1, con->r2), n) * arb->e;
    }
}

static void arbiter_apply_cached(OSpace *s, OArbiter *arb, double dt_coef) {
    if (arb->state == ARB_FIRST) return;
    const OShape *A = &s->shapes[arb->sa], *B = &s->shapes[arb->sb];
    BRef a = bref(s, A->body), b = bref(s, B->body);
    vec2 n = arb->n;
    for (int i = 0; i < arb->count; i++) {
        OContact *con = &arb->con[i];
        vec2 j = vrotate(n, v2(con->jnAcc, con->jtAcc));
        apply_impulses(&a, &b, con->r1, con->r2, vmult(j, dt_coef));
    }
}

static void arbiter_apply(OSpace *s, OArbiter *arb) {
    const OShape *A = &s->shapes[arb->sa], *B = &s->shapes[arb->sb];
    BRef a = bref(s, A->body), b = bref(s, B->body);
    vec2 n = arb->n, surface_vr = arb->surface_vr;
    double friction = arb->u;
    for (int i = 0; i < arb->count; i++) {
        OContact *con = &arb->con[i];
        double nMass = con->nMass;
        vec2 r1 = con->r1, r2 = con->r2;
        vec2 vb1 = vadd(*a.vb, vmult(vperp(r1), *a.wb));
        vec2 vb2 = vadd(*b.vb, vmult(vperp(r2), *b.wb));
        vec2 vr = vadd(relative_velocity(&a, &b, r1, r2), surface_vr);
        double vbn = vdot(vsub(vb2, vb1), n);
        double vrn = vdot(vr, n);
        double vrt = vdot(vr, vperp(n));
        double jbn = (con->bias - vbn) * nMass;
        double jbnOld = con->jBias;
        con->jBias = fmax_cp(jbnOld + jbn, 0.0);
        double jn = -(con->bounce + vrn) * nMass;
        double jnOld = con->jnAcc;
        con->jnAcc = fmax_cp(jnOld + jn, 0.0);
        double jtMax = friction * con->jnAcc;
        double jt = -vrt * con->tMass;
        double jtOld = con->jtAcc;
        con->jtAcc = fclamp(jtOld + jt, -jtMax, jtMax);
        apply_bias_impulses(&a, &b, r1, r2, vmult(n, con->jBias - jbnOld));
        apply_impulses(&a, &b, r1, r2, vrotate(n, v2(con->jnAcc - jnOld, con->jtAcc - jtOld)));
    }
}

/* ---------------- cpSpaceStep ------------------------------------------- */
void ophys_step(OSpace *s, double dt) {
    if (dt == 0.0) return;
    s->stamp++;
    double prev_dt = s->curr_dt;
    s->curr_dt = dt;
    /* reset last step's arbiters to NORMAL */
    for (int i = 0; i < s->nactive; i++) s->arbs[s->active[i]].state = ARB_NORMAL;
    s->nactive = 0;
    /* integrate positions (dynamic + kinematic bodies, add order) */
    for (int i = 0; i < s->nbodies; i++) {
        OBody *b = &s->bodies[i];
        if (b->type == BODY_STATIC) continue;
        b->p = vadd(b->p, vmult(vadd(b->v, b->v_bias), dt));
        b->a = b->a + (b->w + b->w_bias) * dt;
        body_set_transform(b);
        b->v_bias = v2(0.0, 0.0);
        b->w_bias = 0.0;
    }
    /* update dynamic shape caches */
    for (int i = 0; i < s->nshapes; i++)
        if (!is_static_shape(&s->shapes[i])) ophys_shape_update(s, i);
    /* broadphase + narrowphase, canonical order */
    for (int i = 0; i < s->nshapes; i++) {
        OShape *a = &s->shapes[i];
        if (is_static_shape(a) || a->sensor) continue;
        for (int j = 0; j < s->nshapes; j++) {
            OShape *b = &s->shapes[j];
            if (!is_static_shape(b) || b->sensor) continue;
            collide_shapes(s, i, j);
        }
        for (int j = i + 1; j < s->nshapes; j++) {
            OShape *b = &s->shapes[j];
            if (is_static_shape(b) || b->sensor) continue;
            collide_shapes(s, i, j);
        }
    }
    /* cached arbiter filter (cpSpaceArbiterSetFilter) */
    for (int i = 0; i < O_MAX_ARB; i++) {
        OArbiter *arb = &s->arbs[i];
        if (!arb->used) continue;
        uint32_t ticks = s->stamp - arb->stamp;
        if (ticks >= 1 && arb->state != ARB_CACHED) arb->state = ARB_CACHED;
        if (ticks >= 3) { arb->used = 0; arb->count = 0; }
    }
    /* prestep */
    double slop = s->collision_slop;
    double biasCoef = 1.0 - pow(s->collision_bias, dt);
    for (int i = 0; i < s->nactive; i++) arbiter_prestep(s, &s->arbs[s->active[i]], dt, slop, biasCoef);
    for (int i = 0; i < s->ncons; i++) cons_prestep(s, &s->cons[i], dt);
    /* integrate velocities: gravity 0, damping 1, no forces -> v = v*1 + 0*dt */
    for (int i = 0; i < s->nbodies; i++) {
        OBody *b = &s->bodies[i];
        if (b->type != BODY_DYNAMIC) continue;
        b->v = vadd(vmult(b->v, 1.0), vmult(vadd(v2(0.0, 0.0), vmult(v2(0.0, 0.0), b->m_inv)), dt));
        b->w = b->w * 1.0 + 0.0 * b->i_inv * dt;
    }
    /* cached impulses */
    double dt_coef = (prev_dt == 0.0 ? 0.0 : dt / prev_dt);
    for (int i = 0; i < s->nactive; i++) arbiter_apply_cached(s, &s->arbs[s->active[i]], dt_coef);
    for (int i = 0; i < s->ncons; i++) cons_apply_cached(s, &s->cons[i], dt_coef);
    /* solver */
    for (int it = 0; it < s->iterations; it++) {
        for (int i = 0; i < s->nactive; i++) arbiter_apply(s, &s->arbs[s->active[i]]);
        for (int i = 0; i < s->ncons; i++) cons_apply(s, &s->cons[i], dt);
    }
}

/* ---------------- queries ----------------------------------------------- */
/* pymunk Space.shape_query (cpSpaceShapeQuery: every shape, sensors included) minus an ignore set
 * (geom.py:224-226: collisions - ignore_set); ign[j] != 0 ignores shape j, NULL ignores nothing */
int ophys_shape_query_any_ign(OSpace *s, int si, const uint8_t *ign) {
    OShape *a = &s->shapes[si];
    ophys_shape_update(s, si);
    for (int j = 0; j < s->nshapes; j++) {
        if (j == si || (ign && ign[j])) continue;
        OShape *b = &s->shapes[j];
        if (!bb_intersects(a, b)) continue;
        if (filter_reject(a, b)) continue;
        OCollision info; int sw;
        if (ophys_collide(s, si, j, &info, &sw) > 0) return 1;
    }
    return 0;
}

int ophys_shape_query_any(OSpace *s, int si) { return ophys_shape_query_any_ign(s, si, NULL); }

static vec2 closest_point_on_segment(vec2 p, vec2 a, vec2 b) {
    vec2 delta = vsub(a, b);
    double t = fclamp01(vdot(delta, vsub(p, b)) / vlengthsq(delta));
    return vadd(b, vmult(delta, t));
}

double ophys_poly_point_query(const OShape *sh, vec2 p) {
    int count = sh->count;
    vec2 v0 = sh->tv[count - 1];
    double minDist = INFINITY;
    int outside = 0;
    for (int i = 0; i < count; i++) {
        vec2 v1 = sh->tv[i];
        outside = outside || (vdot(sh->tpn[i], vsub(p, v1)) > 0.0);
        vec2 closest = closest_point_on_segment(p, v0, v1);
        double dist = vlength(vsub(p, closest));
        if (dist < minDist) minDist = dist;
        v0 = v1;
    }
    double dist = (outside ? minDist : -minDist);
    return dist - sh->r;
}
