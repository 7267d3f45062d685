/*
 * sandbox.c -- a bare Chipmunk-7 space over the oracle's physics (phys.c) for the
 * known-answer tests (tests/test_oracle_known_answers.py).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The env code (scene.c) builds spaces the way base_env.py:206-208 does; these
 * entry points build arbitrary small ones (a free body, a body pressed into a
 * wall, a single joint) so that each piece of SURVEY.md Appendix A can be checked
 * against its analytic behaviour: free flight, pivot max-force ramps, the contact
 * bias converging a penetration to collision_slop, RotaryLimit, SimpleMotor rate,
 * DampedRotarySpring decay -- and the narrowphase (cpCollide) on hand-placed shape pairs, with the arbiter
 * table's warm-start / persistence behaviour across steps (tests/test_oracle_narrowphase.py).
 */
#include <stdlib.h>
#include "ophys.h"

OSpace *osb_new(void) {
    OSpace *s = (OSpace *)malloc(sizeof(OSpace));
    ophys_init(s);
    return s;
}
void osb_free(OSpace *s) { free(s); }

int osb_add_body(OSpace *s, int type, double m, double i, double px, double py, double a) {
    int b = ophys_add_body(s, type, m, i, (vec2){px, py}, a);
    if (b >= 0) ophys_body_set_angle(s, b, a);
    return b;
}
void osb_set_velocity(OSpace *s, int b, double vx, double vy, double w) {
    s->bodies[b].v = (vec2){vx, vy};
    s->bodies[b].w = w;
}
/* px, py, a, vx, vy, w, v_bias.x, v_bias.y, w_bias */
void osb_get_body(const OSpace *s, int b, double *out) {
    const OBody *B = &s->bodies[b];
    out[0] = B->p.x; out[1] = B->p.y; out[2] = B->a;
    out[3] = B->v.x; out[4] = B->v.y; out[5] = B->w;
    out[6] = B->v_bias.x; out[7] = B->v_bias.y; out[8] = B->w_bias;
}
int osb_add_circle(OSpace *s, int body, double r, double ox, double oy, double u) {
    int sh = ophys_add_circle(s, body, r, (vec2){ox, oy});
    if (sh >= 0) s->shapes[sh].u = u;
    return sh;
}
int osb_add_segment(OSpace *s, double ax, double ay, double bx, double by, double r, double u) {
    int sh = ophys_add_segment(s, (vec2){ax, ay}, (vec2){bx, by}, r);
    if (sh >= 0) s->shapes[sh].u = u;
    return sh;
}
int osb_add_poly(OSpace *s, int body, int n, const double *xy, double r, double u) {
    vec2 v[O_MAX_VERTS];
    if (n > O_MAX_VERTS) return -1;
    for (int i = 0; i < n; i++) v[i] = (vec2){xy[2 * i], xy[2 * i + 1]};
    int sh = ophys_add_poly(s, body, n, v, r, 0);
    if (sh >= 0) s->shapes[sh].u = u;
    return sh;
}
/* kind: 0 pivot (world pivot p0, p1), 1 gear (phase p0, ratio p1), 2 rotary limit (min p0, max p1),
 * 3 simple motor (rate p0), 4 damped rotary spring (rest p0, stiffness p1, damping p2) */
int osb_add_constraint(OSpace *s, int kind, int a, int b, double p0, double p1, double p2) {
    switch (kind) {
    case 0: return ophys_add_pivot1(s, a, b, (vec2){p0, p1});
    case 1: return ophys_add_gear(s, a, b, p0, p1);
    case 2: return ophys_add_rotlimit(s, a, b, p0, p1);
    case 3: return ophys_add_motor(s, a, b, p0);
    case 4: return ophys_add_spring(s, a, b, p0, p1, p2);
    }
    return -1;
}
void osb_set_constraint(OSpace *s, int c, double max_force, double max_bias, double error_bias) {
    s->cons[c].maxForce = max_force;
    s->cons[c].maxBias = max_bias;
    s->cons[c].errorBias = error_bias;
}
double osb_constraint_impulse(const OSpace *s, int c) { return s->cons[c].jAcc; }
void osb_step(OSpace *s, double dt) { ophys_step(s, dt); }
void osb_set_iterations(OSpace *s, int n) { s->iterations = n; }

/* Body.angle / Body.position setters, then the body's shapes re-cached (cpSpaceReindexShapesForBody) */
void osb_set_pose(OSpace *s, int b, double px, double py, double a) {
    ophys_body_set_angle(s, b, a);
    ophys_body_set_position(s, b, (vec2){px, py});
    for (int k = 0; k < s->nshapes; k++)
        if (s->shapes[k].body == b) ophys_shape_update(s, k);
}

/* cpCollide(shape ia, shape ib) (narrowphase only, no broadphase / filters):
 * out = [count, swapped, n.x, n.y, then per contact p1.x, p1.y, p2.x, p2.y], hash[k] = contact k's hash.
 * Shapes in collision order (a = the lower shape type); n points from a to b; depth = -dot(p2 - p1, n). */
int osb_collide(OSpace *s, int ia, int ib, double *out, uint64_t *hash) {
    OCollision info;
    int sw;
    int n = ophys_collide(s, ia, ib, &info, &sw);
    out[0] = n; out[1] = sw; out[2] = info.n.x; out[3] = info.n.y;
    for (int k = 0; k < n; k++) {
        double *o = out + 4 + 4 * k;
        o[0] = info.p1[k].x; o[1] = info.p1[k].y; o[2] = info.p2[k].x; o[3] = info.p2[k].y;
        hash[k] = info.hash[k];
    }
    return n;
}
long osb_epa_runs(void) { return ophys_epa_runs; }

/* the i-th solved arbiter in full: out = [slot, state, count, body a, body b, n.x, n.y, u, then per contact
 * r1.x, r1.y, r2.x, r2.y, jnAcc, jtAcc, nMass, tMass, bias, jBias], hash[k] = contact k's hash */
int osb_arbiter_ex(const OSpace *s, int i, double *out, uint64_t *hash) {
    const int slot = s->active[i];
    const OArbiter *A = &s->arbs[slot];
    out[0] = slot; out[1] = A->state; out[2] = A->count;
    out[3] = s->shapes[A->sa].body; out[4] = s->shapes[A->sb].body;
    out[5] = A->n.x; out[6] = A->n.y; out[7] = A->u;
    for (int k = 0; k < A->count; k++) {
        const OContact *c = &A->con[k];
        double *o = out + 8 + 10 * k;
        o[0] = c->r1.x; o[1] = c->r1.y; o[2] = c->r2.x; o[3] = c->r2.y; o[4] = c->jnAcc; o[5] = c->jtAcc;
        o[6] = c->nMass; o[7] = c->tMass; o[8] = c->bias; o[9] = c->jBias;
        hash[k] = c->hash;
    }
    return A->count;
}
/* overwrite contact k's accumulated impulses of the i-th solved arbiter (warm-start tests) */
void osb_arbiter_set_impulse(OSpace *s, int i, int k, double jn, double jt) {
    OContact *c = &s->arbs[s->active[i]].con[k];
    c->jnAcc = jn; c->jtAcc = jt;
}
int osb_num_arbiters(const OSpace *s) { return s->nactive; }
/* contacts of the i-th solved arbiter: count, normal, and per contact r1, r2, jnAcc, jtAcc */
int osb_arbiter(const OSpace *s, int i, double *out) {
    const OArbiter *A = &s->arbs[s->active[i]];
    out[0] = A->n.x; out[1] = A->n.y;
    for (int k = 0; k < A->count; k++) {
        const OContact *c = &A->con[k];
        double *o = out + 2 + 6 * k;
        o[0] = c->r1.x; o[1] = c->r1.y; o[2] = c->r2.x; o[3] = c->r2.y; o[4] = c->jnAcc; o[5] = c->jtAcc;
    }
    return A->count;
}
