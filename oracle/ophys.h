/*
 * ophys.h -- internal structures of the oracle's Chipmunk2D 7.0.x restatement.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 */
#ifndef MG_OPHYS_H
#define MG_OPHYS_H
#include <stdint.h>
#include "oracle.h"

enum { BODY_DYNAMIC = 0, BODY_KINEMATIC = 1, BODY_STATIC = 2 };
enum { SH_CIRCLE = 0, SH_SEGMENT = 1, SH_POLY = 2 };
enum { C_PIVOT = 0, C_GEAR = 1, C_ROTLIMIT = 2, C_MOTOR = 3, C_SPRING = 4 };
enum { ARB_FIRST = 0, ARB_NORMAL = 1, ARB_CACHED = 3, ARB_IGNORE = 2 };

typedef struct {
    int type;
    double m, m_inv, i, i_inv;
    vec2 p, v, v_bias;
    double a, w, w_bias;
    double rc, rs; /* transform rotation: (cos a, sin a); cog is 0 for every body here */
} OBody;

typedef struct {
    int type;
    int body;  /* index into space bodies; -1 = a static body with transform (sc, ss, sp) */
    vec2 sp;   /* static body position (identity rotation) */
    double r, u;
    int sensor;
    uint32_t group, categories, mask;
    uint64_t hashid;
    int entity;
    /* local geometry */
    vec2 c;             /* circle centre */
    vec2 a, b, n;       /* segment */
    int count;          /* poly */
    vec2 v[O_MAX_VERTS], pn[O_MAX_VERTS];
    /* cached world data */
    vec2 tc, ta, tb, tn;
    vec2 tv[O_MAX_VERTS], tpn[O_MAX_VERTS];
    double bb_l, bb_b, bb_r, bb_t;
} OShape;

typedef struct {
    int type, a, b; /* body indices, -1 = static body */
    double maxForce, maxBias, errorBias;
    /* pivot */
    vec2 anchorA, anchorB, r1, r2, jAccv, biasv;
    double k11, k12, k21, k22;
    /* scalar joints */
    double phase, ratio, ratio_inv, iSum, bias, jAcc;
    double min, max;        /* rotary limit */
    double rate;            /* motor */
    double restAngle, stiffness, damping, w_coef, target_wrn; /* spring */
} OCons;

typedef struct {
    vec2 r1, r2;
    double nMass, tMass, bounce, jnAcc, jtAcc, jBias, bias;
    uint64_t hash;
} OContact;

typedef struct {
    int used;
    int key_lo, key_hi;  /* unordered shape pair */
    int sa, sb;          /* shapes in collision order (a, b) */
    int state;
    uint32_t stamp;
    int count;
    OContact con[2];
    vec2 n, surface_vr;
    double u, e;
} OArbiter;

typedef struct {
    int nbodies, nshapes, ncons;
    OBody bodies[O_MAX_BODIES];
    OShape shapes[O_MAX_SHAPES];
    OCons cons[O_MAX_CONS];
    OArbiter arbs[O_MAX_ARB];
    int active[O_MAX_ARB];
    int nactive;
    uint32_t stamp;
    double curr_dt, prev_dt;
    double collision_slop, collision_bias;
    int iterations;
    int overflow; /* set if a fixed-size table overflowed */
} OSpace;

typedef struct {
    vec2 a, b;   /* surface points */
    vec2 n;
    double d;
} OClosest;

typedef struct {
    int count;
    vec2 n;
    vec2 p1[2], p2[2];
    uint64_t hash[2];
} OCollision;

/* physics API used by scene.c / env.c */
void ophys_init(OSpace *s);
int ophys_add_body(OSpace *s, int type, double m, double i, vec2 p, double a);
void ophys_body_set_angle(OSpace *s, int b, double a);
void ophys_body_set_position(OSpace *s, int b, vec2 p);
int ophys_add_circle(OSpace *s, int body, double r, vec2 offset);
int ophys_add_segment(OSpace *s, vec2 a, vec2 b, double r);
int ophys_add_poly(OSpace *s, int body, int count, const vec2 *verts, double r, int raw);
int ophys_add_static_box(OSpace *s, vec2 pos, double w, double h);
void ophys_shape_update(OSpace *s, int sh);
int ophys_add_pivot2(OSpace *s, int a, int b, vec2 anchorA, vec2 anchorB);
int ophys_add_pivot1(OSpace *s, int a, int b, vec2 pivot);
int ophys_add_gear(OSpace *s, int a, int b, double phase, double ratio);
int ophys_add_rotlimit(OSpace *s, int a, int b, double min, double max);
int ophys_add_motor(OSpace *s, int a, int b, double rate);
int ophys_add_spring(OSpace *s, int a, int b, double rest, double k, double c);
void ophys_step(OSpace *s, double dt);
int ophys_collide(OSpace *s, int a, int b, OCollision *out, int *swapped);
/* shape_query semantics (cpSpaceShapeQuery / pymunk Space.shape_query): any hit */
int ophys_shape_query_any(OSpace *s, int sh);
int ophys_shape_query_any_ign(OSpace *s, int sh, const uint8_t *ign);
double ophys_poly_point_query(const OShape *sh, vec2 p);
extern long ophys_epa_runs; /* EPA runs so far (tests) */

#endif
