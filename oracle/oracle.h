/*
 * oracle.h -- CPU restatement of MAGICAL's physics + render + LoRes hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in this directory is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and only as the checker / CPU baseline.  The product path is the HIP
 * library under magical-1_amd/csrc and fails loudly without it.
 *
 * Parity status: the reference's arithmetic lives in pymunk 5.6 (Chipmunk2D
 * 7.0.x), pygame 1.9.6 and opencv 4.x, none of which exist in this container.
 * This file restates their published algorithms (SURVEY.md Appendices A/B/D).
 * Pinned against golden vectors generated here from the reference's own
 * importable modules (magical/style.py, magical/phys_vars.py), numpy's legacy
 * RandomState (the reference RNG) and numpy's matmul (the reference's render
 * transform arithmetic): see tests/golden/make_golden.py.  Physics / raster /
 * resize parity against real pymunk/pygame/cv2 is UNPINNED.
 *
 * Every number is IEEE double unless stated; compiled with -ffp-contract=off.
 * sin/cos are correctly rounded (crmath.c), the behaviour of glibc <= 2.27
 * used in the reference's era; glibc 2.35 misrounds ~0.15% of arguments.
 */
#ifndef MG_ORACLE_H
#define MG_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { double x, y; } vec2;

/* ---- limits ---------------------------------------------------------- */
#define O_MAX_BODIES 24
#define O_MAX_SHAPES 64
#define O_MAX_CONS 40
#define O_MAX_ARB 96
#define O_MAX_VERTS 12
#define O_MAX_ENTS 16
#define O_MAX_GEOMS 192
#define O_RES 384
#define O_LORES 96

/* ---- tasks / variants / preprocessors (benchmarks/__init__.py:269-307,427-1102) */
enum { TASK_MOVE_TO_REGION = 0, TASK_MOVE_TO_CORNER = 1, TASK_CLUSTER_COLOUR = 2,
       TASK_CLUSTER_SHAPE = 3, TASK_MATCH_REGIONS = 4, TASK_MAKE_LINE = 5,
       TASK_FIND_DUPE = 6, TASK_FIX_COLOUR = 7, TASK_PICK_AND_PLACE = 8 };
enum { RAND_LAYOUT_MINOR = 1, RAND_LAYOUT_FULL = 2, RAND_COLOUR = 4, RAND_SHAPE_TYPE = 8,
       RAND_SHAPE_COUNT = 16, RAND_DYNAMICS = 32,
       DEBUG_REWARD = 64 /* debug_reward=True: dense shaped reward (move_to_corner.py:85-100, pick_and_place.py:108-124) */ };
enum { PREPROC_NONE = 0, PREPROC_LORES4E = 1, PREPROC_LORESSTACK = 2, PREPROC_LORES3EA = 3,
       PREPROC_LORES4A = 4, PREPROC_LORESCHW4E = 5 };

enum { SHAPE_TRIANGLE = 0, SHAPE_SQUARE = 1, SHAPE_PENTAGON = 2, SHAPE_HEXAGON = 3,
       SHAPE_OCTAGON = 4, SHAPE_CIRCLE = 5, SHAPE_STAR = 6 };
enum { COL_RED = 0, COL_GREEN = 1, COL_BLUE = 2, COL_YELLOW = 3, COL_GREY = 4 };

/* ---- low-level pieces exported for golden tests ---------------------- */
double o_crsin(double x);
double o_crcos(double x);
double o_crtan(double x);

typedef struct { uint32_t key[624]; int pos; } o_mt;
void o_mt_seed(o_mt *s, uint32_t seed);
uint32_t o_mt_next32(o_mt *s);
double o_mt_double(o_mt *s);
double o_mt_uniform(o_mt *s, double lo, double hi);
int64_t o_mt_randint(o_mt *s, int64_t lo, int64_t hi); /* [lo, hi) */
uint64_t o_mt_interval(o_mt *s, uint64_t max);

/* geometry tables (entities.py / geom.py formulas, pymunk hull ordering) */
int o_convex_hull(int count, const vec2 *verts, vec2 *result, int *first, double tol);
double o_moment_for_poly(double m, int count, const vec2 *verts, vec2 offset, double r);
/* writes parts into out (flattened, each part's verts incl. closing duplicate);
 * counts[i] = vertex count of part i; returns number of parts */
int o_star_decomposition(double out_rad, double in_rad, vec2 *out, int *counts, int max_parts);
void o_finger_verts(double upper, double fore, double thick, int side, vec2 upper_out[4], vec2 fore_out[4]);

/* 3x3 numpy-arith helpers (render.py Transform) */
void o_mat3_mul(const double *a, const double *b, double *out);
void o_transform_trs(double tx, double ty, double rot, double sx, double sy, double *out);
void o_allo_view(double *out);
void o_ego_view(double rx, double ry, double ra, double *out);

/* ---- env API ----------------------------------------------------------- */
typedef struct OEnv OEnv;
OEnv *oenv_create(int task, int rand_flags, int preproc, int max_episode_steps, uint32_t seed);
void oenv_destroy(OEnv *e);
void oenv_seed(OEnv *e, uint32_t seed);
/* bytes of one observation for this preproc (all keys concatenated in dict order) */
int oenv_obs_bytes(const OEnv *e);
/* 0 ok; -1 table overflow; -2 PlacementError (geom.py:335-336 raises; the
 * reference env would crash, the state is left as after the last retry) */
int oenv_reset(OEnv *e, uint8_t *obs);
int oenv_step(OEnv *e, int action, uint8_t *obs, double *reward, int *done, double *eval_score);
/* full-resolution views of the current state: [384][384][3] each */
void oenv_render_full(OEnv *e, uint8_t *allo, uint8_t *ego);
/* per dynamic/kinematic body: px, py, a, vx, vy, w  (returns body count) */
int oenv_get_bodies(const OEnv *e, double *out, int max_bodies);
int oenv_num_arbiters(const OEnv *e);
int oenv_get_arbiters(const OEnv *e, double *out, uint64_t *hash, int max_arbs);
void oenv_set_body_pose(OEnv *e, int body, double x, double y, double angle);
/* PickAndPlace observation extras: (target_type, target_colour, target_position x, y) */
void oenv_get_target(const OEnv *e, double out[4]);
/* per-env scene summary for tests: entity kinds/types/colours (returns count) */
int oenv_get_entities(const OEnv *e, int *kinds, int *types, int *colours, double *poses);
double oenv_last_score(const OEnv *e);
/* PhysicsVariables values of the current episode (base_env.py:49-57 order) */
void oenv_get_phys_vars(const OEnv *e, double out[5]);
/* palette [colour][base, darken, lighten2, lighten4][rgb] (style.py) */
void o_palette(uint8_t out[5][4][3]);
/* cv2 INTER_AREA 384^2 -> 96^2 restatement on an arbitrary frame */
void o_downsample(const uint8_t *frame384, uint8_t *out96);

/* pure restatements of the reference's scorers / action decode on explicit inputs (reference-fixture tests) */
double o_score_move_to_corner(double rx, double ry);                         /* move_to_corner.py:67-77 */
double o_shaped_move_to_corner(double rx, double ry, double sx, double sy);   /* move_to_corner.py:86-100 */
double o_cluster_score(int nblocks, const int *val, const double *x, const double *y); /* cluster.py:166-216 */
void o_action_decode(int action, double out[3]);                              /* entities.py:148-190,435-453 */

#ifdef __cplusplus
}
#endif
#endif
