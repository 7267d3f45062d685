// mg_common.h -- layout shared by the host C-ABI and the gfx950 kernels.
//
// The scene library (mg_library) holds every per-entity-type constant of
// MAGICAL's scene (entities.py / geom.py / render.py formulas): physics poly
// tables in pymunk hull order, masses and moments, render polygons with their
// transform chains, palette, solver constants.  The Python host
// (magical_amd/tables.py) fills it from the reference formulas; kernels read it
// from device memory.  Per-env state lives in structure-of-arrays buffers
// indexed [slot * N + env] so a wavefront's 64 lanes (64 envs) touch 64
// consecutive elements.
#pragma once
#include <stdint.h>

#define MG_MAX_BODIES 16
#define MG_MAX_SHAPES 64
#define MG_MAX_CONS 32
#define MG_MAX_ARB 48
#define MG_ITERATIONS 10   // Space.iterations (base_env.py:208): solver sweeps per substep
#define MG_MAX_ENTS 14
#define MG_MAX_PVERTS 8
#define MG_MAX_LIB_POLYS 32
#define MG_MAX_RPOLYS 64
#define MG_MAX_RPTS 2400
#define MG_MAX_STATIC_XF 8
#define MG_RES 384
#define MG_LORES 96

// tasks / rand flags / preprocessors (mirror benchmarks/__init__.py:269-307, 427-1102)
enum { MG_TASK_MOVE_TO_REGION = 0, MG_TASK_MOVE_TO_CORNER = 1, MG_TASK_CLUSTER_COLOUR = 2,
       MG_TASK_CLUSTER_SHAPE = 3, MG_TASK_MATCH_REGIONS = 4, MG_TASK_MAKE_LINE = 5,
       MG_TASK_FIND_DUPE = 6, MG_TASK_FIX_COLOUR = 7, MG_TASK_PICK_AND_PLACE = 8 };
enum { MG_RAND_LAYOUT_MINOR = 1, MG_RAND_LAYOUT_FULL = 2, MG_RAND_COLOUR = 4, MG_RAND_SHAPE_TYPE = 8,
       MG_RAND_SHAPE_COUNT = 16, MG_RAND_DYNAMICS = 32,
       MG_DEBUG_REWARD = 64 /* debug_reward=True (move_to_corner.py:85-100, pick_and_place.py:108-124) */ };
enum { MG_PREPROC_NONE = 0, MG_PREPROC_LORES4E = 1, MG_PREPROC_LORESSTACK = 2, MG_PREPROC_LORES3EA = 3,
       MG_PREPROC_LORES4A = 4, MG_PREPROC_LORESCHW4E = 5 };

enum { MG_ENT_ARENA = 0, MG_ENT_GOAL = 1, MG_ENT_ROBOT = 2, MG_ENT_BLOCK = 3 };
enum { MG_SHAPE_TRIANGLE = 0, MG_SHAPE_SQUARE = 1, MG_SHAPE_PENTAGON = 2, MG_SHAPE_HEXAGON = 3,
       MG_SHAPE_OCTAGON = 4, MG_SHAPE_CIRCLE = 5, MG_SHAPE_STAR = 6, MG_NUM_SHAPE_TYPES = 7 };
enum { MG_COL_RED = 0, MG_COL_GREEN = 1, MG_COL_BLUE = 2, MG_COL_YELLOW = 3, MG_COL_GREY = 4 };

// render colour references: palette row is either the entity colour or grey
enum { MG_RC_ENT_BASE = 0, MG_RC_ENT_DARK = 1, MG_RC_ENT_LIGHT2 = 2, MG_RC_GREY_BASE = 3, MG_RC_GREY_DARK = 4,
       MG_RC_GREY_LIGHT4 = 5, MG_RC_WHITE = 6, MG_RC_PUPIL = 7, MG_RC_NONE = 8 };
// transform-chain references (Geom.transforms entries)
enum { MG_XF_MAIN = 0, MG_XF_FINGER_L = 1, MG_XF_FINGER_R = 2, MG_XF_PUPIL_L = 3, MG_XF_PUPIL_R = 4,
       MG_XF_STATIC0 = 8 };
enum { MG_OUTLINE_NONE = 0, MG_OUTLINE_SOLID = 1, MG_OUTLINE_DASHED = 2 };

// shape filter: a shape whose categories were left 0 by pm_randomise_all_poses (geom.py:300-319, after a
// failed layout retry) collides with nothing; reset_env folds that into its group as this bit
#define MG_GROUP_OFF 0x4000

// constraint kinds
enum { MG_C_PIVOT = 0, MG_C_GEAR = 1, MG_C_ROTLIMIT = 2, MG_C_MOTOR = 3, MG_C_SPRING = 4 };

typedef struct {
    int32_t npts, pts_off, outline, col_ref, ocol_ref, nxf;
    int32_t xf[4];
} mg_rpoly;

typedef struct {
    // ---- solver constants (host libm: pow/exp are only needed as constants) ----
    double dt;                  // 1/fps/10 (base_env.py:248-255)
    double collision_bias_coef; // 1 - pow(pow(0.9, 60), dt)
    double slop;                // 0.01 (base_env.py:207)
    double default_bias_coef;   // 1 - pow(pow(0.9, 60), dt): joints with default errorBias
    double spring_w_coef;       // 1 - exp(-3e-3 * dt * (i_inv_robot + i_inv_eye))
    // ---- robot (entities.py:238-433) ----
    double robot_radius, robot_mass, robot_inertia, eye_mass, eye_inertia, finger_mass;
    double finger_inertia[2];
    double finger_rel[2][2];    // (side * r * 0.45, r * 0.1)
    double finger_lim[2][2];    // rotary limit [min, max] per finger
    double finger_angle_off[2]; // +pi/8 left, -pi/8 right
    int32_t finger_poly[4];     // library polys: L0, L1, R0, R1
    // ---- blocks (entities.py:580-754) ----
    int32_t block_nshapes[MG_NUM_SHAPE_TYPES];
    int32_t block_poly[MG_NUM_SHAPE_TYPES][8]; // library poly ids (-1: circle)
    double block_mass[MG_NUM_SHAPE_TYPES], block_inertia[MG_NUM_SHAPE_TYPES];
    double block_circle_r;
    // ---- physics poly library (pymunk hull order; planes[count+i]) ----
    int32_t n_polys;
    int32_t poly_count[MG_MAX_LIB_POLYS];
    double poly_r[MG_MAX_LIB_POLYS];
    double poly_v[MG_MAX_LIB_POLYS][MG_MAX_PVERTS][2];
    double poly_n[MG_MAX_LIB_POLYS][MG_MAX_PVERTS][2];
    // ---- render library (render.py Geom / Poly) ----
    int32_t n_rpolys;
    mg_rpoly rpoly[MG_MAX_RPOLYS];
    double rpts[MG_MAX_RPTS][2];
    int32_t arena_rpoly0, arena_nrpoly, goal_rpoly0, goal_nrpoly, robot_rpoly0, robot_nrpoly;
    int32_t block_rpoly0[MG_NUM_SHAPE_TYPES], block_nrpoly[MG_NUM_SHAPE_TYPES];
    double static_xf[MG_MAX_STATIC_XF][9];
    double allo_view[9];        // Viewer.set_bounds(+-1.02) composed with pygame flip
    double ego_scale_m[9], ego_tr1_m[9], pygame_m[9]; // set_cam_follow constants (render.py:290-371)
    uint8_t palette[5][4][4];   // [colour][base, dark, light2, light4][rgb_]
    uint8_t white[4], pupil[4], background[4];
} mg_library;

// One entity of a scene (an element of BaseEnv._entities in add order).
typedef struct {
    int32_t kind, type, colour, role;
    double x, y, angle; // robot / block pose; goal: top-left x, y
    double h, w;        // goal only
} mg_entity;
