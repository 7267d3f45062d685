// mg_state.h -- per-env structure-of-arrays state of the batched simulator.
//
// Every array is [slot][N] with N the env count padded to a multiple of 64:
// lane l of a wavefront owns env (64*wave + l), so each field access of a
// wavefront is one contiguous 512-byte (double) / 64-byte (int8) segment.
// Physics runs one env per lane (Chipmunk's sequential-impulse solver is a
// Gauss-Seidel sweep in a fixed order, so the parallelism is across envs);
// rendering runs one workgroup per (env, view).
#pragma once
#include "mg_common.h"

struct ShapeW;  // mg_phys.h

struct MGState {
    int N;      // padded env count (multiple of 64); row stride of every [slot][N] array
    int n_envs; // live env count
    int cons_cap, arb_cap; // constraint / arbiter slots per env (MG_MAX_* in HBM; smaller in LDS views)
    int max_tries;         // pm_randomise_pose max_tries (geom.py:198: 10000; tests lower it to force layout retries)
    // ---- bodies [MG_MAX_BODIES][N] ----
    double *bpx, *bpy, *bvx, *bvy, *ba, *bw, *bvbx, *bvby, *bwb, *brc, *brs, *bminv, *biinv, *bacache;
    int8_t *bkin;   // 1 = kinematic
    int32_t *nbodies;
    // ---- dynamic shapes [MG_MAX_SHAPES][N] ----
    int8_t *sbody, *spoly, *sent; // body slot; library poly id (-1 circle); owning entity
    int16_t *sgroup, *shash; // filter group; Chipmunk shape hashid (global add index)
    uint8_t *scat;  // categories != 0 (pm_randomise_all_poses disables shapes)
    double *sr, *su, *sbbl, *sbbb, *sbbr, *sbbt;
    int32_t *nshapes;
    // ---- constraints [MG_MAX_CONS][N] ----
    int8_t *ctype, *ca, *cb; // -1 = static body
    double *cp;              // [16][MG_MAX_CONS][N] parameters / accumulators, see mg_phys.h
    int32_t *ncons;
    // ---- arbiters [MG_MAX_ARB][N] ----
    int32_t *akey;           // lo * 128 + hi, -1 = free
    uint32_t *astamp;
    int8_t *astate, *acount, *asa, *asb; // asa/asb: body slots of shapes a, b (-1 static)
    double *anx, *any, *au;
    double *acon;            // [2 contacts][10 fields][MG_MAX_ARB][N]
    uint64_t *ahash;         // [2][MG_MAX_ARB][N]
    int8_t *active;          // [MG_MAX_ARB][N]
    int32_t *nactive;
    uint32_t *stamp;
    double *curr_dt;
    int32_t *overflow;       // per env error flags
    uint8_t *rg_retry;       // [N][2]: render class chain level that holds each (env, view) this episode
    // ---- robot control + physics variables [N] ----
    double *target_speed, *rel_turn, *target_finger;
    int32_t *robot_body0, *robot_cons0;
    double *pv;              // [5][N]
    // ---- entities [MG_MAX_ENTS][N] ----
    int8_t *ekind, *etype, *ecol, *erole, *ebody0, *eshape0, *enshapes;
    double *ex, *ey, *eang, *eh, *ew;
    int32_t *nents;
    int32_t *goal_ent;       // [N] last goal entity added (-1 none); goal body positions are the goal
                             // entities' ex/ey (static sensors, moved only by reset randomisers)
    // ---- episode ----
    int32_t *episode_steps;
    // PickAndPlace (pick_and_place.py:30-85): target shape entity, (type id, colour id), target position
    int32_t *tgt_ent, *tgt_ids;  // [N], [2][N]
    double *tgt_x, *tgt_y;       // [N]
    double *target_out;          // bound output f64[N][4] (target_type, target_colour, x, y) or null
    // ---- RNG: numpy legacy MT19937 per env ----
    uint32_t *mt_key;        // [624][N]
    int32_t *mt_pos;         // [N]
    // the env's MT19937 state cached in the wave's LDS during a cooperative reset (reset_kernel): key[0..623],
    // [624] = pos; null: draws go to mt_key / mt_pos in HBM (the step kernel's fused resets)
    uint32_t *mt_lds;
    // ---- LoRes frame history (downsampled, newest last) ----
    uint8_t *hist_allo;      // [4][N][96*96*3]
    uint8_t *hist_ego;       // [4][N][96*96*3]
    int32_t *hist_head;      // [N] ring head
    // allocentric static layer: the LoRes allo frame of the env's body-less entities alone (arena, goals --
    // fixed for the whole episode), written by the episode's first allo render; a 4x4 block that no
    // body's geometry reaches copies it instead of being resolved (render_kernel)
    uint8_t *scache;         // [N][96*96*3]
    uint8_t *scache_ok;      // [N] 1: scache holds this episode's static layer
    // LDS views of the compile-time robot scenes: 3 world-space shapes per lane (narrowphase operands:
    // the queried shape, a wall, the other shape) in LDS instead of per-lane scratch; null elsewhere
    ShapeW *shw;
};

// constraint parameter slots (cp[k][c][env])
enum {
    CP_MAXF = 0, CP_MAXB = 1, CP_BCOEF = 2, CP_JACC = 3, CP_JACC2 = 4, CP_ISUM = 5, CP_BIAS = 6, CP_BIAS2 = 7,
    // pivot
    CP_AAX = 8, CP_AAY = 9, CP_ABX = 10, CP_ABY = 11, CP_R1X = 12, CP_R1Y = 13, CP_R2X = 14, CP_R2Y = 15,
    CP_K11 = 16, CP_K12 = 17, CP_K21 = 18, CP_K22 = 19,
    // gear / limit / motor / spring reuse 8..
    CP_PHASE = 8, CP_RATIO = 9, CP_RATIO_INV = 10,
    CP_MIN = 8, CP_MAX = 9,
    CP_RATE = 8,
    CP_REST = 8, CP_STIFF = 9, CP_WCOEF = 10, CP_TWRN = 11,
    CP_NUM = 20
};
// contact fields (acon[k][field][arb][env])
enum { AC_R1X = 0, AC_R1Y, AC_R2X, AC_R2Y, AC_NMASS, AC_TMASS, AC_JN, AC_JT, AC_JB, AC_BIAS, AC_NUM };
enum { ARB_FIRST = 0, ARB_NORMAL = 1, ARB_CACHED = 3 };
