/*
 * oscene.h -- oracle scene model: entities, render geoms, env state.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 */
#ifndef MG_OSCENE_H
#define MG_OSCENE_H
#include "ophys.h"

enum { ENT_ARENA = 0, ENT_GOAL = 1, ENT_ROBOT = 2, ENT_BLOCK = 3 };
enum { OUTLINE_NONE = 0, OUTLINE_SOLID = 1, OUTLINE_DASHED = 2 };

#define O_MAX_PTS 101
#define O_MAX_XF 64

typedef struct { double m[9]; } OXform;

typedef struct {
    int npts;
    vec2 pts[O_MAX_PTS];
    int outline;
    uint8_t col[3], ocol[3];
    int nxf;
    int xf[4]; /* Geom.transforms in list order (index into env xf table) */
} OGeom;

typedef struct {
    int kind, type, colour;
    double gx, gy, gh, gw;   /* goal region x, y, h, w */
    vec2 pos; double angle;  /* initial pose */
    int body0, nbodies;
    int shape0, nshapes;
    int xf_main;             /* per-entity transform updated at pre_draw */
    int xf_aux[4];           /* robot: finger L/R, pupil L/R */
    int role;                /* match regions: 1 target, 2 distractor */
} OEntity;

struct OEnv {
    int task, flags, preproc, max_steps;
    o_mt rng;
    OSpace space;
    OEntity ents[O_MAX_ENTS];
    int nents;
    OGeom geoms[O_MAX_GEOMS];
    int ngeoms;
    OXform xf[O_MAX_XF];
    int nxf;
    int robot;    /* entity index */
    int goal;     /* entity index or -1 */
    int star_groups;
    double pv[5]; /* PhysicsVariables: robot_pos, robot_rot, finger, shape_trans, shape_rot */
    double target_speed, rel_turn, target_finger;
    int episode_steps;
    int max_tries;         /* geom.py:198 max_tries = 10000 (tests lower it to force retries) */
    int placement_retries; /* failed pm_randomise_all_poses retries in the last reset (tests only) */
    int placement_error; /* geom.py:335-336: PlacementError after max_retries */
    double last_score;
    /* PickAndPlace (pick_and_place.py:30-85): target shape entity, ids, position */
    int target_ent, target_type_id, target_colour_id;
    vec2 target_pos;
    /* LoRes frame history (newest last) */
    uint8_t hist_allo[4][O_LORES * O_LORES * 3];
    uint8_t hist_ego[4][O_LORES * O_LORES * 3];
};

/* scene.c */
void oscene_reset(OEnv *e);
void oscene_robot_update(OEnv *e);
void oscene_set_action(OEnv *e, int action);
double oscene_score(OEnv *e);
double oscene_debug_reward(OEnv *e);
int o_longest_line(const double *px, const double *py, int n, double inlier_dist, double max_sep);
void oscene_pre_draw(OEnv *e);
/* raster.c */
void oraster_render(const OEnv *e, int ego, uint8_t *frame384);
void oraster_downsample(const uint8_t *frame384, uint8_t *out96);

extern const uint8_t O_PALETTE[5][4][3]; /* [colour][base, darken, lighten2, lighten4] */

#endif
