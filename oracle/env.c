/*
 * env.c -- single-env API of the oracle: BaseEnv.reset/step + LoRes wrappers.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Follows base_env.py:190-307 (reset/step, 10 substeps of dt = 1/fps/10,
 * done at episode_steps >= max_episode_steps, reward = eval_score at done) and
 * benchmarks/__init__.py:51-190 (EagerDictFrameStack, FlattenFrameStack,
 * ResizeDictObservation), :269-307 (preprocessor table), :193-216 (ChannelsFirst).
 */
#include <stdlib.h>
#include <string.h>
#include "oscene.h"

#define LB (O_LORES * O_LORES * 3)

OEnv *oenv_create(int task, int flags, int preproc, int max_steps, uint32_t seed) {
    OEnv *e = (OEnv *)calloc(1, sizeof(OEnv));
    e->task = task; e->flags = flags; e->preproc = preproc; e->max_steps = max_steps;
    e->max_tries = 10000;
    o_mt_seed(&e->rng, seed);
    return e;
}
void oenv_destroy(OEnv *e) { free(e); }
void oenv_seed(OEnv *e, uint32_t seed) { o_mt_seed(&e->rng, seed); }

int oenv_obs_bytes(const OEnv *e) {
    switch (e->preproc) {
    case PREPROC_NONE: return 2 * O_RES * O_RES * 3;
    case PREPROC_LORESSTACK: return 2 * 4 * LB;
    default: return 6 * LB; /* allo + ego + past_obs(12 ch) */
    }
}

static void write_stack12(uint8_t *dst, const uint8_t *f0, const uint8_t *f1, const uint8_t *f2, const uint8_t *f3) {
    const uint8_t *fs[4] = {f0, f1, f2, f3};
    for (int p = 0; p < O_LORES * O_LORES; p++)
        for (int k = 0; k < 4; k++) memcpy(dst + p * 12 + 3 * k, fs[k] + p * 3, 3);
}
static void chw(uint8_t *dst, const uint8_t *src, int c) {
    for (int p = 0; p < O_LORES * O_LORES; p++)
        for (int k = 0; k < c; k++) dst[k * O_LORES * O_LORES + p] = src[p * c + k];
}

static void write_obs(OEnv *e, uint8_t *obs, const uint8_t *allo384, const uint8_t *ego384) {
    uint8_t(*A)[LB] = e->hist_allo, (*E)[LB] = e->hist_ego;
    switch (e->preproc) {
    case PREPROC_NONE:
        memcpy(obs, allo384, (size_t)O_RES * O_RES * 3);
        memcpy(obs + O_RES * O_RES * 3, ego384, (size_t)O_RES * O_RES * 3);
        break;
    case PREPROC_LORES4E:
        memcpy(obs, A[3], LB); memcpy(obs + LB, E[3], LB);
        write_stack12(obs + 2 * LB, E[0], E[1], E[2], E[3]);
        break;
    case PREPROC_LORES3EA:
        memcpy(obs, A[3], LB); memcpy(obs + LB, E[3], LB);
        write_stack12(obs + 2 * LB, A[3], E[1], E[2], E[3]);
        break;
    case PREPROC_LORES4A:
        memcpy(obs, A[3], LB); memcpy(obs + LB, E[3], LB);
        write_stack12(obs + 2 * LB, A[0], A[1], A[2], A[3]);
        break;
    case PREPROC_LORESSTACK:
        write_stack12(obs, A[0], A[1], A[2], A[3]);
        write_stack12(obs + 4 * LB, E[0], E[1], E[2], E[3]);
        break;
    case PREPROC_LORESCHW4E: {
        uint8_t tmp[4 * LB];
        chw(obs, A[3], 3);
        chw(obs + LB, E[3], 3);
        write_stack12(tmp, E[0], E[1], E[2], E[3]);
        chw(obs + 2 * LB, tmp, 12);
        break;
    }
    }
}

static void render_both(OEnv *e, uint8_t *allo384, uint8_t *ego384) {
    oscene_pre_draw(e);
    oraster_render(e, 0, allo384);
    oraster_render(e, 1, ego384);
}

int oenv_reset(OEnv *e, uint8_t *obs) {
    e->placement_error = 0;
    e->placement_retries = 0;
    oscene_reset(e);
    uint8_t *a = (uint8_t *)malloc((size_t)O_RES * O_RES * 3), *g = (uint8_t *)malloc((size_t)O_RES * O_RES * 3);
    render_both(e, a, g);
    uint8_t la[LB], lg[LB];
    oraster_downsample(a, la);
    oraster_downsample(g, lg);
    for (int k = 0; k < 4; k++) { memcpy(e->hist_allo[k], la, LB); memcpy(e->hist_ego[k], lg, LB); }
    if (obs) write_obs(e, obs, a, g);
    free(a); free(g);
    e->last_score = 0.0;
    if (e->placement_error) return -2;
    return e->space.overflow ? -1 : 0;
}

int oenv_step(OEnv *e, int action, uint8_t *obs, double *reward, int *done, double *eval_score) {
    oscene_set_action(e, action);
    double spf = 1.0 / 8; /* fps = 8 (benchmarks/__init__.py:434-437) */
    double dt = spf / 10;
    for (int i = 0; i < 10; i++) {
        oscene_robot_update(e);
        ophys_step(&e->space, dt);
    }
    e->episode_steps++;
    int d = e->max_steps > 0 && e->episode_steps >= e->max_steps;
    double score = 0.0;
    if (d) score = oscene_score(e);
    e->last_score = score;
    if (reward) *reward = (e->flags & DEBUG_REWARD) ? oscene_debug_reward(e) : score;
    if (done) *done = d;
    if (eval_score) *eval_score = score;
    uint8_t *a = (uint8_t *)malloc((size_t)O_RES * O_RES * 3), *g = (uint8_t *)malloc((size_t)O_RES * O_RES * 3);
    render_both(e, a, g);
    for (int k = 0; k < 3; k++) { memcpy(e->hist_allo[k], e->hist_allo[k + 1], LB); memcpy(e->hist_ego[k], e->hist_ego[k + 1], LB); }
    oraster_downsample(a, e->hist_allo[3]);
    oraster_downsample(g, e->hist_ego[3]);
    if (obs) write_obs(e, obs, a, g);
    free(a); free(g);
    return e->space.overflow ? -1 : 0;
}

void oenv_render_full(OEnv *e, uint8_t *allo, uint8_t *ego) { render_both(e, allo, ego); }

int oenv_get_bodies(const OEnv *e, double *out, int max_bodies) {
    int n = e->space.nbodies < max_bodies ? e->space.nbodies : max_bodies;
    for (int i = 0; i < n; i++) {
        const OBody *b = &e->space.bodies[i];
        out[6 * i + 0] = b->p.x; out[6 * i + 1] = b->p.y; out[6 * i + 2] = b->a;
        out[6 * i + 3] = b->v.x; out[6 * i + 4] = b->v.y; out[6 * i + 5] = b->w;
    }
    return n;
}

int oenv_num_arbiters(const OEnv *e) { return e->space.nactive; }

/* the solved arbiters in active order (cpSpace arbiters list), as mg_get_arbiters dumps them:
 * out[i][28] = [slot, state, count, body a, body b, n.x, n.y, u, 2 x (r1.x, r1.y, r2.x, r2.y, jnAcc, jtAcc,
 * nMass, tMass, bias, jBias)], hash[i][2]; returns the number of arbiters written */
int oenv_get_arbiters(const OEnv *e, double *out, uint64_t *hash, int max_arbs) {
    int n = e->space.nactive < max_arbs ? e->space.nactive : max_arbs;
    for (int i = 0; i < n; i++) {
        const int slot = e->space.active[i];
        const OArbiter *A = &e->space.arbs[slot];
        double *o = out + 28 * i;
        for (int k = 0; k < 28; k++) o[k] = 0.0;
        o[0] = slot; o[1] = A->state; o[2] = A->count;
        o[3] = e->space.shapes[A->sa].body; o[4] = e->space.shapes[A->sb].body;
        o[5] = A->n.x; o[6] = A->n.y; o[7] = A->u;
        hash[2 * i] = hash[2 * i + 1] = 0;
        for (int k = 0; k < A->count; k++) {
            const OContact *c = &A->con[k];
            double *q = o + 8 + 10 * k;
            q[0] = c->r1.x; q[1] = c->r1.y; q[2] = c->r2.x; q[3] = c->r2.y; q[4] = c->jnAcc; q[5] = c->jtAcc;
            q[6] = c->nMass; q[7] = c->tMass; q[8] = c->bias; q[9] = c->jBias;
            hash[2 * i + k] = c->hash;
        }
    }
    return n;
}

/* pymunk Body.angle / Body.position setters on body b (as geom.pm_shift_bodies applies them),
 * shapes reindexed: parity tests move blocks to chosen poses before a step */
void oenv_get_target(const OEnv *e, double out[4]) {
    out[0] = e->target_type_id; out[1] = e->target_colour_id; out[2] = e->target_pos.x; out[3] = e->target_pos.y;
}

void oenv_set_body_pose(OEnv *e, int b, double x, double y, double a) {
    ophys_body_set_angle(&e->space, b, a);
    vec2 p = {x, y};
    ophys_body_set_position(&e->space, b, p);
    for (int k = 0; k < e->space.nshapes; k++)
        if (e->space.shapes[k].body == b) ophys_shape_update(&e->space, k);
}

int oenv_get_entities(const OEnv *e, int *kinds, int *types, int *colours, double *poses) {
    for (int i = 0; i < e->nents; i++) {
        const OEntity *en = &e->ents[i];
        kinds[i] = en->kind; types[i] = en->type; colours[i] = en->colour;
        double x = 0, y = 0, a = 0;
        if (en->kind == ENT_GOAL) { /* the sensor body's current position (centre), h, w */
            x = e->space.shapes[en->shape0].sp.x; y = e->space.shapes[en->shape0].sp.y;
            poses[4 * i + 2] = en->gh; poses[4 * i + 3] = en->gw;
        }
        else if (en->nbodies > 0) {
            x = e->space.bodies[en->body0].p.x; y = e->space.bodies[en->body0].p.y; a = e->space.bodies[en->body0].a;
            poses[4 * i + 3] = 0;
        }
        poses[4 * i + 0] = x; poses[4 * i + 1] = y;
        if (en->kind != ENT_GOAL) poses[4 * i + 2] = a;
    }
    return e->nents;
}

double oenv_last_score(const OEnv *e) { return e->last_score; }

void oenv_get_phys_vars(const OEnv *e, double out[5]) {
    for (int i = 0; i < 5; i++) out[i] = e->pv[i];
}

void o_palette(uint8_t out[5][4][3]) { memcpy(out, O_PALETTE, sizeof(O_PALETTE)); }

void o_downsample(const uint8_t *frame384, uint8_t *out96) { oraster_downsample(frame384, out96); }

int oenv_placement_retries(const OEnv *e) { return e->placement_retries; }
void oenv_set_max_tries(OEnv *e, int n) { e->max_tries = n > 0 ? n : 10000; }
