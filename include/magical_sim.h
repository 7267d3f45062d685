/*
 * magical_sim.h -- C ABI of the MI355X batched MAGICAL simulator.
 *
 * Drop-in boundary for the reference hot path:
 * one mg_sim holds N environment instances of one registered MAGICAL env name
 * (benchmarks/__init__.py:427-1102) on one GPU.  mg_step replaces, for all N
 * instances at once, the reference's per-env call chain
 *     TimeLimit.step -> ResizeDictObservation / FlattenFrameStack /
 *     EagerDictFrameStack (benchmarks/__init__.py:51-190)
 *       -> BaseEnv.step (base_env.py:267-307)
 *            -> Robot.set_action / Robot.update (entities.py:435-476)
 *            -> pymunk Space.step x 10 (base_env.py:248-255)
 *            -> score_on_end_of_traj (task files)
 *            -> BaseEnv.render (base_env.py:324-343, render.py:385-395)
 * and mg_reset replaces BaseEnv.reset (base_env.py:190-246) + on_reset.
 *
 * Conventions: functions return 0 on success or a negative errno-style code;
 * mg_last_error() returns a thread-local message.  No C++ exception crosses the
 * ABI.  Output buffers are caller-owned device pointers; the library owns its
 * internal state and frees it in mg_destroy.  All work is enqueued on the given
 * HIP stream (hipStream_t passed as void*; NULL = default stream).  One handle
 * per GPU, used from one host thread.
 */
#ifndef MAGICAL_SIM_H
#define MAGICAL_SIM_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mg_sim mg_sim;

typedef struct {
    int32_t task;              /* 0 MoveToRegion 1 MoveToCorner 2 ClusterColour 3 ClusterShape 4 MatchRegions 5 MakeLine 6 FindDupe 7 FixColour 8 PickAndPlace */
    int32_t rand_flags;        /* bit 0 layout minor, 1 layout full, 2 colour, 3 shape type, 4 count, 5 dynamics,
                                  6 debug_reward (dense shaped reward: move_to_corner.py:85-100, pick_and_place.py:108-124) */
    int32_t preproc;           /* 0 none, 1 LoRes4E (also LoResCHW4E / LoResCHW4A: same bytes), 2 LoResStack,
                                  3 LoRes3EA, 4 LoRes4A (benchmarks/__init__.py:269-307) */
    int32_t num_envs;
    int32_t device;            /* HIP device ordinal */
    int32_t max_episode_steps; /* TimeLimit / BaseEnv.max_episode_steps */
    uint32_t base_seed;        /* env i seeded base_seed + i when seeds == NULL */
    int32_t auto_reset;        /* 1: finished episodes reset inside mg_step (VecEnv); 0: gym single-env semantics */
    const uint32_t *seeds;     /* host array [num_envs] or NULL */
    const void *library;       /* host pointer to an mg_library (layout: magical-1_amd/csrc/mg_common.h,
                                  built by magical_amd.tables from the reference formulas) */
    int64_t library_size;      /* sizeof(mg_library), checked */
} mg_config;

typedef struct {
    uint8_t *obs_allo;   /* LoRes4E/4A: u8[N,96,96,3]; LoResStack: u8[N,96,96,12] */
    uint8_t *obs_ego;    /* same shapes as obs_allo */
    uint8_t *obs_past;   /* LoRes4E/4A: u8[N,96,96,12]; NULL otherwise */
    float *reward;       /* f32[N] (eval_score at done, else 0) */
    uint8_t *done;       /* u8[N] */
    double *eval_score;  /* f64[N] (info['eval_score']) */
    double *target;      /* PickAndPlace: f64[N,4] = (target_type, target_colour, target_position x, y)
                            (pick_and_place.py:87-107 observation extras), written at reset; NULL otherwise */
    int32_t frames_only; /* 0: the preprocessor's outputs above.  1 (multi-GPU compact gather, magical_amd.dist):
                            obs_allo / obs_ego receive only the current LoRes frame of each view, u8[N,96,96,3],
                            for every LoRes preprocessor; obs_past is ignored and no frame stack or ring is kept
                            (the receivers rebuild the stacks with mg_restack).  Switching modes needs a reset. */
} mg_buffers;

/* replaces gym.make(name) for N instances (benchmarks/__init__.py:232-266) */
int mg_create(const mg_config *cfg, mg_sim **out);
/* caller-owned output buffers (device pointers) */
int mg_bind_outputs(mg_sim *sim, const mg_buffers *buf);
/* BaseEnv.reset for every env (mask == NULL) or envs with mask[i] != 0 (device u8[N]);
 * writes the LoRes observation of the reset envs */
int mg_reset(mg_sim *sim, const uint8_t *mask_dev, void *stream);
/* BaseEnv.step for all envs; actions: device u8[N] in [0, 18); envs that reach
 * max_episode_steps report done/reward/eval_score and are reset in place
 * (their observation is the first frame of the next episode) */
int mg_step(mg_sim *sim, const uint8_t *actions_dev, void *stream);
/* BaseEnv.render('rgb_array') of every env: device u8[N,2,384,384,3] (allo, ego) */
int mg_render_full(mg_sim *sim, uint8_t *out_dev, void *stream);
/* parity dumps: per env per body slot (px, py, angle, vx, vy, w): device f64[N,16,6];
 * counts: device i32[N,4] = (bodies, shapes, constraints, active arbiters) */
int mg_get_bodies(mg_sim *sim, double *out_dev, int32_t *counts_dev, void *stream);
/* parity dumps of the contact solver's state (cpArbiter / cpContact): the solved
 * arbiters of every env in active order, out_dev f64[N,48,28] = (slot, state, count, body a, body b, n.x, n.y,
 * friction u, then per contact r1.x, r1.y, r2.x, r2.y, jnAcc, jtAcc, nMass, tMass, bias, jBias), hash_dev
 * u64[N,48,2] = the contacts' feature hashes; rows past the env's active count are zero.  Test hook of the
 * parity suite (the reference has no such call: pymunk exposes the same data as Arbiter.contact_point_set) */
int mg_get_arbiters(mg_sim *sim, double *out_dev, uint64_t *hash_dev, void *stream);
/* set body `body` of env `env` to (x, y, angle) like pymunk's Body.position / Body.angle setters
 * (geom.py:362-384 pm_shift_bodies applies them); for parity tests that place blocks before a step */
int mg_set_body_pose(mg_sim *sim, int env, int body, double x, double y, double angle, void *stream);
/* per-env error flags, device i32[N]: 1 arbiter table full, 2 PlacementError in the env's latest reset
 * (geom.py:335-336; cleared by the next reset, which draws a new layout), 64 PlacementError in any reset so
 * far (sticky), 4 / 8 allo / ego raster assumption or capacity, 16 / 32 scene outside the step kernel's
 * compiled caps / constraint list */
int mg_get_errors(mg_sim *sim, int32_t *out_dev, void *stream);
/* re-seed env RNGs (env.seed): host u32[num_envs].  The many-block tasks' next-layout shadow (layouts drawn
 * ahead on an internal stream) is invalidated: auto-resets run in place on the caller's stream until the next
 * full (mask == NULL) mg_reset re-primes it -- same results, slower resets. */
int mg_seed(mg_sim *sim, const uint32_t *seeds_host);
/* device-side uniform random actions for throughput runs (Philox 4x32-10, key, counter = (step, env)) */
int mg_random_actions(mg_sim *sim, uint8_t *actions_dev, uint64_t key, uint64_t step, void *stream);
int mg_num_envs(const mg_sim *sim);
/* the step kernel this handle launches (diagnostics for bench.py's byte model): out i32[6] = (form: 0 HBM state,
 * 4 cooperative, 5 / 6 robot-scene quad forms; envs per workgroup; the per-env slot caps its HBM <-> LDS transfer
 * moves: bodies, shapes, constraints, arbiter slots) */
int mg_step_form(const mg_sim *sim, int32_t *out);
/* self-test of the device's correctly rounded sin/cos (the physics and render transforms use it):
 * device f64 x[n] -> sin, cos */
int mg_selftest_sincos(const double *x_dev, double *sin_dev, double *cos_dev, int n, void *stream);
/* per-kernel timing of the next max_steps mg_step calls (hipEvents on the launch stream); 0 disables */
int mg_enable_timing(mg_sim *sim, int max_steps);
/* out[0] = total ms in the physics/step kernel, out[1] = total ms in the render kernel,
 * out[2] = number of mg_step calls timed, out[3] = total ms in the auto-reset kernel; resets the counters */
int mg_read_timing(mg_sim *sim, double *out);
/* overwrite every env's episode step counter (BaseEnv.episode_steps, base_env.py:279-283) from device
 * i32[N]: throughput runs stagger episode phases so resets are spread over the timed steps */
int mg_set_episode_steps(mg_sim *sim, const int32_t *steps_dev, void *stream);
/* Demo replay through the LoRes observation stages (replaces saved_trajectories.py:63-149,
 * _MockDemoEnv + preprocess_demos_with_wrapper, for the LoRes preprocessors of
 * benchmarks/__init__.py:232-307).  frames: device u8[nframes,2,384,384,3] (allo, ego) of one or more
 * trajectories concatenated, 16-byte aligned; episode_start: device i32[nframes], the index of the
 * first frame of each frame's trajectory (its reset observation fills the frame stacks);
 * preproc: 1 LoRes4E (CHW4E/CHW4A: same bytes, channels-first views on the host), 2 LoResStack,
 * 3 LoRes3EA, 4 LoRes4A; scratch: device u8[nframes,2,96,96,3] workspace; outputs as mg_buffers for
 * nframes "envs" (out_past NULL for LoResStack).  No mg_sim needed. */
int mg_replay_lores(const uint8_t *frames, int32_t nframes, const int32_t *episode_start, int32_t preproc,
                    uint8_t *scratch, uint8_t *out_allo, uint8_t *out_ego, uint8_t *out_past, void *stream);
/* Receiver side of the compact multi-GPU gather (magical_amd.dist.ShardedVecEnv): rebuilds the LoRes frame
 * stacks (FlattenFrameStack / EagerDictFrameStack, benchmarks/__init__.py:51-147, reset frame filling every
 * slot) of world * n envs from their all-gathered current frames.
 * recv: device u8, `world` rank blocks of rank_stride bytes; block r holds env r*n+i's current allo frame
 * u8[96,96,3] at off_allo + i*27648, its ego frame at off_ego + i*27648 and its done flag u8 at off_done + i
 * (all offsets 16-byte aligned, as the frames-only outputs of mg_bind_outputs write them).
 * ring: device u8[stacks][4][world*n][27648], stacks = 2 for LoResStack (allo, ego), else 1 (the view the
 * stacked output is built from), caller-owned and persistent across calls (step t writes slot t % 4).
 * all_fresh = 1 after a reset of every env; otherwise an env whose done flag is set restarts its stacks
 * (auto-reset: its frame is the next episode's first).  Outputs for world*n envs, as mg_buffers' stacked
 * outputs: preproc 1 (LoRes4E / CHW4E / CHW4A), 3 (LoRes3EA), 4 (LoRes4A): out_past u8[world*n,96,96,12]
 * (allo / ego are the gathered frames themselves); 2 (LoResStack): out_allo, out_ego u8[world*n,96,96,12]. */
int mg_restack(const uint8_t *recv, int32_t world, int32_t n, int64_t rank_stride, int64_t off_allo, int64_t off_ego,
               int64_t off_done, int32_t preproc, int64_t step, int32_t all_fresh, uint8_t *ring, uint8_t *out_allo,
               uint8_t *out_ego, uint8_t *out_past, void *stream);
/* The same stacks as a window ring (round 5): every received frame is written once, channel-planar
 * (u8[3][96][96]), into ring u8[stacks][world*n][K + 3][3][96][96] (stacks as for mg_restack; caller-owned,
 * persistent; K >= 4): frame t of env g goes to slot t % K, and also to slot K + t % K when t % K < 3, so for
 * every env the frames t-3 .. t (oldest first) occupy the consecutive slots s0 .. s0 + 3, s0 = (t + K - 3) % K.
 * The stacked output of step t is then the strided view [world*n, 96, 96, 12] of the ring at byte offset
 * s0 * 27648 with strides (env (K + 3) * 27648, y 96, x 1, channel 9216) -- channel k of a stack = plane k % 3
 * of its frame k / 3 -- identical to mg_restack's outputs value for value, with no stack written.  A fresh env
 * (all_fresh, or its done flag) writes its frame into the slots of frames t-3 .. t.  preproc 1 (LoRes4E /
 * CHW4E / CHW4A), 2 (LoResStack), 4 (LoRes4A); LoRes3EA (allo frame in front of 3 ego frames) is not a window
 * of one ring: use mg_restack.  Step t's views stay valid until the call for step t + 1 is ordered after
 * their readers (the ring's slot t + 1 - K ... is rewritten then; for a fresh env the slots of t-3 .. t). */
int mg_restack_window(const uint8_t *recv, int32_t world, int32_t n, int64_t rank_stride, int64_t off_allo,
                      int64_t off_ego, int64_t off_done, int32_t preproc, int64_t step, int32_t all_fresh, int32_t K,
                      uint8_t *ring, void *stream);
/* Stacked outputs as window rings on the simulator itself (round 5).  ring_allo / ring_ego: device
 * u8[num_envs][K + 3][3][96][96], caller-owned, 16-byte aligned, one for each stacked view of the preprocessor
 * (LoResStack: allo and ego; LoRes4E / CHW4E / CHW4A: ego; LoRes4A: allo), NULL for the others; both NULL
 * turns it off.  Each step's frame of a stacked view is written once, channel-planar, into slot w % K (and
 * K + w % K when w % K < 3; w = the number of mg_step calls so far), a freshly reset env into the slots of
 * frames w-3 .. w, instead of the [96][96][12] stack and its frame ring: the stack is the strided view of the
 * ring at slot mg_window_start() with strides (env (K + 3) * 27648, y 96, x 1, channel 9216), value for value
 * the stack mg_bind_outputs would receive (FlattenFrameStack / EagerDictFrameStack, benchmarks/__init__.py:
 * 51-147).  The stacked outputs of mg_bind_outputs may then be NULL.  Bind before mg_reset; not with
 * frames_only outputs.  A step's views stay valid until the next mg_step / mg_reset on the stream. */
int mg_bind_window(mg_sim *sim, uint8_t *ring_allo, uint8_t *ring_ego, int32_t K);
/* *slot = the window's first slot for the current outputs ((w + K - 3) % K), -1 when no ring is bound */
int mg_window_start(const mg_sim *sim, int32_t *slot);
void mg_destroy(mg_sim *sim);
const char *mg_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
