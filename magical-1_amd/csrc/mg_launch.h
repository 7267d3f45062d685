// mg_launch.h -- host-side launchers of the device kernels (one translation unit
// per kernel family: mg_physics.hip, mg_raster.hip; the C ABI lives in mg_sim.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "mg_state.h"

// coop: one env per 64-lane wave (reset_kernel_coop); fused_reset: the step kernel runs the auto-reset of its
// done envs itself (robot scenes without layout randomisation, mg_step)
struct TaskCfg { int task, flags, coop, fused_reset; };

struct RenderOut {
    uint8_t *full;        // [N][2][384][384][3] (full-resolution mode) or null
    uint8_t *obs_allo;    // LoRes outputs (layout per preproc), or null
    uint8_t *obs_ego;
    uint8_t *obs_past;
    const uint8_t *mask;  // reset mask: envs with mask[e] == 0 are left untouched (null: all)
    int preproc;
    int frames_only;      // 1: obs_allo / obs_ego get the current [N][96][96][3] frames only (no stacks, no ring)
    int debug_skip;      // profiling builds only: 1 skip outlines, 2 skip fill, 4 skip HBM stores, 8 skip spans
    int small;            // 1: robot + arena + goal + one block at most (MoveToRegion, MoveToCorner) -> small LDS class
    int retry_in;         // set by mg_launch_render: class chain, render only the pairs at this class's level
                          // (S.rg_retry: the level that holds each (env, view) this episode)
    int retry_out;        // ... a pair this class cannot hold moves to the next level (else an env error)
    int cls_level;        // ... position of this class in the chain
    int first_level;      // ... the chain's first class for this task (0: medium-0, 1: medium-1)
    int force_retry;      // tests: classes below this level hand every pair on (1: skip the first, 2: the first two)
    int scache_mode;      // tests / A-B (MG_DEBUG_SCACHE): 1 = no allocentric static layer, 2 = its copied blocks
                          // poisoned (0x55) -- shows where the layer is used
    // window rings (mg_bind_window): a stacked view writes its current frame channel-planar into
    // wring[view] u8[N][wK + 3][3][96][96] (slot wpos = step % wK, and wK + wpos when wpos < 3; a fresh env the
    // slots of frames step-3 .. step) instead of its [96][96][12] stack and frame ring; null: the stack as before
    uint8_t *wring[2];
    int wK, wpos;
    int wnsl[2];              // window slots of this step's frame: [0] a running env (wpos, and wK + wpos when
    int8_t wsl[2][8];         // wpos < 3), [1] a fresh env (the slots of frames step-3 .. step, with duplicates)
};

hipError_t mg_launch_seed(const MGState &S, const uint32_t *seeds_dev, hipStream_t st);
// max_waves > 0 (masked launches only): at most that many wavefronts, each resetting the masked envs of its
// grid-stride range in turn; 0: one wavefront per env
hipError_t mg_launch_reset(const MGState &S, const mg_library *L, TaskCfg cfg, const uint8_t *mask, hipStream_t st,
                           int max_waves = 0);
// LDS-resident substeps: per-env slot caps of a task and envs per workgroup
struct StepCaps { int nb, ns, nc, na, blk, shw; };  // shw: world-space shape scratch per lane in LDS
size_t mg_step_lds_bytes(const StepCaps &c, int blk);
// compiled LDS variant matching these caps for n_envs (0: the HBM-state kernel)
int mg_step_variant(const StepCaps &c, int n_envs);
// compiled envs-per-workgroup sizes of a variant
bool mg_step_blk_ok(int variant, int blk);
// Slot caps of the LDS-resident variants (compile-time, so every LDS address folds to a constant
// offset from the lane's column): 0 = state stays in HBM.
__host__ __device__ constexpr StepCaps step_variant_caps(int v) {
    return v == 1 ? StepCaps{6, 5, 10, 20, 16, 3}    // robot only (MoveToRegion)
         : v == 2 ? StepCaps{7, 6, 12, 32, 16, 0}    // robot + one single-shape block (MoveToCorner; no LDS left for shapes)
         : v == 3 ? StepCaps{14, 53, 26, 48, 1, 0}   // up to 8 blocks incl. stars (Cluster*, MatchRegions): runtime lists
         : v == 4 ? StepCaps{14, 53, 26, 48, 1, 0}   // the same scenes, one env per 64-lane wavefront (cooperative)
         : StepCaps{0, 0, 0, 0, 0, 0};
}

// one compiled step-kernel form (defined in mg_stepk.h, instantiated in mg_step_*.hip)
template <int VAR, int BLK>
hipError_t launch_step_var(const MGState &S, const mg_library *L, TaskCfg cfg, int max_steps, int auto_reset,
                           const uint8_t *actions, float *reward, uint8_t *done, double *eval_score,
                           uint8_t *reset_mask, hipStream_t st);
hipError_t mg_launch_step(const MGState &S, const mg_library *L, TaskCfg cfg, int variant, int blk, int max_steps,
                          int auto_reset, const uint8_t *actions, float *reward, uint8_t *done, double *eval_score,
                          uint8_t *reset_mask, hipStream_t st);
hipError_t mg_launch_render(const MGState &S, const mg_library *L, const RenderOut &ro, int mode, hipStream_t st);
hipError_t mg_launch_compose3ea(const MGState &S, const uint8_t *obs_allo, const uint8_t *mask, uint8_t *obs_past,
                                hipStream_t st);
// profiling builds (-DMG_PROFILE): copy and clear each translation unit's phase timers
hipError_t mg_prof_read_physics(unsigned long long *out64);
hipError_t mg_prof_read_reset(unsigned long long *out64);
hipError_t mg_prof_read_step_v4(unsigned long long *out64);
hipError_t mg_prof_read_step_hbm(unsigned long long *out64);
hipError_t mg_prof_read_raster(unsigned long long *out64);
