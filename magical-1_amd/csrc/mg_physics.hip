// mg_physics.hip -- step-kernel dispatch: the compiled form for a scene's slot caps (5/6: compile-time
// constraint lists with 4 lanes per env, 4: cooperative LDS view with runtime lists, one env per wavefront,
// 0: HBM state for scenes beyond the LDS caps) and envs per workgroup.  The forms live in mg_step_*.hip (one
// translation unit each).  The one-lane forms 1/2/3 that 5/6/4 superseded were deleted in round 5 (their A/B
// results are in DESIGN.md); variants 1/2/3 survive only as the slot caps mg_step_variant matches.
#include "mg_launch.h"
#include "mg_phys.h"   // sizeof(ShapeW) of the LDS views

hipError_t mg_prof_read_step_quad(unsigned long long *out64);   // mg_step_quad.hip

// LDS bytes of one env's view (same carve order as carve_view, per-lane columns)
size_t mg_step_lds_bytes(const StepCaps &c, int blk) {
    size_t off = 0;
    auto take = [&](size_t count, size_t size) { off = (off + 15) & ~(size_t)15; off += count * size; };
    const size_t B = (size_t)c.nb * blk, SH = (size_t)c.ns * blk, C = (size_t)c.nc * blk, A = (size_t)c.na * blk;
    for (int i = 0; i < 14; i++) take(B, 8);
    for (int i = 0; i < 6; i++) take(SH, 8);
    take((size_t)CP_NUM * C, 8);
    for (int i = 0; i < 3; i++) take(A, 8);
    take((size_t)2 * AC_NUM * A, 8); take(2 * A, 8);
    for (int i = 0; i < 4; i++) take(blk, 8);
    take(A, 4); take(A, 4);
    for (int i = 0; i < 8; i++) take(blk, 4);
    take(SH, 2); take(SH, 2); take(SH, 1); take(SH, 1);
    for (int i = 0; i < 3; i++) take(C, 1);
    for (int i = 0; i < 5; i++) take(A, 1);
    take((size_t)c.shw * blk, sizeof(ShapeW));
    return (off + 15) & ~(size_t)15;
}


int mg_step_variant(const StepCaps &c, int n_envs) {
    (void)n_envs;
    for (int v = 1; v <= 2; v++) {
        const StepCaps k = step_variant_caps(v);
        if (c.nb == k.nb && c.ns == k.ns && c.nc == k.nc && c.na == k.na) return v;
    }
    // runtime constraint lists: any scene within the caps (arbiter slots must match exactly: the HBM
    // slots beyond the task's cap are never initialised)
    const StepCaps k = step_variant_caps(3);
    if (c.nb <= k.nb && c.ns <= k.ns && c.nc <= k.nc && c.na == k.na) return 3;
    return 0;
}

// envs per workgroup: compiled sizes only
bool mg_step_blk_ok(int variant, int blk) {
    return variant == 0 ? (blk == 1 || blk == 8 || blk == 64)
         : variant == 4 ? blk == 1
         : variant == 5 ? (blk == 16 || blk == 8)     // 8: grids below 16 envs per CU (mg_sim.hip pick_step_blk)
         : variant == 6 ? (blk == 16 || blk == 8)     // (4 envs per workgroup, 16 lanes per env: removed in round 6,
                                                      // profiles/r06_blk4)
         : false;
}

hipError_t mg_launch_step(const MGState &S, const mg_library *L, TaskCfg cfg, int variant, int blk, int max_steps,
                          int auto_reset, const uint8_t *actions, float *reward, uint8_t *done, double *eval_score,
                          uint8_t *reset_mask, hipStream_t st) {
#define MG_STEP_CASE(V, B) \
    if (variant == V && blk == B) \
        return launch_step_var<V, B>(S, L, cfg, max_steps, auto_reset, actions, reward, done, eval_score, reset_mask, st);
    MG_STEP_CASE(4, 1)
    MG_STEP_CASE(5, 16) MG_STEP_CASE(5, 8) MG_STEP_CASE(6, 16) MG_STEP_CASE(6, 8)
    MG_STEP_CASE(0, 1) MG_STEP_CASE(0, 8) MG_STEP_CASE(0, 64)
#undef MG_STEP_CASE
    return hipErrorInvalidValue;
}

hipError_t mg_prof_read_physics(unsigned long long *out) {
    hipError_t e;
    if ((e = mg_prof_read_reset(out)) != hipSuccess) return e;
    if ((e = mg_prof_read_step_v4(out)) != hipSuccess) return e;
    if ((e = mg_prof_read_step_quad(out)) != hipSuccess) return e;
    return mg_prof_read_step_hbm(out);
}
