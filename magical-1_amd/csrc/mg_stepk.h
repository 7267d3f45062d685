// mg_stepk.h -- the step kernel template (action decode, 10 x [Robot.update + cpSpaceStep], episode
// counter, score) and its launcher.  Each form is instantiated in its own translation unit
// (mg_step_quad.hip: 5 / 6, mg_step_v4.hip: 4, mg_step_hbm.hip: 0) so they compile in parallel;
// mg_physics.hip dispatches.
#pragma once
#include <cstdio>
#include "mg_launch.h"
#include "mg_step.h"
#include "mg_stepq.h"
#include "mg_score.h"
#include "mg_reset.h"

// slot caps of every compiled form: the LDS variants of mg_launch.h, plus the QL-lanes-per-env forms of the
// compile-time scenes (5: the caps of 1 with two world-shape slots per lane in LDS -- 2 x 64 per workgroup,
// so 128 / blk per env; 6: the caps of 2, world shapes in per-lane locals as there)
// Form 5's narrowphase operands (two ShapeW per lane) in LDS (1, rounds 2-5) or per-lane locals (0, round 6, as
// form 6).  The LDS slots were 51 of the 8-env workgroup's 78 KB; without them the step workgroup takes 27 KB, so
// more of the other chunk's render workgroups co-run beside it: step kernel 0.400 -> 0.415 ms alone, 0.61 -> 0.52 ms
// co-running, MoveToRegion 3.04 -> 3.16 M env-steps/s (profiles/r06_q5)
#ifndef MG_Q5_LDS_SHAPES
#define MG_Q5_LDS_SHAPES 0
#endif
__host__ __device__ constexpr StepCaps step_form_caps(int v, int blk) {
    return v == 5 ? StepCaps{6, 5, 10, 20, 16, MG_Q5_LDS_SHAPES ? 128 / blk : 0}
         : v == 6 ? StepCaps{7, 6, 12, 32, 16, 0} : step_variant_caps(v);
}

// ---- LDS-resident substeps ------------------------------------------------
// The 10 substeps of an env-step touch only the env's bodies, shapes,
// constraints, arbiters and a few scalars.  They are copied once per env-step
// from HBM ([slot][N] arrays) into LDS ([slot][BLK] arrays, one column per lane)
// and the MGState "view" V points there with V.N = BLK and e = lane, so the same
// device code runs against LDS; everything is copied back before scoring and
// the in-place reset (which use the HBM state).  A lane only touches its own
// column, so no barrier is needed.
template <typename T>
__device__ __forceinline__ T *carve(unsigned char *base, size_t &off, size_t count) {
    off = (off + 15) & ~(size_t)15;
    T *p = (T *)(base + off);
    off += count * sizeof(T);
    return p;
}

__device__ __forceinline__ void carve_view(MGState &V, unsigned char *smem, const StepCaps &c, int blk) {
    size_t off = 0;
    const size_t B = (size_t)c.nb * blk, SH = (size_t)c.ns * blk, C = (size_t)c.nc * blk, A = (size_t)c.na * blk;
    V.bpx = carve<double>(smem, off, B); V.bpy = carve<double>(smem, off, B); V.bvx = carve<double>(smem, off, B);
    V.bvy = carve<double>(smem, off, B); V.ba = carve<double>(smem, off, B); V.bw = carve<double>(smem, off, B);
    V.bvbx = carve<double>(smem, off, B); V.bvby = carve<double>(smem, off, B); V.bwb = carve<double>(smem, off, B);
    V.brc = carve<double>(smem, off, B); V.brs = carve<double>(smem, off, B); V.bminv = carve<double>(smem, off, B);
    V.biinv = carve<double>(smem, off, B); V.bacache = carve<double>(smem, off, B);
    V.sr = carve<double>(smem, off, SH); V.su = carve<double>(smem, off, SH); V.sbbl = carve<double>(smem, off, SH);
    V.sbbb = carve<double>(smem, off, SH); V.sbbr = carve<double>(smem, off, SH); V.sbbt = carve<double>(smem, off, SH);
    V.cp = carve<double>(smem, off, (size_t)CP_NUM * C);
    V.anx = carve<double>(smem, off, A); V.any = carve<double>(smem, off, A); V.au = carve<double>(smem, off, A);
    V.acon = carve<double>(smem, off, (size_t)2 * AC_NUM * A); V.ahash = carve<uint64_t>(smem, off, 2 * A);
    V.curr_dt = carve<double>(smem, off, blk); V.target_speed = carve<double>(smem, off, blk);
    V.rel_turn = carve<double>(smem, off, blk); V.target_finger = carve<double>(smem, off, blk);
    V.akey = carve<int32_t>(smem, off, A); V.astamp = carve<uint32_t>(smem, off, A);
    V.nbodies = carve<int32_t>(smem, off, blk); V.nshapes = carve<int32_t>(smem, off, blk);
    V.ncons = carve<int32_t>(smem, off, blk); V.nactive = carve<int32_t>(smem, off, blk);
    V.stamp = carve<uint32_t>(smem, off, blk); V.overflow = carve<int32_t>(smem, off, blk);
    V.robot_body0 = carve<int32_t>(smem, off, blk); V.robot_cons0 = carve<int32_t>(smem, off, blk);
    V.sgroup = carve<int16_t>(smem, off, SH); V.shash = carve<int16_t>(smem, off, SH);
    V.sbody = carve<int8_t>(smem, off, SH); V.spoly = carve<int8_t>(smem, off, SH);
    V.ctype = carve<int8_t>(smem, off, C); V.ca = carve<int8_t>(smem, off, C); V.cb = carve<int8_t>(smem, off, C);
    V.astate = carve<int8_t>(smem, off, A); V.acount = carve<int8_t>(smem, off, A); V.asa = carve<int8_t>(smem, off, A);
    V.asb = carve<int8_t>(smem, off, A); V.active = carve<int8_t>(smem, off, A);
    V.shw = c.shw ? carve<ShapeW>(smem, off, (size_t)c.shw * blk) : nullptr;
    V.N = blk;
    V.cons_cap = c.nc;
    V.arb_cap = c.na;
}

// rows [0, rows) of a [row][N] HBM array <-> [row][BLK] LDS array (lane's column); for the
// cp / acon / ahash blocks the HBM row of LDS row (k, r) is k * hcap + r
template <typename T>
__device__ __forceinline__ void xfer(T *lds, T *hbm, int rows, int blk, int lane, int N, int e, bool to_lds,
                                     int r0 = 0, int rs = 1, int groups = 1, int lcap = 0, int hcap = 0) {
#pragma unroll 1
    for (int g = 0; g < groups; g++)
#pragma unroll 2
        for (int r = r0; r < rows; r += rs) {
            const uint32_t li = (uint32_t)(g * lcap + r) * blk + lane, hi = (uint32_t)(g * hcap + r) * N + e;
            if (to_lds) lds[li] = hbm[hi]; else hbm[hi] = lds[li];
        }
}

// The cooperative form's transfer (one env per wavefront: rows r0 = lane, step 64, so each array is at most one
// row per lane) with runtime loops: the compile-time form below raised its VGPRs 248 -> 276 (one wavefront per SIMD
// instead of two), round 5.  HBM <-> LDS view transfer of what the substeps read (in) / what later env-steps need (out):
// bodies (incl. bias velocities and the rotation cache), the constraints' parameters and
// warm-start impulses, the live arbiters (key, contacts, warm-start hashes) and the active list.
// Cached shape BBs and the constraints' pre-step products are recomputed before use.
// (r0, rs): rows r0, r0 + rs, ... of every array (rs = 64, r0 = lane: the cooperative form, one env per
// wavefront, each lane a share of the rows)
__device__ __forceinline__ void xfer_state(const MGState &S, const MGState &V, const StepCaps &c, int lane, int e,
                                           bool in, bool cons_list = false, int r0 = 0, int rs = 1) {
    const int blk = V.N, N = S.N;
#define XF(f, rows) xfer(V.f, S.f, rows, blk, lane, N, e, in, r0, rs)
#define XS(f, r) do { if (in) V.f[(uint32_t)(r) * blk + lane] = S.f[(uint32_t)(r) * N + e]; \
                      else S.f[(uint32_t)(r) * N + e] = V.f[(uint32_t)(r) * blk + lane]; } while (0)
    XF(bpx, c.nb); XF(bpy, c.nb); XF(bvx, c.nb); XF(bvy, c.nb); XF(ba, c.nb); XF(bw, c.nb); XF(bvbx, c.nb);
    XF(bvby, c.nb); XF(bwb, c.nb); XF(brc, c.nb); XF(brs, c.nb); XF(bacache, c.nb);
    // constraint parameter slots: in = MAXF, MAXB, BCOEF, JACC, JACC2, type parameters 8-11; out = JACC, JACC2
#pragma unroll 1
    for (int k = 0; k < CP_NUM; k++) {
        const bool need = in ? (k <= CP_JACC2 || (k >= 8 && k <= 11)) : (k == CP_JACC || k == CP_JACC2);
        if (!need) continue;
#pragma unroll 2
        for (int r = r0; r < c.nc; r += rs) {
            const uint32_t li = (uint32_t)(k * c.nc + r) * blk + lane, hi = (uint32_t)(k * MG_MAX_CONS + r) * N + e;
            if (in) V.cp[li] = S.cp[hi]; else S.cp[hi] = V.cp[li];
        }
    }
#pragma unroll 1
    for (int r = r0; r < c.na; r += rs) { // arbiter slots: only live ones carry data
        XS(akey, r);
        const int key = in ? V.akey[(uint32_t)r * blk + lane] : V.akey[(uint32_t)r * blk + lane];
        if (key < 0) continue;
        XS(anx, r); XS(any, r); XS(au, r); XS(astamp, r); XS(astate, r); XS(acount, r); XS(asa, r); XS(asb, r);
#pragma unroll 1
        for (int f = 0; f < 2 * AC_NUM; f++) {
            if (in) V.acon[(uint32_t)(f * c.na + r) * blk + lane] = S.acon[(uint32_t)(f * MG_MAX_ARB + r) * N + e];
            else S.acon[(uint32_t)(f * MG_MAX_ARB + r) * N + e] = V.acon[(uint32_t)(f * c.na + r) * blk + lane];
        }
        for (int k = 0; k < 2; k++) {
            if (in) V.ahash[(uint32_t)(k * c.na + r) * blk + lane] = S.ahash[(uint32_t)(k * MG_MAX_ARB + r) * N + e];
            else S.ahash[(uint32_t)(k * MG_MAX_ARB + r) * N + e] = V.ahash[(uint32_t)(k * c.na + r) * blk + lane];
        }
    }
    XF(nactive, 1);
    const int nact = in ? S.nactive[e] : V.nactive[lane];
#pragma unroll 1
    for (int r = r0; r < nact; r += rs) XS(active, r);
    XF(curr_dt, 1); XF(stamp, 1); XF(overflow, 1);
    if (in) { // read-only during the substeps
        XF(target_speed, 1); XF(rel_turn, 1); XF(target_finger, 1);
        XF(bminv, c.nb); XF(biinv, c.nb);
        XF(sr, c.ns); XF(su, c.ns); XF(sgroup, c.ns); XF(shash, c.ns); XF(sbody, c.ns); XF(spoly, c.ns);
        XF(nbodies, 1); XF(nshapes, 1); XF(ncons, 1); XF(robot_body0, 1); XF(robot_cons0, 1);
        if (cons_list) { XF(ctype, c.nc); XF(ca, c.nc); XF(cb, c.nc); } // runtime constraint list
    }
#undef XS
#undef XF
}

// HBM <-> LDS view transfer of what the substeps read (in) / what later env-steps need (out): bodies (incl. bias
// velocities and the rotation cache), the constraints' parameters and warm-start impulses, the live arbiters
// (key, contacts, warm-start hashes) and the active list; cached shape BBs and the constraints' pre-step products
// are recomputed before use.  Rows sub, sub + QL, ... of every [row][N] HBM array <-> the [row][BLK] LDS array's
// column `lane`.  The slot caps are compile-time, so every loop has a constant trip count and no branch (rows
// past the cap repeat the last row: the same value loaded and stored twice) and each array's loads are in
// flight together instead of one HBM round trip per row (round 5: the `in` transfer was ~15% of the robot
// scenes' step kernel as a chain of dependent HBM latencies).  Live arbiters' contact rows likewise in one
// block per slot.
template <int ROWS, int QL, typename T>
MG_DEV void xq(T *lds, T *hbm, int blk, int lane, int N, int e, int sub, bool in, int lrow0 = 0, int hrow0 = 0) {
#pragma unroll
    for (int k = 0; k < (ROWS + QL - 1) / QL; k++) {
        const int r = sub + k * QL < ROWS ? sub + k * QL : ROWS - 1;
        const uint32_t li = (uint32_t)(lrow0 + r) * blk + lane, hi = (uint32_t)(hrow0 + r) * N + e;
        if (in) lds[li] = hbm[hi]; else hbm[hi] = lds[li];
    }
}

// (QL = 64, lane = 0, sub = the thread: the cooperative form, one env per wavefront; CONS: its runtime constraint
// list is transferred too)
template <int NB, int NS, int NC, int NA, int QL, bool CONS = false>
__device__ __forceinline__ void xfer_state_quad(const MGState &S, const MGState &V, int lane, int e, int sub, bool in) {
    const int blk = V.N, N = S.N;
    // groups of a few arrays are scheduled on their own (sched_barrier): their loads are in flight together,
    // but the whole transfer is not hoisted into one block (that held ~200 VGPRs of loaded values and made
    // the kernel spill)
#define XQ(f, rows) xq<rows, QL>(V.f, S.f, blk, lane, N, e, sub, in)
#define XQ_GROUP() __builtin_amdgcn_sched_barrier(0)
    XQ(bpx, NB); XQ(bpy, NB); XQ(bvx, NB); XQ(bvy, NB); XQ_GROUP();
    XQ(ba, NB); XQ(bw, NB); XQ(bvbx, NB); XQ(bvby, NB); XQ_GROUP();
    XQ(bwb, NB); XQ(brc, NB); XQ(brs, NB); XQ(bacache, NB); XQ_GROUP();
    if (in) {   // constraint parameter slots MAXF, MAXB, BCOEF, JACC, JACC2 and the type parameters 8-11
#pragma unroll
        for (int k = 0; k < CP_NUM; k++) {
            if (k <= CP_JACC2 || (k >= 8 && k <= 11)) xq<NC, QL>(V.cp, S.cp, blk, lane, N, e, sub, true, k * NC, k * MG_MAX_CONS);
            if (k == 2 || k == 8 || k == 11) XQ_GROUP();
        }
    } else {    // the warm-start impulses
        xq<NC, QL>(V.cp, S.cp, blk, lane, N, e, sub, false, CP_JACC * NC, CP_JACC * MG_MAX_CONS);
        xq<NC, QL>(V.cp, S.cp, blk, lane, N, e, sub, false, CP_JACC2 * NC, CP_JACC2 * MG_MAX_CONS);
    }
    XQ_GROUP();
    XQ(akey, NA);   // arbiter slots: only live ones carry data
#pragma unroll
    for (int k = 0; k < (NA + QL - 1) / QL; k++) {
        const int r = sub + k * QL;
        if (r >= NA || V.akey[(uint32_t)r * blk + lane] < 0) continue;
#define XA(f) do { if (in) V.f[(uint32_t)r * blk + lane] = S.f[(uint32_t)r * N + e]; \
                   else S.f[(uint32_t)r * N + e] = V.f[(uint32_t)r * blk + lane]; } while (0)
        XA(anx); XA(any); XA(au); XA(astamp); XA(astate); XA(acount); XA(asa); XA(asb);
#pragma unroll
        for (int f = 0; f < 2 * AC_NUM; f++) {
            if (in) V.acon[(uint32_t)(f * NA + r) * blk + lane] = S.acon[(uint32_t)(f * MG_MAX_ARB + r) * N + e];
            else S.acon[(uint32_t)(f * MG_MAX_ARB + r) * N + e] = V.acon[(uint32_t)(f * NA + r) * blk + lane];
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (in) V.ahash[(uint32_t)(h * NA + r) * blk + lane] = S.ahash[(uint32_t)(h * MG_MAX_ARB + r) * N + e];
            else S.ahash[(uint32_t)(h * MG_MAX_ARB + r) * N + e] = V.ahash[(uint32_t)(h * NA + r) * blk + lane];
        }
#undef XA
    }
    if (sub == 0) {
        if (in) V.nactive[lane] = S.nactive[e]; else S.nactive[e] = V.nactive[lane];
    }
    // the active list: its length is read back from this lane's own copy (sub-lane 0 wrote it just above for
    // `in`; the solver lane wrote it before the closing barrier for `out`) -- rows past it are dead
    const int nact = in ? S.nactive[e] : V.nactive[lane];
#pragma unroll
    for (int k = 0; k < (NA + QL - 1) / QL; k++) {
        const int r = sub + k * QL;
        if (r < nact) {
            if (in) V.active[(uint32_t)r * blk + lane] = S.active[(uint32_t)r * N + e];
            else S.active[(uint32_t)r * N + e] = V.active[(uint32_t)r * blk + lane];
        }
    }
    if (sub == 0) {
#define XS1(f) do { if (in) V.f[lane] = S.f[e]; else S.f[e] = V.f[lane]; } while (0)
        XS1(curr_dt); XS1(stamp); XS1(overflow);
        if (in) { XS1(target_speed); XS1(rel_turn); XS1(target_finger); XS1(nbodies); XS1(nshapes); XS1(ncons);
                  XS1(robot_body0); XS1(robot_cons0); }
#undef XS1
    }
    if (in) {   // read-only during the substeps
        XQ(bminv, NB); XQ(biinv, NB); XQ(sr, NS); XQ(su, NS); XQ_GROUP();
        XQ(sgroup, NS); XQ(shash, NS); XQ(sbody, NS); XQ(spoly, NS);
        if constexpr (CONS) { XQ(ctype, NC); XQ(ca, NC); XQ(cb, NC); }
        XQ_GROUP();
    }
#undef XQ_GROUP
#undef XQ
}

// Workgroups are dispatched round-robin over the 8 XCDs (workgroup b -> XCD b % 8); map them so
// that each XCD owns one contiguous range of envs: neighbouring envs share [slot][N] cache lines,
// and with few envs per workgroup those lines are then reused in the XCD's own L2.
__device__ __forceinline__ int xcd_block(int b, int g) {
    const int q = g >> 3, r = g & 7, x = b & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// Robot.set_action + 10 x (Robot.update, cpSpaceStep): base_env.py:248-276 (one lane per env, HBM state)
__device__ __forceinline__ void env_substeps(const MGState &V, const mg_library *L, int ev, int a, MGProf &P) {
    robot_set_action(V, L, ev, a < 18 ? a : 0);
    const double dt = L->dt;
    for (int i = 0; i < 10; i++) {
        robot_update(V, L, ev);
        MG_PP(P, 0);
        space_step(V, L, ev, dt, P);
    }
}

// the same with one env per wavefront: lane 0 drives the robot, every lane takes part in the step
__device__ __forceinline__ void env_substeps_coop(const MGState &V, const mg_library *L, int lane, int a, MGProf &P) {
    if (lane == 0) robot_set_action(V, L, 0, a < 18 ? a : 0);
    const double dt = L->dt;
    __syncthreads();
    const CoopPlan Q = coop_plan(V, lane);
    // robot.update() before every space.step() (base_env.py:248-255), on lane 0 right after the previous
    // substep's closing barrier: space_step_coop reads only its step scalars before its first barrier, and
    // the robot update writes the control body and the finger springs' rates (as mg_stepq.h)
    if (lane == 0) robot_update(V, L, 0);
    for (int i = 0; i < 10; i++) {
        MG_PP(P, 0);
        space_step_coop(V, L, dt, lane, Q, P);   // ends with a workgroup barrier
        if (lane == 0 && i < 9) robot_update(V, L, 0);
    }
}

template <int VAR, int BLK>
__global__ void __launch_bounds__(64) step_kernel(MGState S, const mg_library *__restrict__ L, TaskCfg cfg, int max_steps,
                                                  int auto_reset, const uint8_t *__restrict__ actions, float *reward,
                                                  uint8_t *done, double *eval_score, uint8_t *reset_mask) {
    extern __shared__ __align__(16) unsigned char smem[];
    constexpr StepCaps C = step_form_caps(VAR, BLK);
    static_assert(VAR == 0 || VAR == 4 || VAR == 5 || VAR == 6, "compiled forms: 0 (HBM state), 4 (cooperative), 5 / 6");
    constexpr bool LDS = VAR != 0;
    constexpr bool COOP = VAR == 4;            // one env per workgroup of 64 lanes
    constexpr bool QUAD = VAR == 5 || VAR == 6; // QL lanes per env, BLK envs in one 64-lane workgroup
    constexpr int QL = QUAD ? 64 / BLK : 1;
    constexpr int NCS = VAR == 4 ? 0 : C.nc;   // compile-time constraint list (0: the env's runtime list)
    const int lane = COOP ? (int)threadIdx.x : QUAD ? (int)threadIdx.x / QL : BLK == 1 ? 0 : (int)threadIdx.x;
    const int sub = QUAD ? (int)threadIdx.x % QL : 0;
    int e = xcd_block(blockIdx.x, gridDim.x) * BLK + (COOP ? 0 : lane);
    // QUAD: lanes without an env of their own (past n_envs, or a scene the form cannot hold) still take
    // part in the workgroup barriers as shadows of a valid env; they never write HBM
    bool shadow = false;
    if (e >= S.n_envs) {
        if (!QUAD) return;
        shadow = true;
        e = S.n_envs - 1;
    }
    const int a = actions[e];
    MGProf P;
    MG_PP_INIT(P);
    if constexpr (LDS) {
        bool fits = true;
        if (S.nbodies[e] > C.nb || S.nshapes[e] > C.ns || S.ncons[e] > C.nc) {
            if (!shadow && sub == 0) {
                S.overflow[e] |= 16; // scene larger than the variant's LDS caps (never expected)
                if (reset_mask) reset_mask[e] = 0;
            }
            if (!QUAD) return;
            fits = false;
        }
        bool ok = NCS == 0 || (S.ncons[e] == C.nc && S.robot_body0[e] == 0 && S.robot_cons0[e] == 0);
        for (int c = 0; c < NCS; c++) {
            const ConsDesc d = static_cons(c);
            ok = ok && AT(S.ctype, c) == d.type && AT(S.ca, c) == d.a && AT(S.cb, c) == d.b;
        }
        for (int k = 0; k < S.nshapes[e] && k < C.ns && NCS > 0; k++) ok = ok && shape_body_slot(AT(S.sbody, k)); // arb_body
        if (!ok && fits) { // the compiled constraint list does not describe this scene (never expected)
            if (!shadow && sub == 0) {
                S.overflow[e] |= 32;
                if (reset_mask) reset_mask[e] = 0;
            }
            if (!QUAD) return;
        }
        // the view is built from the LDS carve only (never merged with the HBM pointers), so every
        // access through it compiles to ds_* with a constant offset from the lane's column
        MGState V = S;
        carve_view(V, smem, C, BLK);
        if constexpr (QUAD) {
            const bool own = !shadow && fits && ok;
            xfer_state_quad<C.nb, C.ns, C.nc, C.na, QL>(S, V, lane, e, sub, true);
            if (!fits && sub == 0) { // an empty scene in the env's column: nothing indexes past the caps
                V.nbodies[lane] = 0; V.nshapes[lane] = 0; V.ncons[lane] = 0; V.nactive[lane] = 0;
            }
            env_substeps_quad<NCS, QL, (C.shw > 0)>(V, L, lane, sub, a, P);
            if (own) xfer_state(S, V, C, lane, e, false, false, sub, QL);   // stores: no latency chain to batch
            // the env's lane 0 scores from HBM rows its sibling lanes just wrote back: order them
            // by the memory model, not by one wavefront's in-order memory pipe
            __threadfence_block();
            __syncthreads();
            if (!own || sub != 0) return;
        } else {   // COOP
            xfer_state(S, V, C, 0, e, true, true, lane, 64);
            __syncthreads();
            env_substeps_coop(V, L, lane, a, P);
            xfer_state(S, V, C, 0, e, false, true, lane, 64);
            __syncthreads();
            if (lane != 0) return;
        }
    } else {
        env_substeps(S, L, e, a, P);
    }
    int steps = S.episode_steps[e] + 1;
    S.episode_steps[e] = steps;
    bool d = max_steps > 0 && steps >= max_steps;
    double sc = d ? score_env(S, L, e, cfg.task) : 0.0;
    if (reward) reward[e] = (float)((cfg.flags & MG_DEBUG_REWARD) ? debug_reward(S, L, e, cfg.task) : sc);
    if (done) done[e] = d ? 1 : 0;
    if (eval_score) eval_score[e] = sc;
    // VecEnv auto-reset (next obs = first frame of the new episode) runs as reset_kernel on this mask -- or,
    // for the robot scenes without layout randomisation, here: their reset is serial straight-line code (no
    // rejection sampling), so the env's own lane runs it and the step saves a launch (cfg.fused_reset)
    if constexpr (VAR == 5 || VAR == 6) {
        if (cfg.fused_reset && d && auto_reset) {
            TaskCfg rc = cfg;
            rc.coop = 0;
            reset_env<VAR == 5 ? MG_TASK_MOVE_TO_REGION : MG_TASK_MOVE_TO_CORNER, 0>(S, L, e, rc);
        }
    }
    if (reset_mask) reset_mask[e] = (d && auto_reset && !cfg.fused_reset) ? 1 : 0;
    MG_PP(P, 7);
    MG_PP_END(P, (threadIdx.x & 63) == 0, 32);
}

template <int VAR, int BLK>
hipError_t launch_step_var(const MGState &S, const mg_library *L, TaskCfg cfg, int max_steps, int auto_reset,
                                  const uint8_t *actions, float *reward, uint8_t *done, double *eval_score,
                                  uint8_t *reset_mask, hipStream_t st) {
    constexpr StepCaps C = step_form_caps(VAR, BLK);
    const size_t lds = VAR == 0 ? 0 : mg_step_lds_bytes(C, BLK);
    static bool attr_set = false;
    if (VAR != 0 && !attr_set) {
        hipError_t err = hipFuncSetAttribute((const void *)step_kernel<VAR, BLK>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (err != hipSuccess) {
            fprintf(stderr, "step form %d/%d: LDS attribute %zu B: %s\n", VAR, BLK, lds, hipGetErrorString(err));
            return err;
        }
        attr_set = true;
    }
    hipLaunchKernelGGL((step_kernel<VAR, BLK>), dim3((S.n_envs + BLK - 1) / BLK), dim3(VAR == 4 || VAR == 5 || VAR == 6 ? 64 : BLK), lds, st, S, L, cfg,
                       max_steps, auto_reset, actions, reward, done, eval_score, reset_mask);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess)
        fprintf(stderr, "step form %d/%d: launch of %d workgroups, LDS %zu B: %s\n", VAR, BLK,
                (S.n_envs + BLK - 1) / BLK, lds, hipGetErrorString(err));
    return err;
}
