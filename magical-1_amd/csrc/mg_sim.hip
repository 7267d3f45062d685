// mg_sim.hip -- gfx950 kernels and the C ABI (include/magical_sim.h).
//
// Per env-step (mg_step): step_kernel (mg_physics.hip: one env per lane: action
// decode, 10 x [Robot.update + cpSpaceStep], episode counter, score, in-place
// reset of finished episodes) then render_kernel (mg_raster.hip: one workgroup
// per (env, view): 384^2 raster in LDS bands -> 96^2 area downsample -> LoRes
// frame stack).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/magical_sim.h"
#include "mg_launch.h"
#include "mg_phys.h"

static thread_local std::string g_err;
static int set_err(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
#define HIPC(x)                                                                                        \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess) return set_err(-5, std::string(#x) + ": " + hipGetErrorString(_e));      \
    } while (0)

// one [slot][N] row of the per-env state: env e's element is at pool + off + e * esize
struct StateRow { uint64_t off; uint32_t esize, pad; };

struct mg_sim {
    MGState S;
    // Next-layout shadow (reset prefetch).  BaseEnv.reset draws the whole layout from the env's RNG and
    // nothing else (mg_reset.h reset_env), so the layout of an env's NEXT episode is known as soon as its
    // current one starts.  SH is a second copy of the per-env state (same layout, no frame rings): right
    // after an env resets, reset_kernel runs on SH for it on a side stream, overlapping the step and render
    // kernels; when the episode ends the auto-reset is a copy SH -> S of that env (reset_copy_kernel).
    MGState SH;
    void *shadow_pool;
    StateRow *rows;        // device table of the per-env state rows (both pools)
    int nrows;
    uint8_t *pend;         // device u8[N]: envs whose shadow the side stream is preparing
    hipStream_t side;
    hipEvent_t ev_copied, ev_prepared;
    int shadow_ok;         // every env's shadow holds its next layout (set by a full mg_reset)
    int shadow_pending;    // a reset_kernel on SH is in flight on the side stream
    int reset_waves;          // auto-reset launches: wavefronts cap (0: one per env; MG_RESET_WAVES, A/B)
    int no_fused_reset;       // MG_FUSED_RESET=0: the robot scenes' auto-reset as its own launch (A/B, tests)
    int reset_waves_shadow;   // the shadow's next-layout launches: the same (MG_RESET_WAVES_SHADOW)
    int copy_wg;              // reset_copy_kernel's workgroups cap (MG_COPY_WG: tests, A/B)
    int force_render_retry;   // tests: the first k render classes of the chain hand every (env, view) on
    int scache_mode;          // tests: RenderOut::scache_mode
    mg_library *dlib;
    void *pool;
    size_t pool_bytes;
    int task, flags, preproc, max_steps, device, auto_reset;
    mg_buffers out;
    int bound;
    // window rings of the stacked views (mg_bind_window; null: materialised stacks), their period, and the step
    // counter that picks the slot (advanced by every mg_step before its render; resets do not advance it)
    uint8_t *wring[2];
    int wK;
    long long wstep;
    StepCaps caps;     // the task's per-env slot caps
    int step_variant;  // compiled LDS-resident step variant (0: HBM state)
    int step_blk;      // envs per step workgroup
    uint8_t *reset_mask; // device u8[N]: envs to auto-reset after the step
    // optional per-kernel timing (hipEvents on the launch stream)
    int timing;
    std::vector<hipEvent_t> ev;   // quadruples: before step_kernel, after it, after the auto-reset, after render_kernel
    size_t ev_used;
};

// ---------------------------------------------------------------------------
// kernels
__global__ void __launch_bounds__(64) bodies_kernel(MGState S, double *out, int32_t *counts) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= S.n_envs) return;
    for (int b = 0; b < MG_MAX_BODIES; b++) {
        double *o = out + ((size_t)e * MG_MAX_BODIES + b) * 6;
        if (b < S.nbodies[e]) {
            o[0] = AT(S.bpx, b); o[1] = AT(S.bpy, b); o[2] = AT(S.ba, b);
            o[3] = AT(S.bvx, b); o[4] = AT(S.bvy, b); o[5] = AT(S.bw, b);
        } else {
            for (int k = 0; k < 6; k++) o[k] = 0.0;
        }
    }
    if (counts) {
        counts[4 * e + 0] = S.nbodies[e]; counts[4 * e + 1] = S.nshapes[e];
        counts[4 * e + 2] = S.ncons[e]; counts[4 * e + 3] = S.nactive[e];
    }
}

// the solved arbiters of every env in active order (oracle/env.c oenv_get_arbiters has the same layout)
#define MG_ARB_DUMP 28
__global__ void __launch_bounds__(64) arbiters_kernel(MGState S, double *out, uint64_t *hash) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= S.n_envs) return;
    const int na = S.nactive[e];
    for (int i = 0; i < MG_MAX_ARB; i++) {
        double *o = out + ((size_t)e * MG_MAX_ARB + i) * MG_ARB_DUMP;
        uint64_t *h = hash + ((size_t)e * MG_MAX_ARB + i) * 2;
        for (int k = 0; k < MG_ARB_DUMP; k++) o[k] = 0.0;
        h[0] = h[1] = 0;
        if (i >= na) continue;
        const int slot = AT(S.active, i), cnt = AT(S.acount, slot);
        o[0] = slot; o[1] = AT(S.astate, slot); o[2] = cnt; o[3] = AT(S.asa, slot); o[4] = AT(S.asb, slot);
        o[5] = AT(S.anx, slot); o[6] = AT(S.any, slot); o[7] = AT(S.au, slot);
        for (int k = 0; k < cnt && k < 2; k++) {
            double *q = o + 8 + 10 * k;
            q[0] = ACON(k, AC_R1X, slot); q[1] = ACON(k, AC_R1Y, slot); q[2] = ACON(k, AC_R2X, slot);
            q[3] = ACON(k, AC_R2Y, slot); q[4] = ACON(k, AC_JN, slot); q[5] = ACON(k, AC_JT, slot);
            q[6] = ACON(k, AC_NMASS, slot); q[7] = ACON(k, AC_TMASS, slot); q[8] = ACON(k, AC_BIAS, slot);
            q[9] = ACON(k, AC_JB, slot);
            h[k] = AHASH(k, slot);
        }
    }
}

__global__ void __launch_bounds__(64) errors_kernel(MGState S, int32_t *out) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= S.n_envs) return;
    out[e] = S.overflow[e];
}

// self-test of the device correctly rounded sincos (tests/test_gpu_parity.py compares with the oracle)
__global__ void __launch_bounds__(256) sincos_kernel(const double *x, double *s, double *c, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    mg_sincos(x[i], s[i], c[i]);
}

// Philox4x32-10 (Salmon et al. 2011): counter = (step lo, step hi, env, 0), key = (k lo, k hi)
__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t &hi) {
    uint64_t p = (uint64_t)a * b;
    hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}
__global__ void __launch_bounds__(256) actions_kernel(uint8_t *out, int n, uint64_t key, uint64_t step) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    uint32_t c0 = (uint32_t)step, c1 = (uint32_t)(step >> 32), c2 = (uint32_t)e, c3 = 0;
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    for (int r = 0; r < 10; r++) {
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo(0xD2511F53u, c0, hi0);
        uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[e] = (uint8_t)(c0 % 18u);
}

// env e's per-env state rows src -> dst for the envs in mask (pend[e] = mask[e] for every env): the
// auto-reset from the next-layout shadow (src = shadow, to_main), or an explicit reset's state handed to
// the shadow (src = main).  Error flags: bit 2 (PlacementError of this reset) and the sticky bit 64 come
// from the reset that produced the layout.  A grid of at most copy_wg workgroups (mg_sim; 2048, MG_COPY_WG for
// tests): pend is written for every env with coalesced stores, then each workgroup walks its envs (grid-stride)
// and copies the rows of the masked ones -- an auto-reset step masks a few dozen of 8192 envs, and one workgroup
// per env (8192 mostly idle ones on the step's critical path) measured 0.095 -> 0.080 ms per step for the copy and
// reset phase (ClusterColour; MatchRegions 0.107 -> 0.090, profiles/r06_cw).
__global__ void __launch_bounds__(256) reset_copy_kernel(const char *__restrict__ src, char *__restrict__ dst,
                                                         const StateRow *__restrict__ rows, int nrows,
                                                         const uint8_t *__restrict__ mask, uint8_t *__restrict__ pend,
                                                         MGState S, MGState SH, int to_main) {
    const int tid = threadIdx.x;
    for (int e = blockIdx.x * 256 + tid; e < S.n_envs; e += gridDim.x * 256)
        pend[e] = (!mask || mask[e] != 0) ? 1 : 0;
    for (int e = blockIdx.x; e < S.n_envs; e += gridDim.x) {
        if (mask && mask[e] == 0) continue;   // uniform over the workgroup
        for (int r = tid; r < nrows; r += 256) {
            const StateRow w = rows[r];
            const size_t o = w.off + (size_t)e * w.esize;
            switch (w.esize) {
            case 8: *(uint64_t *)(dst + o) = *(const uint64_t *)(src + o); break;
            case 4: *(uint32_t *)(dst + o) = *(const uint32_t *)(src + o); break;
            case 2: *(uint16_t *)(dst + o) = *(const uint16_t *)(src + o); break;
            default: dst[o] = src[o]; break;
            }
        }
        if (tid == 0) {
            if (to_main) {
                S.overflow[e] = (S.overflow[e] & ~2) | (SH.overflow[e] & (2 | 64));
                if (S.target_out) {   // PickAndPlace: reset_env writes the bound target output at reset
                    double *t = S.target_out + 4 * (size_t)e;
                    t[0] = SH.tgt_ids[e]; t[1] = SH.tgt_ids[S.N + e]; t[2] = SH.tgt_x[e]; t[3] = SH.tgt_y[e];
                }
            } else {
                SH.overflow[e] = S.overflow[e];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// allocation
struct Carver {
    char *base;
    size_t off;
    std::vector<StateRow> *rows = nullptr;   // records every take as [n / N] rows (n = slots x N)
    size_t N = 0;
    template <typename T> T *take(size_t n) {
        off = (off + 255) & ~(size_t)255;
        T *p = (T *)(base ? base + off : nullptr);
        if (rows)
            for (size_t k = 0; k < n / N; k++) rows->push_back(StateRow{off + k * N * sizeof(T), (uint32_t)sizeof(T), 0u});
        off += n * sizeof(T);
        return p;
    }
};

static void layout(MGState &S, Carver &c, bool frames = true) {
    size_t N = (size_t)S.N;
    c.N = N;
    size_t B = MG_MAX_BODIES * N, SH = MG_MAX_SHAPES * N, C = MG_MAX_CONS * N, A = MG_MAX_ARB * N, E = MG_MAX_ENTS * N;
    S.bpx = c.take<double>(B); S.bpy = c.take<double>(B); S.bvx = c.take<double>(B); S.bvy = c.take<double>(B);
    S.ba = c.take<double>(B); S.bw = c.take<double>(B); S.bvbx = c.take<double>(B); S.bvby = c.take<double>(B);
    S.bwb = c.take<double>(B); S.brc = c.take<double>(B); S.brs = c.take<double>(B); S.bminv = c.take<double>(B);
    S.biinv = c.take<double>(B); S.bacache = c.take<double>(B); S.bkin = c.take<int8_t>(B);
    S.nbodies = c.take<int32_t>(N);
    S.sbody = c.take<int8_t>(SH); S.spoly = c.take<int8_t>(SH); S.sent = c.take<int8_t>(SH);
    S.sgroup = c.take<int16_t>(SH); S.shash = c.take<int16_t>(SH); S.scat = c.take<uint8_t>(SH);
    S.sr = c.take<double>(SH); S.su = c.take<double>(SH); S.sbbl = c.take<double>(SH); S.sbbb = c.take<double>(SH);
    S.sbbr = c.take<double>(SH); S.sbbt = c.take<double>(SH);
    S.nshapes = c.take<int32_t>(N);
    S.ctype = c.take<int8_t>(C); S.ca = c.take<int8_t>(C); S.cb = c.take<int8_t>(C);
    S.cp = c.take<double>((size_t)CP_NUM * C);
    S.ncons = c.take<int32_t>(N);
    S.akey = c.take<int32_t>(A); S.astamp = c.take<uint32_t>(A); S.astate = c.take<int8_t>(A);
    S.acount = c.take<int8_t>(A); S.asa = c.take<int8_t>(A); S.asb = c.take<int8_t>(A);
    S.anx = c.take<double>(A); S.any = c.take<double>(A); S.au = c.take<double>(A);
    S.acon = c.take<double>((size_t)2 * AC_NUM * A); S.ahash = c.take<uint64_t>(2 * A);
    S.active = c.take<int8_t>(A); S.nactive = c.take<int32_t>(N); S.stamp = c.take<uint32_t>(N);
    S.curr_dt = c.take<double>(N);
    {   // not state rows: the error flags are merged by reset_copy_kernel, rg_retry is render scratch
        std::vector<StateRow> *r = c.rows;
        c.rows = nullptr;
        S.overflow = c.take<int32_t>(N); S.rg_retry = c.take<uint8_t>(2 * N);
        c.rows = r;
    }
    S.target_speed = c.take<double>(N); S.rel_turn = c.take<double>(N); S.target_finger = c.take<double>(N);
    S.robot_body0 = c.take<int32_t>(N); S.robot_cons0 = c.take<int32_t>(N); S.pv = c.take<double>(5 * N);
    S.ekind = c.take<int8_t>(E); S.etype = c.take<int8_t>(E); S.ecol = c.take<int8_t>(E); S.erole = c.take<int8_t>(E);
    S.ebody0 = c.take<int8_t>(E); S.eshape0 = c.take<int8_t>(E); S.enshapes = c.take<int8_t>(E);
    S.ex = c.take<double>(E); S.ey = c.take<double>(E); S.eang = c.take<double>(E); S.eh = c.take<double>(E);
    S.ew = c.take<double>(E); S.nents = c.take<int32_t>(N);
    S.goal_ent = c.take<int32_t>(N); S.episode_steps = c.take<int32_t>(N);
    S.tgt_ent = c.take<int32_t>(N); S.tgt_ids = c.take<int32_t>(2 * N);
    S.tgt_x = c.take<double>(N); S.tgt_y = c.take<double>(N);
    S.target_out = nullptr;
    S.mt_key = c.take<uint32_t>(624 * N); S.mt_pos = c.take<int32_t>(N);
    c.rows = nullptr;   // state rows end here (frames and render scratch below are not part of a layout)
    if (!frames) { S.hist_allo = S.hist_ego = S.scache = S.scache_ok = nullptr; S.hist_head = nullptr; return; }
    size_t FR = (size_t)MG_LORES * MG_LORES * 3;
    S.hist_allo = c.take<uint8_t>(4 * N * FR); S.hist_ego = c.take<uint8_t>(4 * N * FR);
    S.hist_head = c.take<int32_t>(2 * N);
    S.scache = c.take<uint8_t>(N * FR); S.scache_ok = c.take<uint8_t>(N);
}

static hipStream_t as_stream(void *s) { return (hipStream_t)s; }

// Per-env slot caps of a (task, variant): bodies, shapes, constraints, arbiter slots.
static StepCaps step_caps(int task, int flags, int n_envs, const mg_library &lib) {
    int nblk = 0, star_ok = 1;
    switch (task) {
    case MG_TASK_MOVE_TO_REGION: nblk = 0; break;
    case MG_TASK_MOVE_TO_CORNER: nblk = 1; star_ok = (flags & MG_RAND_SHAPE_TYPE) != 0; break;
    case MG_TASK_CLUSTER_COLOUR:
    case MG_TASK_CLUSTER_SHAPE: nblk = (flags & MG_RAND_SHAPE_COUNT) ? 10 : 8; break;
    case MG_TASK_MAKE_LINE: nblk = 4; break;
    case MG_TASK_FIND_DUPE: nblk = 7; break;
    case MG_TASK_FIX_COLOUR: nblk = 3; break;
    case MG_TASK_PICK_AND_PLACE: nblk = 3; break;
    default: nblk = (flags & MG_RAND_SHAPE_COUNT) ? 8 : 5; break;
    }
    const int per_blk = star_ok ? lib.block_nshapes[MG_SHAPE_STAR] : 1;
    StepCaps c;
    c.nb = 6 + nblk;
    c.ns = 5 + nblk * per_blk;
    c.nc = 10 + 2 * nblk;
    int pairs = 4 * c.ns + 5 * (c.ns - 5) + ((c.ns - 5) * (c.ns - 6)) / 2; // walls, robot-block, block-block
    c.na = pairs < MG_MAX_ARB ? (pairs + 3) / 4 * 4 : MG_MAX_ARB;
    c.blk = 16;
    (void)n_envs;
    return c;
}

// Step kernel per scene (measured on MI355X, 8192 envs, ms per env-step of physics):
// * compiled constraint lists (robot only / robot + one block): forms 5/6, 16 envs per 64-lane workgroup,
//   4 lanes per env (4096 envs: MoveToRegion 0.62 ms, MoveToCorner 1.15; one env per lane, variants 1/2:
//   0.73 / 1.42);
// * every other scene (up to 8 blocks, runtime constraint lists): the cooperative LDS variant 4, one env
//   per 64-lane wavefront with the order-free parts across lanes -- MatchRegions-TestAll 6.0 ms (variant
//   3, one env per single-lane workgroup: 10.6; HBM-state kernel, 64 envs per wavefront: 21.1),
//   ClusterColour-Demo 8.6 ms (variant 3: 15.1; HBM-state kernel: 10.7).
static int pick_step_variant(const StepCaps &c, int n_envs, int task) {
    (void)task;
    int v = mg_step_variant(c, n_envs);
    if (v == 3) v = 4;
    if (v == 1 || v == 2) v += 4;
    const char *ov = getenv("MG_STEP_VARIANT");
    if (ov) { // experiments: 0 (HBM state), the scene's compiled variant (5 / 6; 1 / 2 in comparison builds),
              // 3 / 4 (LDS runtime lists)
        const int w = atoi(ov), base = mg_step_variant(c, n_envs);
        if (w == 0 || ((w == base || w == 3) && mg_step_blk_ok(w, w == 3 ? 1 : 16)) || w == 4) v = w;
        if ((base == 1 || base == 2) && w == base + 4) v = w;  // 5 / 6: the compiled lists, 4 lanes per env
    }
    return v;
}

// Robot-only scenes (variant 5) below 16 envs x CUs run 8 envs per workgroup: the grid then still reaches
// every CU, and a workgroup takes half a CU's LDS, so render workgroups of another env chunk fit beside it
// (the pipelined pool's 2048-env chunks: MoveToRegion 2.82 -> 2.84 M env-steps/s, profiles/r04_check7/).  At 4096 envs and more,
// 16 (8 measured slower there: two workgroups per CU, 0.83 vs 0.61 ms).
static int pick_step_blk(int variant, int n_envs, int cus) {
    int b = variant == 0 ? 64 : variant == 3 || variant == 4 ? 1 : 16;
    if ((variant == 5 || variant == 6) && n_envs < 16 * cus) b = 8;
    const char *ov = getenv(variant == 0 ? "MG_STEP_BLK0" : "MG_STEP_BLK"); // experiments
    if (ov && mg_step_blk_ok(variant, atoi(ov))) b = atoi(ov);
    return b;
}

static int grid64(const mg_sim *s) { return (s->S.n_envs + 63) / 64; }

static int render_lores(mg_sim *s, hipStream_t st, const uint8_t *mask) {
    RenderOut ro = {};
    ro.full = nullptr;
    ro.mask = mask;
    ro.debug_skip = 0;
    ro.small = s->task == MG_TASK_MOVE_TO_REGION || s->task == MG_TASK_MOVE_TO_CORNER;
    ro.first_level = s->task == MG_TASK_CLUSTER_COLOUR ? 0 : 1;   // render class chain start (mg_raster.hip)
    ro.force_retry = s->force_render_retry;
    ro.scache_mode = s->scache_mode;
#ifdef MG_PROFILE
    if (getenv("MG_DEBUG_SKIP")) ro.debug_skip = atoi(getenv("MG_DEBUG_SKIP"));
#endif
    ro.obs_allo = s->out.obs_allo; ro.obs_ego = s->out.obs_ego; ro.obs_past = s->out.obs_past;
    ro.preproc = s->preproc;
    ro.frames_only = s->out.frames_only;
    ro.wring[0] = s->wring[0]; ro.wring[1] = s->wring[1]; ro.wK = s->wK;
    ro.wpos = s->wK > 0 ? (int)(s->wstep % s->wK) : 0;
    for (int fr = 0; fr < 2 && s->wK > 0; fr++) {   // slot lists of a running / a fresh env (mg_bind_window)
        int n = 0;
        for (int d = 0; d < (fr ? 4 : 1); d++) {
            const int f = (ro.wpos + s->wK - d) % s->wK;
            ro.wsl[fr][n++] = (int8_t)f;
            if (f < 3) ro.wsl[fr][n++] = (int8_t)(s->wK + f);
        }
        ro.wnsl[fr] = n;
    }
    HIPC(mg_launch_render(s->S, s->dlib, ro, 0, st));
    if (s->preproc == MG_PREPROC_LORES3EA && !s->out.frames_only)
        HIPC(mg_launch_compose3ea(s->S, (const uint8_t *)s->out.obs_allo, mask, (uint8_t *)s->out.obs_past, st));
    return 0;
}

// hand the state of the envs in mask (null: all) from one pool to the other on st, then prepare their
// next layouts on the side stream (reset_kernel on the shadow)
static int shadow_handover(mg_sim *s, hipStream_t st, const uint8_t *mask, int to_main) {
    if (s->shadow_pending) HIPC(hipStreamWaitEvent(st, s->ev_prepared, 0));   // pend and the shadow are free
    const char *src = (const char *)(to_main ? s->shadow_pool : s->pool);
    char *dst = (char *)(to_main ? s->pool : s->shadow_pool);
    const int cgrid = (s->copy_wg > 0 && s->S.n_envs > s->copy_wg) ? s->copy_wg : s->S.n_envs;
    hipLaunchKernelGGL(reset_copy_kernel, dim3(cgrid), dim3(256), 0, st, src, dst, s->rows, s->nrows, mask,
                       s->pend, s->S, s->SH, to_main);
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(s->ev_copied, st));
    HIPC(hipStreamWaitEvent(s->side, s->ev_copied, 0));
    TaskCfg cfg = {s->task, s->flags};
    HIPC(mg_launch_reset(s->SH, s->dlib, cfg, s->pend, s->side, s->reset_waves_shadow));
    HIPC(hipEventRecord(s->ev_prepared, s->side));
    s->shadow_pending = 1;
    return 0;
}

// ---------------------------------------------------------------------------
// C ABI
extern "C" {

const char *mg_last_error(void) { return g_err.c_str(); }

#ifdef MG_PROFILE
// profiling builds only (tools/gpu_phase.py): phase timer totals, then cleared
int mg_debug_read_profile(unsigned long long *out) {
    HIPC(hipDeviceSynchronize());
    for (int i = 0; i < 64; i++) out[i] = 0;
    HIPC(mg_prof_read_physics(out));
    HIPC(mg_prof_read_raster(out));
    return 0;
}
#endif

int mg_create(const mg_config *cfg, mg_sim **out) {
    if (!cfg || !out) return set_err(-22, "mg_create: null argument");
    if (cfg->library_size != (int64_t)sizeof(mg_library))
        return set_err(-22, "mg_create: library_size mismatch (expected " + std::to_string(sizeof(mg_library)) + ")");
    if (cfg->num_envs <= 0) return set_err(-22, "mg_create: num_envs must be positive");
    if (cfg->task < 0 || cfg->task > MG_TASK_PICK_AND_PLACE) return set_err(-22, "mg_create: unknown task");
    if (cfg->preproc != MG_PREPROC_LORES4E && cfg->preproc != MG_PREPROC_LORESSTACK &&
        cfg->preproc != MG_PREPROC_LORES4A && cfg->preproc != MG_PREPROC_LORES3EA && cfg->preproc != MG_PREPROC_NONE)
        return set_err(-95, "mg_create: preprocessor not supported by the GPU path");
    HIPC(hipSetDevice(cfg->device));
    mg_sim *s = new mg_sim();
    memset(&s->S, 0, sizeof(MGState));
    s->timing = 0; s->ev_used = 0; s->bound = 0;
    s->wring[0] = s->wring[1] = nullptr; s->wK = 0; s->wstep = 0;
    s->task = cfg->task; s->flags = cfg->rand_flags; s->preproc = cfg->preproc;
    s->max_steps = cfg->max_episode_steps; s->device = cfg->device; s->auto_reset = cfg->auto_reset;
    s->S.n_envs = cfg->num_envs;
    s->S.cons_cap = MG_MAX_CONS;
    s->S.arb_cap = MG_MAX_ARB;
    s->S.max_tries = 10000; // geom.py:198
    s->S.shw = nullptr;     // HBM-state kernels keep their narrowphase shapes in registers / scratch
    if (const char *mt = getenv("MG_DEBUG_MAX_TRIES")) s->S.max_tries = atoi(mt) > 0 ? atoi(mt) : 10000; // tests only
    s->reset_waves = getenv("MG_RESET_WAVES") ? atoi(getenv("MG_RESET_WAVES")) : 0;
    s->no_fused_reset = getenv("MG_FUSED_RESET") && atoi(getenv("MG_FUSED_RESET")) == 0;
    // the shadow's next layouts run beside the step stream's kernels: 256 wavefronts scanning the pending mask
    // instead of one 352-VGPR wavefront per env, most of which only exit (512: ClusterColour 1.458 -> 1.468 M,
    // MatchRegions 1.329 -> 1.358 M env-steps/s, same box; the in-place robot-scene resets gained nothing).
    // Round 5: 256 -- fewer 352-VGPR wavefronts holding SIMDs beside the render -- MatchRegions 1.375 -> 1.393 M,
    // ClusterColour unchanged; 64 makes a wavefront's serial run of layouts outlast the step (MatchRegions 1.11 M)
    s->reset_waves_shadow = getenv("MG_RESET_WAVES_SHADOW") ? atoi(getenv("MG_RESET_WAVES_SHADOW")) : 256;
    s->copy_wg = getenv("MG_COPY_WG") ? atoi(getenv("MG_COPY_WG")) : 2048;
    if (const char *rr = getenv("MG_DEBUG_RENDER_RETRY")) s->force_render_retry = atoi(rr);                 // tests only
    else s->force_render_retry = 0;
    s->scache_mode = getenv("MG_DEBUG_SCACHE") ? atoi(getenv("MG_DEBUG_SCACHE")) : 0;                    // tests only
    s->S.N = (cfg->num_envs + 63) / 64 * 64;
    std::vector<StateRow> rows;
    Carver sizing = {nullptr, 0};
    sizing.rows = &rows;
    layout(s->S, sizing);
    s->pool_bytes = sizing.off + 256;
    hipError_t err = hipMalloc(&s->pool, s->pool_bytes);
    if (err != hipSuccess) { delete s; return set_err(-12, std::string("mg_create: hipMalloc pool: ") + hipGetErrorString(err)); }
    HIPC(hipMemset(s->pool, 0, s->pool_bytes));
    Carver real = {(char *)s->pool, 0};
    layout(s->S, real);
    err = hipMalloc((void **)&s->dlib, sizeof(mg_library));
    if (err != hipSuccess) { (void)hipFree(s->pool); delete s; return set_err(-12, "mg_create: hipMalloc library"); }
    HIPC(hipMemcpy(s->dlib, cfg->library, sizeof(mg_library), hipMemcpyHostToDevice));
    s->caps = step_caps(cfg->task, cfg->rand_flags, cfg->num_envs, *(const mg_library *)cfg->library);
    s->step_variant = pick_step_variant(s->caps, cfg->num_envs, cfg->task);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
    s->step_blk = pick_step_blk(s->step_variant, cfg->num_envs, cus);
    err = hipMalloc((void **)&s->reset_mask, (size_t)s->S.N);
    if (err != hipSuccess) { (void)hipFree(s->pool); (void)hipFree(s->dlib); delete s; return set_err(-12, "mg_create: hipMalloc mask"); }
    HIPC(hipMemset(s->reset_mask, 0, (size_t)s->S.N));
    // next-layout shadow: the many-block tasks, whose rejection-sampled layouts make a reset long (the
    // robot scenes reset in ~0.03 ms); MG_RESET_PREFETCH=0/1 overrides
    s->shadow_pool = nullptr; s->rows = nullptr; s->pend = nullptr; s->side = nullptr;
    s->shadow_ok = 0; s->shadow_pending = 0; s->nrows = 0;
    bool prefetch = s->auto_reset && s->task != MG_TASK_MOVE_TO_REGION && s->task != MG_TASK_MOVE_TO_CORNER;
    if (const char *pf = getenv("MG_RESET_PREFETCH")) prefetch = s->auto_reset && atoi(pf) != 0;
    if (prefetch) {
        s->SH = s->S;
        s->SH.target_out = nullptr;
        Carver ssz = {nullptr, 0};
        layout(s->SH, ssz, false);
        HIPC(hipMalloc(&s->shadow_pool, ssz.off + 256));
        HIPC(hipMemset(s->shadow_pool, 0, ssz.off + 256));
        Carver sreal = {(char *)s->shadow_pool, 0};
        layout(s->SH, sreal, false);
        s->nrows = (int)rows.size();
        HIPC(hipMalloc((void **)&s->rows, rows.size() * sizeof(StateRow)));
        HIPC(hipMemcpy(s->rows, rows.data(), rows.size() * sizeof(StateRow), hipMemcpyHostToDevice));
        HIPC(hipMalloc((void **)&s->pend, (size_t)s->S.N));
        HIPC(hipMemset(s->pend, 0, (size_t)s->S.N));
        HIPC(hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking));
        HIPC(hipEventCreateWithFlags(&s->ev_copied, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&s->ev_prepared, hipEventDisableTiming));
    }
    std::vector<uint32_t> seeds(cfg->num_envs);
    for (int i = 0; i < cfg->num_envs; i++) seeds[i] = cfg->seeds ? cfg->seeds[i] : cfg->base_seed + (uint32_t)i;
    *out = s;
    return mg_seed(s, seeds.data());
}

int mg_seed(mg_sim *s, const uint32_t *seeds_host) {
    if (!s || !seeds_host) return set_err(-22, "mg_seed: null argument");
    HIPC(hipSetDevice(s->device));
    if (s->shadow_pending) HIPC(hipEventSynchronize(s->ev_prepared));
    s->shadow_pending = 0;
    s->shadow_ok = 0;   // the shadow's layouts came from the old seeds: valid again after a full mg_reset
    uint32_t *d = nullptr;
    HIPC(hipMalloc(&d, sizeof(uint32_t) * s->S.n_envs));
    HIPC(hipMemcpy(d, seeds_host, sizeof(uint32_t) * s->S.n_envs, hipMemcpyHostToDevice));
    HIPC(mg_launch_seed(s->S, d, 0));
    HIPC(hipDeviceSynchronize());
    HIPC(hipFree(d));
    return 0;
}

int mg_bind_outputs(mg_sim *s, const mg_buffers *b) {
    if (!s || !b) return set_err(-22, "mg_bind_outputs: null argument");
    // with window rings bound (mg_bind_window) the stacked outputs are views of the rings: LoResStack's
    // obs_allo / obs_ego and LoRes4E / LoRes4A's obs_past may be null
    const bool win = !b->frames_only && (s->wring[0] || s->wring[1]);
    const bool stack_ae = s->preproc == MG_PREPROC_LORESSTACK;
    if (s->preproc != MG_PREPROC_NONE && (!b->obs_allo || !b->obs_ego) && !(win && stack_ae))
        return set_err(-22, "mg_bind_outputs: obs_allo / obs_ego required");
    if (b->frames_only != 0 && b->frames_only != 1) return set_err(-22, "mg_bind_outputs: frames_only must be 0 or 1");
    if (b->frames_only && s->preproc == MG_PREPROC_NONE)
        return set_err(-22, "mg_bind_outputs: frames_only needs a LoRes preprocessor");
    if ((s->preproc == MG_PREPROC_LORES4E || s->preproc == MG_PREPROC_LORES4A || s->preproc == MG_PREPROC_LORES3EA) &&
        !b->frames_only && !b->obs_past && !(win && s->preproc != MG_PREPROC_LORES3EA))
        return set_err(-22, "mg_bind_outputs: obs_past required for this preprocessor");
    const void *ptrs[3] = {b->obs_allo, b->obs_ego, b->frames_only ? nullptr : b->obs_past};
    for (const void *p : ptrs)
        if (((uintptr_t)p & 15) != 0) return set_err(-22, "mg_bind_outputs: observation buffers must be 16-byte aligned");
    if (s->task == MG_TASK_PICK_AND_PLACE && !b->target)
        return set_err(-22, "mg_bind_outputs: target required for PickAndPlace");
    s->out = *b;
    s->S.target_out = b->target;
    s->bound = 1;
    return 0;
}

int mg_reset(mg_sim *s, const uint8_t *mask, void *stream) {
    if (!s) return set_err(-22, "mg_reset: null sim");
    if (!s->bound && s->preproc != MG_PREPROC_NONE) return set_err(-22, "mg_reset: outputs not bound");
    HIPC(hipSetDevice(s->device));
    hipStream_t st = as_stream(stream);
    TaskCfg cfg = {s->task, s->flags};
    HIPC(mg_launch_reset(s->S, s->dlib, cfg, mask, st));
    if (s->shadow_pool) {
        const int rc = shadow_handover(s, st, mask, 0);
        if (rc) return rc;
        if (!mask) s->shadow_ok = 1;
    }
    if (s->preproc != MG_PREPROC_NONE) return render_lores(s, st, mask);
    return 0;
}

int mg_step(mg_sim *s, const uint8_t *actions, void *stream) {
    if (!s || !actions) return set_err(-22, "mg_step: null argument");
    if (!s->bound && s->preproc != MG_PREPROC_NONE) return set_err(-22, "mg_step: outputs not bound");
    HIPC(hipSetDevice(s->device));
    hipStream_t st = as_stream(stream);
    TaskCfg cfg = {s->task, s->flags};
    // robot scenes without layout randomisation: the step kernel runs the auto-reset itself (mg_stepk.h)
    const bool layout = (s->flags & (MG_RAND_LAYOUT_MINOR | MG_RAND_LAYOUT_FULL)) != 0;
    cfg.fused_reset = s->auto_reset && !s->shadow_ok && !layout && !s->no_fused_reset &&
                      ((s->task == MG_TASK_MOVE_TO_REGION && s->step_variant == 5) ||
                       (s->task == MG_TASK_MOVE_TO_CORNER && s->step_variant == 6));
    hipEvent_t *ev = nullptr;
    if (s->timing && s->ev_used + 4 <= s->ev.size()) { ev = &s->ev[s->ev_used]; s->ev_used += 4; }
    if (ev) HIPC(hipEventRecord(ev[0], st));
    HIPC(mg_launch_step(s->S, s->dlib, cfg, s->step_variant, s->step_blk, s->max_steps, s->auto_reset, actions, s->out.reward,
                        s->out.done, s->out.eval_score, s->reset_mask, st));
    if (ev) HIPC(hipEventRecord(ev[1], st));
    if (s->auto_reset) {
        if (s->shadow_ok) {
            const int rc = shadow_handover(s, st, s->reset_mask, 1);
            if (rc) return rc;
        } else if (!cfg.fused_reset) {
            HIPC(mg_launch_reset(s->S, s->dlib, cfg, s->reset_mask, st, s->reset_waves));
        }
    }
    if (ev) HIPC(hipEventRecord(ev[2], st));
    int rc = 0;
    s->wstep++;   // this step's frame goes to the window rings' next slot
    if (s->preproc != MG_PREPROC_NONE) rc = render_lores(s, st, nullptr);
    if (ev) HIPC(hipEventRecord(ev[3], st));
    return rc;
}

hipError_t mg_launch_replay(const uint8_t *frames, int32_t nframes, const int32_t *episode_start, int32_t preproc,
                            uint8_t *scratch, uint8_t *out_allo, uint8_t *out_ego, uint8_t *out_past, hipStream_t st);

int mg_replay_lores(const uint8_t *frames, int32_t nframes, const int32_t *episode_start, int32_t preproc,
                    uint8_t *scratch, uint8_t *out_allo, uint8_t *out_ego, uint8_t *out_past, void *stream) {
    if (nframes <= 0 || !frames || !episode_start || !scratch || !out_allo || !out_ego)
        return set_err(-22, "mg_replay_lores: null argument or nframes <= 0");
    if (preproc != MG_PREPROC_LORES4E && preproc != MG_PREPROC_LORESSTACK && preproc != MG_PREPROC_LORES3EA &&
        preproc != MG_PREPROC_LORES4A)
        return set_err(-22, "mg_replay_lores: preproc must be 1 (LoRes4E), 2 (LoResStack), 3 (LoRes3EA) or 4 (LoRes4A)");
    if (preproc != MG_PREPROC_LORESSTACK && !out_past) return set_err(-22, "mg_replay_lores: out_past required");
    const void *ptrs[6] = {frames, scratch, out_allo, out_ego, out_past ? out_past : out_allo, episode_start};
    for (const void *p : ptrs)
        if (((uintptr_t)p & 15) != 0) return set_err(-22, "mg_replay_lores: buffers must be 16-byte aligned");
    HIPC(mg_launch_replay(frames, nframes, episode_start, preproc, scratch, out_allo, out_ego, out_past,
                          as_stream(stream)));
    return 0;
}

hipError_t mg_launch_restack(const uint8_t *recv, int32_t world, int32_t n, int64_t stride, int64_t off_a,
                             int64_t off_e, int64_t off_d, int32_t preproc, int64_t step, int32_t all_fresh,
                             uint8_t *ring, uint8_t *out_allo, uint8_t *out_ego, uint8_t *out_past, hipStream_t st);

int mg_restack(const uint8_t *recv, int32_t world, int32_t n, int64_t rank_stride, int64_t off_allo, int64_t off_ego,
               int64_t off_done, int32_t preproc, int64_t step, int32_t all_fresh, uint8_t *ring, uint8_t *out_allo,
               uint8_t *out_ego, uint8_t *out_past, void *stream) {
    if (!recv || !ring || world <= 0 || n <= 0 || step < 0) return set_err(-22, "mg_restack: null argument or bad size");
    const int64_t FR = (int64_t)MG_LORES * MG_LORES * 3;
    if ((int64_t)world * n * (MG_LORES * MG_LORES / 4) >= ((int64_t)1 << 31))
        return set_err(-22, "mg_restack: world * n too large for one launch");
    if (preproc == MG_PREPROC_LORESSTACK) {
        if (!out_allo || !out_ego) return set_err(-22, "mg_restack: LoResStack needs out_allo and out_ego");
    } else if (preproc == MG_PREPROC_LORES4E || preproc == MG_PREPROC_LORES4A || preproc == MG_PREPROC_LORES3EA) {
        if (!out_past) return set_err(-22, "mg_restack: out_past required for this preprocessor");
    } else {
        return set_err(-22, "mg_restack: preproc must be 1 (LoRes4E), 2 (LoResStack), 3 (LoRes3EA) or 4 (LoRes4A)");
    }
    if (off_allo < 0 || off_ego < 0 || off_done < 0 || off_allo + n * FR > rank_stride || off_ego + n * FR > rank_stride ||
        off_done + n > rank_stride)
        return set_err(-22, "mg_restack: a key of the rank block lies outside rank_stride");
    const int64_t al[4] = {(int64_t)(uintptr_t)recv, rank_stride, off_allo, off_ego};
    for (int64_t a : al)
        if (a & 15) return set_err(-22, "mg_restack: recv, rank_stride and frame offsets must be 16-byte aligned");
    const void *ptrs[4] = {ring, out_allo, out_ego, out_past};
    for (const void *p : ptrs)
        if (((uintptr_t)p & 15) != 0) return set_err(-22, "mg_restack: buffers must be 16-byte aligned");
    HIPC(mg_launch_restack(recv, world, n, rank_stride, off_allo, off_ego, off_done, preproc, step, all_fresh, ring,
                           out_allo, out_ego, out_past, as_stream(stream)));
    return 0;
}

hipError_t mg_launch_restack_window(const uint8_t *recv, int32_t world, int32_t n, int64_t stride, int64_t off_a,
                                    int64_t off_e, int64_t off_d, int32_t preproc, int64_t step, int32_t all_fresh,
                                    int32_t K, uint8_t *ring, hipStream_t st);

int mg_restack_window(const uint8_t *recv, int32_t world, int32_t n, int64_t rank_stride, int64_t off_allo,
                      int64_t off_ego, int64_t off_done, int32_t preproc, int64_t step, int32_t all_fresh, int32_t K,
                      uint8_t *ring, void *stream) {
    if (!recv || !ring || world <= 0 || n <= 0 || step < 0) return set_err(-22, "mg_restack_window: null argument or bad size");
    if (K < 4 || K > 64) return set_err(-22, "mg_restack_window: K must be in [4, 64]");
    if (preproc != MG_PREPROC_LORES4E && preproc != MG_PREPROC_LORESSTACK && preproc != MG_PREPROC_LORES4A)
        return set_err(-22, "mg_restack_window: preproc must be 1 (LoRes4E), 2 (LoResStack) or 4 (LoRes4A); "
                            "LoRes3EA's stack is not one ring's window (use mg_restack)");
    if ((int64_t)world * n * (MG_LORES * MG_LORES / 16) >= ((int64_t)1 << 31))
        return set_err(-22, "mg_restack_window: world * n too large for one launch");
    const int64_t FR = (int64_t)MG_LORES * MG_LORES * 3;
    if (off_allo < 0 || off_ego < 0 || off_done < 0 || off_allo + n * FR > rank_stride || off_ego + n * FR > rank_stride ||
        off_done + n > rank_stride)
        return set_err(-22, "mg_restack_window: a key of the rank block lies outside rank_stride");
    const int64_t al[5] = {(int64_t)(uintptr_t)recv, rank_stride, off_allo, off_ego, (int64_t)(uintptr_t)ring};
    for (int64_t a : al)
        if (a & 15) return set_err(-22, "mg_restack_window: recv, ring, rank_stride and frame offsets must be 16-byte aligned");
    HIPC(mg_launch_restack_window(recv, world, n, rank_stride, off_allo, off_ego, off_done, preproc, step, all_fresh, K,
                                  ring, as_stream(stream)));
    return 0;
}

int mg_bind_window(mg_sim *s, uint8_t *ring_allo, uint8_t *ring_ego, int32_t K) {
    if (!s) return set_err(-22, "mg_bind_window: null sim");
    // outputs bound while rings were on may leave the stacked outputs null (mg_bind_outputs): turning the rings
    // off, or changing which views have one, would then make the next render write its stacks through null
    // pointers -- refuse until outputs with the stacks are bound
    if (s->bound && !s->out.frames_only) {
        const int pp = s->preproc;
        const bool lost = pp == MG_PREPROC_LORESSTACK ? ((!ring_allo && !s->out.obs_allo) || (!ring_ego && !s->out.obs_ego))
                        : pp == MG_PREPROC_LORES4E    ? (!ring_ego && !s->out.obs_past)
                        : pp == MG_PREPROC_LORES4A    ? (!ring_allo && !s->out.obs_past) : false;
        if (lost)
            return set_err(-22, "mg_bind_window: a stacked view would have neither a ring nor an output buffer (the "
                                "bound outputs' stacks are null); bind outputs with the stacks (mg_bind_outputs) first");
    }
    if (!ring_allo && !ring_ego) { s->wring[0] = s->wring[1] = nullptr; s->wK = 0; return 0; }
    if (K < 4 || K > 64) return set_err(-22, "mg_bind_window: K must be in [4, 64]");
    const int pp = s->preproc;
    const bool want_a = pp == MG_PREPROC_LORESSTACK || pp == MG_PREPROC_LORES4A;
    const bool want_e = pp == MG_PREPROC_LORESSTACK || pp == MG_PREPROC_LORES4E;
    if (!want_a && !want_e)
        return set_err(-22, "mg_bind_window: preproc must be 1 (LoRes4E), 2 (LoResStack) or 4 (LoRes4A)");
    if ((ring_allo != nullptr) != want_a || (ring_ego != nullptr) != want_e)
        return set_err(-22, "mg_bind_window: a ring for each stacked view (LoResStack: allo and ego; LoRes4E: ego; "
                            "LoRes4A: allo) and none for the others");
    if (((uintptr_t)ring_allo | (uintptr_t)ring_ego) & 15) return set_err(-22, "mg_bind_window: rings must be 16-byte aligned");
    s->wring[0] = ring_allo; s->wring[1] = ring_ego; s->wK = K;
    return 0;
}

int mg_window_start(const mg_sim *s, int32_t *slot) {
    if (!s || !slot) return set_err(-22, "mg_window_start: null argument");
    *slot = s->wK > 0 ? (int32_t)((s->wstep + s->wK - 3) % s->wK) : -1;
    return 0;
}

int mg_render_full(mg_sim *s, uint8_t *out, void *stream) {
    if (!s || !out) return set_err(-22, "mg_render_full: null argument");
    HIPC(hipSetDevice(s->device));
    RenderOut ro;
    memset(&ro, 0, sizeof(ro));
    ro.full = out;
    ro.preproc = s->preproc;
    ro.small = s->task == MG_TASK_MOVE_TO_REGION || s->task == MG_TASK_MOVE_TO_CORNER;
    ro.first_level = s->task == MG_TASK_CLUSTER_COLOUR ? 0 : 1;   // render class chain start (mg_raster.hip)
    ro.force_retry = s->force_render_retry;
    HIPC(mg_launch_render(s->S, s->dlib, ro, 1, as_stream(stream)));
    return 0;
}

int mg_get_bodies(mg_sim *s, double *out, int32_t *counts, void *stream) {
    if (!s || !out) return set_err(-22, "mg_get_bodies: null argument");
    HIPC(hipSetDevice(s->device));
    hipLaunchKernelGGL(bodies_kernel, dim3(grid64(s)), dim3(64), 0, as_stream(stream), s->S, out, counts);
    HIPC(hipGetLastError());
    return 0;
}

int mg_get_arbiters(mg_sim *s, double *out, uint64_t *hash, void *stream) {
    if (!s || !out || !hash) return set_err(-22, "mg_get_arbiters: null argument");
    HIPC(hipSetDevice(s->device));
    hipLaunchKernelGGL(arbiters_kernel, dim3(grid64(s)), dim3(64), 0, as_stream(stream), s->S, out, hash);
    HIPC(hipGetLastError());
    return 0;
}

int mg_selftest_sincos(const double *x, double *s_out, double *c_out, int n, void *stream) {
    if (!x || !s_out || !c_out || n < 0) return set_err(-22, "mg_selftest_sincos: bad argument");
    if (n == 0) return 0;
    hipLaunchKernelGGL(sincos_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), x, s_out, c_out, n);
    HIPC(hipGetLastError());
    return 0;
}

// pymunk Body.angle / Body.position setters (as geom.pm_shift_bodies applies them): parity tests
__global__ void set_body_pose_kernel(MGState S, int e, int b, double x, double y, double a) {
    body_set_angle(S, e, b, a);
    const double c = AT(S.brc, b), sn = AT(S.brs, b);
    AT(S.bpx, b) = (c * 0.0 + (-sn) * 0.0) + x; // cpBodySetPosition: p = T(cog = 0) + position
    AT(S.bpy, b) = (sn * 0.0 + c * 0.0) + y;
}

int mg_set_body_pose(mg_sim *s, int env, int body, double x, double y, double angle, void *stream) {
    if (!s || env < 0 || env >= s->S.n_envs || body < 0 || body >= MG_MAX_BODIES)
        return set_err(-22, "mg_set_body_pose: bad argument");
    HIPC(hipSetDevice(s->device));
    hipLaunchKernelGGL(set_body_pose_kernel, dim3(1), dim3(1), 0, as_stream(stream), s->S, env, body, x, y, angle);
    HIPC(hipGetLastError());
    return 0;
}

int mg_get_errors(mg_sim *s, int32_t *out, void *stream) {
    if (!s || !out) return set_err(-22, "mg_get_errors: null argument");
    HIPC(hipSetDevice(s->device));
    hipLaunchKernelGGL(errors_kernel, dim3(grid64(s)), dim3(64), 0, as_stream(stream), s->S, out);
    HIPC(hipGetLastError());
    return 0;
}

int mg_random_actions(mg_sim *s, uint8_t *actions, uint64_t key, uint64_t step, void *stream) {
    if (!s || !actions) return set_err(-22, "mg_random_actions: null argument");
    HIPC(hipSetDevice(s->device));
    hipLaunchKernelGGL(actions_kernel, dim3((s->S.n_envs + 255) / 256), dim3(256), 0, as_stream(stream), actions,
                       s->S.n_envs, key, step);
    HIPC(hipGetLastError());
    return 0;
}

int mg_num_envs(const mg_sim *s) { return s ? s->S.n_envs : -22; }

int mg_step_form(const mg_sim *s, int32_t *out) {
    if (!s || !out) return set_err(-22, "mg_step_form: null argument");
    out[0] = s->step_variant; out[1] = s->step_blk;
    out[2] = s->caps.nb; out[3] = s->caps.ns; out[4] = s->caps.nc; out[5] = s->caps.na;
    if (s->step_variant == 5 || s->step_variant == 6) {   // the quad forms' compile-time caps (mg_stepk.h)
        const int q[2][4] = {{6, 5, 10, 20}, {7, 6, 12, 32}};
        for (int k = 0; k < 4; k++) out[2 + k] = q[s->step_variant - 5][k];
    } else if (s->step_variant != 0) {
        const StepCaps c = step_variant_caps(s->step_variant);
        out[2] = c.nb; out[3] = c.ns; out[4] = c.nc; out[5] = c.na;
    }
    return 0;
}

__global__ void __launch_bounds__(64) set_episode_steps_kernel(MGState S, const int32_t *steps) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < S.n_envs) S.episode_steps[e] = steps[e];
}

int mg_set_episode_steps(mg_sim *s, const int32_t *steps, void *stream) {
    if (!s || !steps) return set_err(-22, "mg_set_episode_steps: null argument");
    HIPC(hipSetDevice(s->device));
    hipLaunchKernelGGL(set_episode_steps_kernel, dim3(grid64(s)), dim3(64), 0, as_stream(stream), s->S, steps);
    HIPC(hipGetLastError());
    return 0;
}

int mg_enable_timing(mg_sim *s, int max_steps) {
    if (!s) return set_err(-22, "mg_enable_timing: null sim");
    HIPC(hipSetDevice(s->device));
    for (hipEvent_t e : s->ev) HIPC(hipEventDestroy(e));
    s->ev.clear();
    s->ev_used = 0;
    s->timing = max_steps > 0;
    for (int i = 0; i < 4 * max_steps; i++) {
        hipEvent_t e;
        HIPC(hipEventCreate(&e));
        s->ev.push_back(e);
    }
    return 0;
}

int mg_read_timing(mg_sim *s, double *out) {
    if (!s || !out) return set_err(-22, "mg_read_timing: null argument");
    double t_step = 0.0, t_render = 0.0, t_reset = 0.0;
    int n = (int)(s->ev_used / 4);
    for (int i = 0; i < n; i++) {
        float a = 0.f, b = 0.f, c = 0.f;
        const hipEvent_t *ev = &s->ev[4 * i];
        HIPC(hipEventSynchronize(ev[3]));
        HIPC(hipEventElapsedTime(&a, ev[0], ev[1]));
        HIPC(hipEventElapsedTime(&c, ev[1], ev[2]));
        HIPC(hipEventElapsedTime(&b, ev[2], ev[3]));
        t_step += a; t_render += b; t_reset += c;
    }
    out[0] = t_step; out[1] = t_render; out[2] = n; out[3] = t_reset;
    s->ev_used = 0;
    return 0;
}

void mg_destroy(mg_sim *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    for (hipEvent_t e : s->ev) (void)hipEventDestroy(e);
    if (s->side) {
        (void)hipStreamSynchronize(s->side);
        (void)hipEventDestroy(s->ev_copied); (void)hipEventDestroy(s->ev_prepared);
        (void)hipStreamDestroy(s->side);
        (void)hipFree(s->shadow_pool); (void)hipFree(s->rows); (void)hipFree(s->pend);
    }
    (void)hipFree(s->pool);
    (void)hipFree(s->dlib);
    (void)hipFree(s->reset_mask);
    delete s;
}

} // extern "C"
