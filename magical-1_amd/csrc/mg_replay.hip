// mg_replay.hip -- demo replay through the LoRes observation stages.
//
// Replaces saved_trajectories.py:63-149 (_MockDemoEnv replaying stored observations through
// preprocess_demos_with_wrapper) for the LoRes preprocessors of benchmarks/__init__.py:232-307:
// FlattenFrameStack / EagerDictFrameStack (:51-147; a trajectory's reset frame fills every stack slot)
// and cv2.resize(INTER_AREA) to 96^2 (:150-190, the 4x area case: round-half-even of sum / 16).
// Input: the trajectories' 384^2 (allo, ego) frames, concatenated, already on the device.  Two passes,
// both HBM-bound byte work: (1) every frame's two views downsampled once into a workspace, (2) each
// frame's outputs assembled from the workspace frames its stacks reach back to (clamped to the first
// frame of its trajectory).
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mg_common.h"

namespace {
constexpr int RES = MG_RES, LO = MG_LORES;
constexpr size_t LOFR = (size_t)LO * LO * 3;   // bytes of one 96^2 RGB frame

// round-half-even of s / 16 (cv2 resizeAreaFast: saturate_cast<uchar>(sum * (1.f / 16)))
__device__ __forceinline__ uint32_t area16(uint32_t s) {
    const uint32_t q = s >> 4, r = s & 15;
    return q + (r > 8 || (r == 8 && (q & 1)));
}

// pass 1: one thread per 4 LoRes pixels of one view (16 input pixels per row = 48 B = 3 x 16 B per row)
__global__ __launch_bounds__(256) void replay_downsample_kernel(const uint8_t *__restrict__ frames, int64_t nviews,
                                                                uint8_t *__restrict__ lo) {
    constexpr int QPR = LO / 4;                        // pixel quads per LoRes row
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t fv = gid / (LO * QPR);
    if (fv >= nviews) return;
    const int rem = (int)(gid % (LO * QPR)), oy = rem / QPR, q = rem % QPR;
    const uint8_t *src = frames + (size_t)fv * RES * RES * 3 + ((size_t)(4 * oy) * RES + 16 * q) * 3;
    uint32_t sum[12];
#pragma unroll
    for (int i = 0; i < 12; i++) sum[i] = 0;
#pragma unroll
    for (int dy = 0; dy < 4; dy++) {
        const uint4 *row = (const uint4 *)(src + (size_t)dy * RES * 3);
        const uint4 a = row[0], b = row[1], c = row[2];
        const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
        for (int k = 0; k < 48; k++) {               // byte k: input pixel k / 3 (-> output k / 12), channel k % 3
            const uint32_t byte = (w[k / 4] >> (8 * (k % 4))) & 255u;
            sum[(k / 12) * 3 + k % 3] += byte;
        }
    }
    uint32_t o[3] = {0, 0, 0};
#pragma unroll
    for (int i = 0; i < 12; i++) o[i / 4] |= area16(sum[i]) << (8 * (i % 4));
    uint32_t *dst = (uint32_t *)(lo + (size_t)fv * LOFR + ((size_t)oy * LO + 4 * q) * 3);
    dst[0] = o[0]; dst[1] = o[1]; dst[2] = o[2];
}

// Stacked outputs concatenate, per pixel, the frames oldest..newest (3 bytes each): f[k] holds 4 pixels
// (3 dwords) of stack slot k, written as 3 x 16 B.
__device__ __forceinline__ void stack_pack(const uint32_t (&f)[4][3], uint4 (&d)[3]) {
#pragma unroll
    for (int q = 0; q < 3; q++) {
        uint32_t o[4];
#pragma unroll
        for (int bb = 0; bb < 16; bb++) {  // output byte b: pixel b / 12, slot (b % 12) / 3, channel b % 3
            const int b = 16 * q + bb, px = b / 12, k = (b % 12) / 3, sb = 3 * px + b % 3;
            const uint32_t byte = (f[k][sb / 4] >> (8 * (sb % 4))) & 255u;
            if (bb % 4 == 0) o[bb / 4] = byte; else o[bb / 4] |= byte << (8 * (bb % 4));
        }
        d[q] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}
__device__ __forceinline__ void stack_regs(const uint32_t (&f)[4][3], uint8_t *dst) {
    uint4 d[3];
    stack_pack(f, d);
    uint4 *o = (uint4 *)dst;
#pragma unroll
    for (int q = 0; q < 3; q++) o[q] = d[q];
}

// pass 2: one thread per 4 pixels of one frame; src[k] is the workspace frame of stack slot k.
__device__ __forceinline__ void stack4(const uint8_t *const src[4], size_t pix_off, uint8_t *dst) {
    uint32_t f[4][3];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int w = 0; w < 3; w++) f[k][w] = ((const uint32_t *)(src[k] + pix_off))[w];
    stack_regs(f, dst);
}

__global__ __launch_bounds__(256) void replay_assemble_kernel(const uint8_t *__restrict__ lo,
                                                              const int32_t *__restrict__ episode_start,
                                                              int32_t nframes, int32_t preproc, uint8_t *out_allo,
                                                              uint8_t *out_ego, uint8_t *out_past) {
    constexpr int Q = LO * LO / 4;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int f = (int)(gid / Q), q = (int)(gid % Q);
    if (f >= nframes) return;
    const int s0 = episode_start[f];
    const size_t po = (size_t)q * 12;                  // byte offset of this quad in a 96^2 RGB frame
    auto view = [&](int frame, int v) { return lo + ((size_t)frame * 2 + v) * LOFR; };
    auto back = [&](int k) { const int g = f - k; return g > s0 ? g : s0; };  // deque filled at reset
    if (preproc == MG_PREPROC_LORESSTACK) {            // ResizeDictObservation then EagerDictFrameStack(4)
        for (int v = 0; v < 2; v++) {
            const uint8_t *src[4] = {view(back(3), v), view(back(2), v), view(back(1), v), view(f, v)};
            stack4(src, po, (v ? out_ego : out_allo) + (size_t)f * LOFR * 4 + po * 4);
        }
        return;
    }
    // FlattenFrameStack then resize: allo / ego are the current frames, past_obs the stacks
    const uint32_t *a32 = (const uint32_t *)(view(f, 0) + po), *g32 = (const uint32_t *)(view(f, 1) + po);
    uint32_t *oa = (uint32_t *)(out_allo + (size_t)f * LOFR + po), *og = (uint32_t *)(out_ego + (size_t)f * LOFR + po);
#pragma unroll
    for (int w = 0; w < 3; w++) { oa[w] = a32[w]; og[w] = g32[w]; }
    const uint8_t *src[4];
    if (preproc == MG_PREPROC_LORES4A) {               // allo depth 4, ego depth 0
        for (int k = 0; k < 4; k++) src[k] = view(back(3 - k), 0);
    } else if (preproc == MG_PREPROC_LORES3EA) {       // allo depth 1, then ego depth 3
        src[0] = view(f, 0);
        for (int k = 1; k < 4; k++) src[k] = view(back(3 - k), 1);
    } else {                                           // LoRes4E / LoResCHW4E / LoResCHW4A: ego depth 4
        for (int k = 0; k < 4; k++) src[k] = view(back(3 - k), 1);
    }
    stack4(src, po, out_past + (size_t)f * LOFR * 4 + po * 4);
}

// Receiver-side frame stacks of the compact multi-GPU gather (mg_restack, magical_amd.dist): one thread per
// 4 pixels of one env and one output stack (blockIdx.y: LoResStack 0 allo / 1 ego; else 0 = past_obs).
// The ring view of the stack keeps the env's last 4 frames (slot t % 4 = this step); a fresh env (reset,
// or done = auto-reset) fills every slot with its current frame, as the deques of
// benchmarks/__init__.py:75-82,139-147 are filled at reset.  Byte work: per env and stack 12 B read (+ 36 B
// of ring unless fresh), 12 B ring write and 48 B stacked output per 4 pixels -- HBM bound.
// The 48 output bytes of a thread's 4 pixels go through LDS (LDSST, the default): the workgroup's 256
// threads cover 1024 consecutive pixels of one env (a frame is 9 x 1024 pixels), so its stacked output is
// 12 KB of contiguous memory, stored as 3 fully coalesced 16-byte-per-lane rounds instead of 3 stores of
// 16 B at a 48 B lane stride.  (A 16-pixel form with 16-byte accesses measured 5x slower, round 4: each
// store instruction then writes 16 B into 64 different cache lines, 192 B apart.)
template <bool LDSST>
__global__ __launch_bounds__(256) void restack_kernel(const uint8_t *__restrict__ recv, uint32_t world, uint32_t n,
                                                      int64_t stride, int64_t off_a, int64_t off_e, int64_t off_d,
                                                      int32_t preproc, uint32_t slot, int32_t all_fresh,
                                                      uint8_t *__restrict__ ring, uint8_t *__restrict__ out0,
                                                      uint8_t *__restrict__ out1) {
    constexpr uint32_t Q = LO * LO / 4;
    static_assert(Q % 256 == 0, "a workgroup's 256 pixel quads stay inside one env");
    __shared__ uint4 st[LDSST ? 3 * 256 : 1];
    const uint32_t W = world * n;
    const int s = blockIdx.y;
    uint8_t *const out = s ? out1 : out0;
    // grid-stride (a capped grid leaves the SIMDs' register files to the simulator's kernels, MG_RESTACK_WGS);
    // W * Q is a multiple of 256, so every thread of a workgroup runs the same trips
    for (uint32_t gid = blockIdx.x * 256u + threadIdx.x; gid < W * Q; gid += gridDim.x * 256u) {
        const uint32_t g = gid / Q, q = gid - g * Q;
        const uint32_t r = g / n, i = g - r * n;
        const uint8_t *blk = recv + (size_t)r * stride;
        const bool fresh = all_fresh || blk[off_d + i] != 0;
        // the view this stack's frames come from (LoRes3EA: ego, with the current allo frame in slot 0)
        const int rv = (preproc == MG_PREPROC_LORES4A || (preproc == MG_PREPROC_LORESSTACK && s == 0)) ? 0 : 1;
        const size_t po = (size_t)q * 12;
        const uint32_t *cur = (const uint32_t *)(blk + (rv ? off_e : off_a) + (size_t)i * LOFR + po);
        uint8_t *rring = ring + (size_t)s * 4 * W * LOFR;   // one ring per output stack (LoResStack: 2, else 1)
        auto rslot = [&](uint32_t sl) { return (uint32_t *)(rring + ((size_t)(sl & 3) * W + g) * LOFR + po); };
        uint32_t f[4][3];
#pragma unroll
        for (int w = 0; w < 3; w++) f[3][w] = cur[w];
        if (fresh) {
#pragma unroll
            for (int k = 0; k < 3; k++)
#pragma unroll
                for (int w = 0; w < 3; w++) f[k][w] = f[3][w];
#pragma unroll
            for (uint32_t sl = 0; sl < 4; sl++) {
                uint32_t *d = rslot(sl);
                d[0] = f[3][0]; d[1] = f[3][1]; d[2] = f[3][2];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 3; k++) {          // stack slot k = frame t - (3 - k)
                const uint32_t *src = rslot(slot + 1 + k);
#pragma unroll
                for (int w = 0; w < 3; w++) f[k][w] = src[w];
            }
            uint32_t *d = rslot(slot);
            d[0] = f[3][0]; d[1] = f[3][1]; d[2] = f[3][2];
        }
        if (preproc == MG_PREPROC_LORES3EA) {      // allo depth 1 in front of the ego frames t-2, t-1, t
            const uint32_t *a = (const uint32_t *)(blk + off_a + (size_t)i * LOFR + po);
#pragma unroll
            for (int w = 0; w < 3; w++) f[0][w] = a[w];
        }
        if constexpr (LDSST) {
            uint4 d[3];
            stack_pack(f, d);
            const uint32_t t = threadIdx.x;
#pragma unroll
            for (int k = 0; k < 3; k++) st[3 * t + k] = d[k];
            __syncthreads();
            // the workgroup's quads q0 .. q0 + 255 of env g: 12 KB of output from q0 * 48 on
            uint4 *dst = (uint4 *)(out + (size_t)g * LOFR * 4 + (size_t)(q - t) * 48);
#pragma unroll
            for (int k = 0; k < 3; k++) dst[t + 256 * k] = st[t + 256 * k];
            __syncthreads();
        } else {
            stack_regs(f, out + (size_t)g * LOFR * 4 + po * 4);
        }
    }
}

// Receiver-side frame stacks as a window ring (mg_restack_window, round 5): instead of materialising every
// env's [96][96][12] stack each step (read the current frame + 3 ring frames, write 1 ring frame + 4 stack
// frames: 9 frame passes), each received frame is written once, channel-planar ([3][96][96]), into a ring of
// K + 3 slots per env and stack: frame f goes to slot f % K, and the frames with f % K < 3 also to slot
// K + f % K.  The 4 frames t-3 .. t then sit in the 4 consecutive slots from s0 = (t - 3) mod K on, for every
// env, so the stack of step t is a strided view of the ring (channel k = 4-frame slot k / 3, plane k % 3:
// channel stride 96 * 96, pixel strides 96 / 1) -- the host returns it with as_strided, no copy.  Per env-step
// and stacked view: 1 frame read, 1 + 3 / K frames written.  A fresh env (reset, or done = auto-reset) writes
// its frame into the slots of frames t-3 .. t (the deques of benchmarks/__init__.py:75-82,139-147 are filled
// with the reset frame).  One thread per 16 pixels: 3 x 16 B loads of HWC bytes, 3 x 16 B planar stores
// (consecutive lanes store consecutive 16 B of a plane: fully coalesced).
__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[12], int k) { return (w[k >> 2] >> (8 * (k & 3))) & 255u; }

__global__ __launch_bounds__(256) void restack_window_kernel(const uint8_t *__restrict__ recv, uint32_t world,
                                                             uint32_t n, int64_t stride, int64_t off_a, int64_t off_e,
                                                             int64_t off_d, int32_t preproc, int64_t step,
                                                             int32_t all_fresh, uint32_t K, uint8_t *__restrict__ ring) {
    constexpr uint32_t PL = LO * LO;          // bytes of one colour plane
    constexpr uint32_t Q = PL / 16;           // 16-pixel groups per frame
    const uint32_t WN = world * n;
    const int s = blockIdx.y;                 // output stack (LoResStack: 0 allo / 1 ego; else 0)
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    if (gid >= WN * Q) return;
    const uint32_t g = gid / Q, q = gid - g * Q;
    const uint32_t r = g / n, i = g - r * n;
    const uint8_t *blk = recv + (size_t)r * stride;
    const bool fresh = all_fresh || blk[off_d + i] != 0;
    const int rv = (preproc == MG_PREPROC_LORES4A || (preproc == MG_PREPROC_LORESSTACK && s == 0)) ? 0 : 1;
    const uint4 *cur = (const uint4 *)(blk + (rv ? off_e : off_a) + (size_t)i * LOFR + (size_t)q * 48);
    uint32_t w[12];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint4 v = cur[k];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
    uint4 pl[3];                              // plane c, pixels 16q .. 16q + 15
#pragma unroll
    for (int c = 0; c < 3; c++) {
        uint32_t o[4];
#pragma unroll
        for (int d = 0; d < 4; d++)
            o[d] = byte_of(w, 3 * (4 * d) + c) | byte_of(w, 3 * (4 * d + 1) + c) << 8 |
                   byte_of(w, 3 * (4 * d + 2) + c) << 16 | byte_of(w, 3 * (4 * d + 3) + c) << 24;
        pl[c] = make_uint4(o[0], o[1], o[2], o[3]);
    }
    uint8_t *env_ring = ring + ((size_t)s * WN + g) * (K + 3) * LOFR + (size_t)q * 16;
    auto put = [&](uint32_t slot) {
#pragma unroll
        for (int c = 0; c < 3; c++) *(uint4 *)(env_ring + (size_t)slot * LOFR + (size_t)c * PL) = pl[c];
    };
    const uint32_t p = (uint32_t)(step % K);
    for (uint32_t j = 0; j < (fresh ? 4u : 1u); j++) {   // frames t, t-1, t-2, t-3 (fresh: all four slots)
        const uint32_t f = (p + K - j) % K;
        put(f);
        if (f < 3) put(K + f);
    }
}

}  // namespace

extern "C" hipError_t mg_launch_restack_window(const uint8_t *recv, int32_t world, int32_t n, int64_t stride,
                                               int64_t off_a, int64_t off_e, int64_t off_d, int32_t preproc,
                                               int64_t step, int32_t all_fresh, int32_t K, uint8_t *ring,
                                               hipStream_t st) {
    const int64_t t = (int64_t)world * n * (LO * LO / 16);
    const bool two = preproc == MG_PREPROC_LORESSTACK;
    hipLaunchKernelGGL(restack_window_kernel, dim3((unsigned)((t + 255) / 256), two ? 2 : 1), dim3(256), 0, st, recv,
                       (uint32_t)world, (uint32_t)n, stride, off_a, off_e, off_d, preproc, step, all_fresh,
                       (uint32_t)K, ring);
    return hipGetLastError();
}

// launcher, C linkage (declared in mg_sim.hip next to the ABI entry mg_replay_lores)
extern "C" hipError_t mg_launch_replay(const uint8_t *frames, int32_t nframes, const int32_t *episode_start,
                                       int32_t preproc, uint8_t *scratch, uint8_t *out_allo, uint8_t *out_ego,
                                       uint8_t *out_past, hipStream_t st) {
    const int64_t nviews = (int64_t)nframes * 2;
    const int64_t t1 = nviews * LO * (LO / 4);
    hipLaunchKernelGGL(replay_downsample_kernel, dim3((unsigned)((t1 + 255) / 256)), dim3(256), 0, st, frames, nviews,
                       scratch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t t2 = (int64_t)nframes * (LO * LO / 4);
    hipLaunchKernelGGL(replay_assemble_kernel, dim3((unsigned)((t2 + 255) / 256)), dim3(256), 0, st, scratch,
                       episode_start, nframes, preproc, out_allo, out_ego, out_past);
    return hipGetLastError();
}

extern "C" hipError_t mg_launch_restack(const uint8_t *recv, int32_t world, int32_t n, int64_t stride, int64_t off_a,
                                        int64_t off_e, int64_t off_d, int32_t preproc, int64_t step, int32_t all_fresh,
                                        uint8_t *ring, uint8_t *out_allo, uint8_t *out_ego, uint8_t *out_past,
                                        hipStream_t st) {
    const int64_t t = (int64_t)world * n * (LO * LO / 4);
    const bool two = preproc == MG_PREPROC_LORESSTACK;
    int64_t wgs = (t + 255) / 256;
    static const int64_t cap = getenv("MG_RESTACK_WGS") ? atoll(getenv("MG_RESTACK_WGS")) : 0;   // experiments
    if (cap > 0 && wgs > cap) wgs = cap;
    // A/B: MG_RESTACK_LDS=0 direct 16-byte stores at a 48-byte lane stride.  (A form staging every load
    // through LDS as well -- 192 lanes x 16 B per frame chunk -- measured no faster, round 4: 2.13 vs 2.06 ms
    // MoveToRegion, 10.5 vs 9.9 ms ClusterColour at 8 emulated ranks.)
    static const bool lds = !getenv("MG_RESTACK_LDS") || atoi(getenv("MG_RESTACK_LDS")) != 0;
    hipLaunchKernelGGL(lds ? restack_kernel<true> : restack_kernel<false>, dim3((unsigned)wgs, two ? 2 : 1),
                       dim3(256), 0, st, recv, (uint32_t)world, (uint32_t)n, stride, off_a, off_e, off_d, preproc,
                       (uint32_t)(step & 3), all_fresh, ring, two ? out_allo : out_past, out_ego);
    return hipGetLastError();
}
