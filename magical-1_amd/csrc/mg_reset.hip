// mg_reset.hip -- seed (MT19937 per env) and reset (BaseEnv.reset + on_reset, masked) kernels.
// the reset is off the step path (next-layout shadow): one out-of-line collide()
// for its shape queries keeps this unit's compile time bounded (about 1 min instead of 35+)
#define MG_COLLIDE_ATTR __device__ __attribute__((noinline))
#include <cstdlib>
#include "mg_launch.h"
#include "mg_reset.h"
__global__ void __launch_bounds__(64) seed_kernel(MGState S, const uint32_t *__restrict__ seeds) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= S.n_envs) return;
    mt_seed(S, e, seeds[e]);
}

// one env per 64-lane wave: the serial reset runs on every lane (identical values, identical stores),
// the rejection samplers' shape queries are split across the lanes (query_hits)
// waves per SIMD the reset kernels are compiled for (their register cap): uncapped, the generic kernel took a
// SIMD's whole register file (256 VGPR + 256 AGPR), so each of the next-layout shadow's wavefronts waited for a
// SIMD to drain beside the step and render kernels; 4 (128 VGPRs, the rest in scratch) measured MatchRegions
// 1.404 -> 1.423 M env-steps/s, ClusterColour 1.531 -> 1.535 M (profiles/r06_rc)
#ifndef MG_RESET_CAP
#define MG_RESET_CAP 4
#endif
template <int TASK, int LAYOUT>
__global__ void __launch_bounds__(64)
#if MG_RESET_CAP
__attribute__((amdgpu_waves_per_eu(MG_RESET_CAP)))
#endif
reset_kernel(MGState S, const mg_library *__restrict__ L, TaskCfg cfg, const uint8_t *__restrict__ mask) {
    cfg.coop = 1;
    // the env's MT19937 state in LDS for the reset: each draw of the serial rejection samplers is then an LDS
    // round trip, not two dependent HBM ones (mt_pos, the key word), and the twist runs 64 words at a time
    __shared__ uint32_t mt[625];
    const int lane = (int)threadIdx.x;
    MGState V = S;
    V.mt_lds = mt;
    // grid-stride over the envs (a masked launch may run fewer wavefronts than envs: mg_launch_reset)
    for (int e = blockIdx.x; e < S.n_envs; e += gridDim.x) {
        if (mask && !mask[e]) continue;
        for (int i = lane; i < 624; i += 64) mt[i] = S.mt_key[(size_t)i * S.N + e];
        if (lane == 0) mt[624] = (uint32_t)S.mt_pos[e];
        __syncthreads();
        reset_env<TASK, LAYOUT>(V, L, e, cfg);
        __syncthreads();
        for (int i = lane; i < 624; i += 64) S.mt_key[(size_t)i * S.N + e] = mt[i];
        if (lane == 0) S.mt_pos[e] = (int32_t)mt[624];
        __syncthreads();
    }
}

static int grid64(const MGState &S) { return (S.n_envs + 63) / 64; }

hipError_t mg_launch_seed(const MGState &S, const uint32_t *seeds_dev, hipStream_t st) {
    hipLaunchKernelGGL(seed_kernel, dim3(grid64(S)), dim3(64), 0, st, S, seeds_dev);
    return hipGetLastError();
}

// The robot scenes' variants without layout randomisation (MoveToRegion / MoveToCorner Demo and the
// colour / shape / dynamics variants) run a kernel compiled for that task alone: the auto-reset of a step
// is a launch over every env that mostly exits at once, and with the generic kernel's register file (every
// task's samplers, the rejection sampler's collide) each of those wavefronts waited for a whole SIMD to drain
// when the render of another env chunk was running (0.03 ms alone, 0.17 ms beside it).
hipError_t mg_launch_reset(const MGState &S, const mg_library *L, TaskCfg cfg, const uint8_t *mask, hipStream_t st,
                           int max_waves) {
    const bool layout = (cfg.flags & (MG_RAND_LAYOUT_MINOR | MG_RAND_LAYOUT_FULL)) != 0;
    auto k = reset_kernel<-1, -1>;
    if (!layout && cfg.task == MG_TASK_MOVE_TO_REGION) k = reset_kernel<MG_TASK_MOVE_TO_REGION, 0>;
    else if (!layout && cfg.task == MG_TASK_MOVE_TO_CORNER) k = reset_kernel<MG_TASK_MOVE_TO_CORNER, 0>;
    else if (!layout) k = reset_kernel<-1, 0>;   // every other task's variants without layout randomisation
    const int grid = (mask && max_waves > 0 && S.n_envs > max_waves) ? max_waves : S.n_envs;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, st, S, L, cfg, mask);
    return hipGetLastError();
}

MG_PROF_READER(mg_prof_read_reset)
