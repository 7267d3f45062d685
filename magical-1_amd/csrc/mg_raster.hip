// mg_raster.hip -- render kernel (one workgroup per (env, view)), see mg_render.h.
#include "mg_launch.h"
#include "mg_render.h"

hipError_t mg_launch_render(const MGState &S, const mg_library *L, const RenderOut &ro, int mode, hipStream_t st) {
    const dim3 grid(S.n_envs, 2), blk(RG_THREADS);
    RenderOut r = ro;
    r.retry_in = r.retry_out = r.cls_level = 0;
    if (mode == 0 && (ro.wring[0] || ro.wring[1]) && !ro.frames_only) mode = 2;   // window rings: own kernels
    if (ro.small) {   // the small class holds every MoveToRegion / MoveToCorner scene
        if (mode == 0) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_SMALL>, 0>), grid, blk, 0, st, S, L, r);
        else if (mode == 2) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_SMALL>, 2>), grid, blk, 0, st, S, L, r);
        else hipLaunchKernelGGL((render_kernel<RenderSmem<RG_SMALL>, 1>), grid, blk, 0, st, S, L, r);
        return hipGetLastError();
    }
    // many-block tasks: a chain of classes, each with more LDS (fewer workgroups per CU) than the last.  A
    // class renders the (env, view) pairs at its chain level (S.rg_retry, kept for the episode); a pair it
    // cannot hold moves to the next level and is rendered by the next class (the others exit at once).
    // Medium-0 (8 workgroups/CU) holds every ClusterColour scene, medium-1 (7) most scenes of the other
    // benchmark tasks, medium-2 (5) nearly all, the large class (3) every scene.
    // Where the chain starts is the task's (first_level): medium-0 holds every ClusterColour scene, but a third
    // of MatchRegions-TestAll's, whose frames then pay a launch more and measured slower (3.30 -> 3.59 ms), so
    // the other tasks start at medium-1.
    r.retry_in = 1; r.retry_out = 1;
    hipError_t e;
    if (r.first_level == 0) {
        if (mode == 0) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM0>, 0>), grid, blk, 0, st, S, L, r);
        else if (mode == 2) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM0>, 2>), grid, blk, 0, st, S, L, r);
        else hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM0>, 1>), grid, blk, 0, st, S, L, r);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    r.cls_level = 1;
    if (mode == 0) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM1>, 0>), grid, blk, 0, st, S, L, r);
    else if (mode == 2) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM1>, 2>), grid, blk, 0, st, S, L, r);
    else hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM1>, 1>), grid, blk, 0, st, S, L, r);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    r.cls_level = 2;
    if (mode == 0) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM2>, 0>), grid, blk, 0, st, S, L, r);
    else if (mode == 2) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM2>, 2>), grid, blk, 0, st, S, L, r);
    else hipLaunchKernelGGL((render_kernel<RenderSmem<RG_MEDIUM2>, 1>), grid, blk, 0, st, S, L, r);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    r.retry_out = 0; r.cls_level = 3;
    if (mode == 0) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_LARGE>, 0>), grid, blk, 0, st, S, L, r);
    else if (mode == 2) hipLaunchKernelGGL((render_kernel<RenderSmem<RG_LARGE>, 2>), grid, blk, 0, st, S, L, r);
    else hipLaunchKernelGGL((render_kernel<RenderSmem<RG_LARGE>, 1>), grid, blk, 0, st, S, L, r);
    return hipGetLastError();
}

// LoRes3EA (benchmarks/__init__.py lores_ea_entry_point: FlattenFrameStack with allo depth 1, ego
// depth 3): past_obs[y][x] = allo_t | ego_t-2 | ego_t-1 | ego_t (12 bytes per pixel). The two views are
// rendered by different workgroups, so this small pass runs after the render kernel and interleaves the
// current allo frame (obs_allo) with the ego ring (slot nh = t, nh-1, nh-2; all slots equal after reset).
// One thread per 4 pixels: 4 x 3 dwords in, 3 x 16 B out.
__global__ __launch_bounds__(256) void compose3ea_kernel(MGState S, const uint8_t *obs_allo, const uint8_t *mask,
                                                         uint8_t *obs_past) {
    constexpr int Q = MG_LORES * MG_LORES / 4;   // pixel quads per frame
    const size_t FR = (size_t)MG_LORES * MG_LORES * 3;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int e = (int)(gid / Q), q = (int)(gid % Q);
    if (e >= S.n_envs || (mask && !mask[e])) return;
    const int nh = S.hist_head[S.N + e];
    const uint32_t *src[4];
    src[0] = (const uint32_t *)(obs_allo + (size_t)e * FR);
    for (int k = 1; k < 4; k++) src[k] = (const uint32_t *)(S.hist_ego + ((size_t)((nh + k + 1) & 3) * S.N + e) * FR);
    uint32_t f[4][3];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int w = 0; w < 3; w++) f[k][w] = src[k][3 * q + w];
    uint32_t o[12];
#pragma unroll
    for (int b = 0; b < 48; b++) {   // output byte b: pixel b / 12, source (b % 12) / 3, channel b % 3
        const int px = b / 12, k = (b % 12) / 3, sb = 3 * px + b % 3;
        const uint32_t byte = (f[k][sb / 4] >> (8 * (sb % 4))) & 255u;
        if (b % 4 == 0) o[b / 4] = byte; else o[b / 4] |= byte << (8 * (b % 4));
    }
    uint4 *dst = (uint4 *)(obs_past + (size_t)e * FR * 4) + 3 * q;
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
    dst[2] = make_uint4(o[8], o[9], o[10], o[11]);
}

hipError_t mg_launch_compose3ea(const MGState &S, const uint8_t *obs_allo, const uint8_t *mask, uint8_t *obs_past,
                                hipStream_t st) {
    const int64_t n = (int64_t)S.n_envs * (MG_LORES * MG_LORES / 4);
    hipLaunchKernelGGL(compose3ea_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, S, obs_allo, mask,
                       obs_past);
    return hipGetLastError();
}

MG_PROF_READER(mg_prof_read_raster)
