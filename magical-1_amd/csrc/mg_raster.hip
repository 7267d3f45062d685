// mg_raster.hip -- render kernel (one workgroup per (env, view)), see mg_render.h.
#include "mg_launch.h"
#include "mg_render.h"

hipError_t mg_launch_render(const MGState &S, const mg_library *L, const RenderOut &ro, int mode, hipStream_t st) {
    if (ro.small)
        hipLaunchKernelGGL(render_kernel<RenderSmem<RG_SMALL>>, dim3(S.n_envs, 2), dim3(RG_THREADS), 0, st, S, L, ro, mode);
    else
        hipLaunchKernelGGL(render_kernel<RenderSmem<RG_LARGE>>, dim3(S.n_envs, 2), dim3(RG_THREADS), 0, st, S, L, ro, mode);
    return hipGetLastError();
}

hipError_t mg_prof_read_raster(unsigned long long *out) {
#ifdef MG_PROFILE
    unsigned long long v[64], z[64] = {0};
    hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_prof), sizeof(v));
    if (e != hipSuccess) return e;
    for (int i = 0; i < 64; i++) out[i] += v[i];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z));
#else
    (void)out;
    return hipSuccess;
#endif
}
