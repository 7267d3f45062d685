// mg_physics.hip -- physics kernels: seed (MT19937 per env), reset (BaseEnv.reset +
// on_reset), step (action decode, 10 x [Robot.update + cpSpaceStep], episode
// counter, score, in-place reset of finished episodes).  One env per lane.
#include "mg_launch.h"
#include "mg_reset.h"
#include "mg_score.h"

__global__ void __launch_bounds__(64) seed_kernel(MGState S, const uint32_t *__restrict__ seeds) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= S.n_envs) return;
    mt_seed(S, e, seeds[e]);
}

__global__ void __launch_bounds__(64) reset_kernel(MGState S, const mg_library *__restrict__ L, TaskCfg cfg,
                                                   const uint8_t *__restrict__ mask) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= S.n_envs) return;
    if (mask && !mask[e]) return;
    reset_env(S, L, e, cfg);
}

__global__ void __launch_bounds__(64) step_kernel(MGState S, const mg_library *__restrict__ L, TaskCfg cfg, int max_steps,
                                                  int auto_reset, const uint8_t *__restrict__ actions, float *reward,
                                                  uint8_t *done, double *eval_score) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= S.n_envs) return;
    int a = actions[e];
    robot_set_action(S, L, e, a < 18 ? a : 0);
    const double dt = L->dt;
    MGProf P;
    MG_PP_INIT(P);
    for (int i = 0; i < 10; i++) {
        robot_update(S, L, e);
        MG_PP(P, 0);
        space_step(S, L, e, dt, P);
    }
    int steps = S.episode_steps[e] + 1;
    S.episode_steps[e] = steps;
    bool d = max_steps > 0 && steps >= max_steps;
    double sc = d ? score_env(S, L, e, cfg.task) : 0.0;
    if (reward) reward[e] = (float)sc;
    if (done) done[e] = d ? 1 : 0;
    if (eval_score) eval_score[e] = sc;
    if (d && auto_reset) reset_env(S, L, e, cfg); // VecEnv auto-reset: next obs is the new episode's first frame
    MG_PP(P, 7);
    MG_PP_END(P, (threadIdx.x & 63) == 0, 32);
}


static int grid64(const MGState &S) { return (S.n_envs + 63) / 64; }

hipError_t mg_launch_seed(const MGState &S, const uint32_t *seeds_dev, hipStream_t st) {
    hipLaunchKernelGGL(seed_kernel, dim3(grid64(S)), dim3(64), 0, st, S, seeds_dev);
    return hipGetLastError();
}

hipError_t mg_launch_reset(const MGState &S, const mg_library *L, TaskCfg cfg, const uint8_t *mask, hipStream_t st) {
    hipLaunchKernelGGL(reset_kernel, dim3(grid64(S)), dim3(64), 0, st, S, L, cfg, mask);
    return hipGetLastError();
}

hipError_t mg_launch_step(const MGState &S, const mg_library *L, TaskCfg cfg, int max_steps, int auto_reset,
                          const uint8_t *actions, float *reward, uint8_t *done, double *eval_score, hipStream_t st) {
    hipLaunchKernelGGL(step_kernel, dim3(grid64(S)), dim3(64), 0, st, S, L, cfg, max_steps, auto_reset, actions, reward,
                       done, eval_score);
    return hipGetLastError();
}

hipError_t mg_prof_read_physics(unsigned long long *out) {
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
