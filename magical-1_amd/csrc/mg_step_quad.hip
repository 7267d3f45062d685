// mg_step_quad.hip -- step kernel forms of the compile-time robot scenes with 4 lanes per env (5: robot
// only, 6: robot + one block; mg_stepq.h)
#include "mg_stepk.h"

template hipError_t launch_step_var<5, 16>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<6, 16>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
// 8 envs per workgroup (half the LDS): robot-scene grids below 16 envs per CU (mg_sim.hip pick_step_blk)
template hipError_t launch_step_var<5, 8>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<6, 8>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
MG_PROF_READER(mg_prof_read_step_quad)
