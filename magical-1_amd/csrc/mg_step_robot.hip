// mg_step_robot.hip -- step kernel forms with compile-time constraint lists (variants 1, 2)
#include "mg_stepk.h"

template hipError_t launch_step_var<1, 1>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<1, 4>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<1, 16>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<2, 1>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<2, 4>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<2, 16>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);

MG_PROF_READER(mg_prof_read_step_robot)
