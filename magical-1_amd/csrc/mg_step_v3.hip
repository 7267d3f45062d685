// mg_step_v3.hip -- LDS step kernel with runtime constraint lists, one env per workgroup of 1 or 4 lanes (variant 3)
#include "mg_stepk.h"

template hipError_t launch_step_var<3, 1>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<3, 4>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);

MG_PROF_READER(mg_prof_read_step_v3)
