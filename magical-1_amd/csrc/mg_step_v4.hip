// mg_step_v4.hip -- cooperative LDS step kernel, one env per 64-lane wavefront (variant 4)
#include "mg_stepk.h"

template hipError_t launch_step_var<4, 1>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);

MG_PROF_READER(mg_prof_read_step_v4)
