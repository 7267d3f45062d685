// mg_step_hbm.hip -- HBM-state step kernel (variant 0)
#include "mg_stepk.h"

template hipError_t launch_step_var<0, 1>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<0, 8>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);
template hipError_t launch_step_var<0, 64>(const MGState &, const mg_library *, TaskCfg, int, int, const uint8_t *, float *, uint8_t *, double *, uint8_t *, hipStream_t);

MG_PROF_READER(mg_prof_read_step_hbm)
