// mg_prof.h -- optional phase timers (build with -DMG_PROFILE; see tools/gpu_phase.py).
// One lane per wave accumulates s_memtime deltas per phase in registers and adds
// them to g_prof at the end; the production build compiles these to nothing.
#pragma once
#ifdef MG_PROFILE
static __device__ unsigned long long g_prof[64]; // one per translation unit
#define MG_PROF_BEGIN(on) const bool _pon = (on); unsigned long long _pt = __builtin_amdgcn_s_memtime(); \
    unsigned long long _pacc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define MG_PROF(i) do { unsigned long long _t = __builtin_amdgcn_s_memtime(); _pacc[i] += _t - _pt; _pt = _t; } while (0)
#define MG_PROF_END(base) do { if (_pon) for (int _i = 0; _i < 16; _i++) if (_pacc[_i]) atomicAdd(&g_prof[(base) + _i], _pacc[_i]); } while (0)
// own-work time of the slowest thread of the workgroup (before a barrier): thread-local start, then
// max into an LDS slot which thread 0 adds to g_prof[slot]
#define MG_PROF_MARK(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#define MG_PROF_MAXW(slotvar, v) atomicMax(&(slotvar), (unsigned int)(__builtin_amdgcn_s_memtime() - (v)))
#else
#define MG_PROF_MARK(v) do { } while (0)
#define MG_PROF_MAXW(slotvar, v) do { } while (0)
#define MG_PROF_BEGIN(on)
#define MG_PROF(i) do { } while (0)
#define MG_PROF_END(base) do { } while (0)
#endif

// host reader of this translation unit's timers: adds them to out[64] and clears them
#ifdef MG_PROFILE
#define MG_PROF_READER(fn)                                                                     \
    hipError_t fn(unsigned long long *out) {                                                   \
        unsigned long long v[64], z[64] = {0};                                                 \
        hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_prof), sizeof(v));                  \
        if (e != hipSuccess) return e;                                                         \
        for (int i = 0; i < 64; i++) out[i] += v[i];                                           \
        return hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z));                            \
    }
#else
#define MG_PROF_READER(fn) \
    hipError_t fn(unsigned long long *out) { (void)out; return hipSuccess; }
#endif

// phase timers threaded through device functions
struct MGProf {
#ifdef MG_PROFILE
    unsigned long long t, acc[16];
#endif
};
#ifdef MG_PROFILE
#define MG_PP_INIT(P) do { (P).t = __builtin_amdgcn_s_memtime(); for (int _i = 0; _i < 16; _i++) (P).acc[_i] = 0; } while (0)
#define MG_PP(P, i) do { unsigned long long _t = __builtin_amdgcn_s_memtime(); (P).acc[i] += _t - (P).t; (P).t = _t; } while (0)
#define MG_PP_END(P, on, base) do { if (on) for (int _i = 0; _i < 16; _i++) if ((P).acc[_i]) atomicAdd(&g_prof[(base) + _i], (P).acc[_i]); } while (0)
#else
#define MG_PP_INIT(P) do { } while (0)
#define MG_PP(P, i) do { } while (0)
#define MG_PP_END(P, on, base) do { } while (0)
#endif
