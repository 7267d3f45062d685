// Micro-benchmark: does a wave64 FP64 dependent chain run faster when fewer lanes are active, and does it
// matter WHICH lanes (contiguous 16 in the first half vs spread every 4th)?  One wave per CU (or W waves per
// SIMD), a chain of N dependent v_mul_f64 + v_add_f64 per lane, timed with s_memtime around the chain.
// Output: ticks per chain step for each exec pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(64) chain(double *out, unsigned long long *ticks, int n, int mode, double a, double b) {
    const int lane = threadIdx.x & 63;
    bool act;
    switch (mode) {
    case 0: act = true; break;                 // 64 lanes
    case 1: act = lane < 32; break;            // first half
    case 2: act = lane < 16; break;            // first quarter
    case 3: act = (lane & 3) == 0; break;      // 16 lanes spread (the quad step forms' solver lanes)
    case 4: act = lane == 0; break;            // one lane
    default: act = (lane & 1) == 0; break;     // 32 lanes spread
    }
    double x = out[blockIdx.x * 64 + lane];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (act) {
#pragma unroll 8
        for (int i = 0; i < n; i++) { x = x * a; x = x + b; }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = x;
    if (lane == 0) ticks[blockIdx.x] = t1 - t0;
}

int main(int argc, char **argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 256, n = 1 << 16;
    double *out; unsigned long long *ticks;
    hipMalloc(&out, blocks * 64 * sizeof(double)); hipMalloc(&ticks, blocks * sizeof(unsigned long long));
    hipMemset(out, 0, blocks * 64 * sizeof(double));
    unsigned long long *h = (unsigned long long *)malloc(blocks * sizeof(unsigned long long));
    const char *names[6] = {"64 lanes", "32 lanes (0-31)", "16 lanes (0-15)", "16 lanes (every 4th)", "1 lane", "32 lanes (even)"};
    for (int rep = 0; rep < 2; rep++)
        for (int mode = 0; mode < 6; mode++) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(chain, dim3(blocks), dim3(64), 0, 0, out, ticks, n, mode, 0.999999, 1e-9);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h, ticks, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            double avg = 0; for (int i = 0; i < blocks; i++) avg += h[i]; avg /= blocks;
            if (rep) printf("blocks %d  %-22s  %.3f ms  %.2f ticks/step  (%.3f ns/step by events)\n", blocks, names[mode], ms,
                            avg / n, ms * 1e6 / n);
        }
    return 0;
}
