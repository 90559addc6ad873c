// Probe: VALU fp32 FMA throughput per SIMD with 1, 2, 4 waves per SIMD (independent chains).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int W>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
    float a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
    const float b = 1.0001f, c = 0.0001f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = fmaf(a[i], b, c);
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i];
    if (s == 1234.5f) out[threadIdx.x] = s;
}
int main() {
    float* d;
    hipMalloc(&d, 4096);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int iters = 20000;
    for (int wps = 1; wps <= 4; wps *= 2) {
        // 256 threads = 4 waves per WG (1 per SIMD); wps WGs per CU
        const int grid = cus * wps;
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, d, 10);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, d, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double fma = (double)grid * 256 * iters * 16 * 8;
        const double clk = p.clockRate * 1e3;   // Hz
        const double per_simd_cycles = ms * 1e-3 * clk;
        const double instr_per_simd = (double)wps * iters * 16 * 8;   // wave-instructions per SIMD
        printf("waves/SIMD %d: %.3f ms, %.1f TFMA/s, %.2f cycles per wave-instruction per SIMD (clock %.0f MHz)\n",
               wps, ms, fma / (ms * 1e-3) / 1e12, per_simd_cycles / instr_per_simd, clk / 1e6);
    }
    return 0;
}
