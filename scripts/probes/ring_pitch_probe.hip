// Probe: time one tick of ring ingest (8192 streams x 1600 floats scattered into
// per-stream rings) as a function of the ring pitch (scripts/probes).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ __launch_bounds__(256) void k_scatter(const float* __restrict__ src, float* __restrict__ dst,
                                                 int64_t pitch, int off, int n_streams) {
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (s >= n_streams) return;
    const float* a = src + (int64_t)s * 1600;
    float* b = dst + (int64_t)s * pitch + off;
    float x[25];
#pragma unroll
    for (int m = 0; m < 25; ++m) x[m] = __builtin_nontemporal_load(a + lane + 64 * m);
#pragma unroll
    for (int m = 0; m < 25; ++m) b[lane + 64 * m] = x[m];
}
int main() {
    const int S = 8192;
    const int64_t pitches[] = {1600, 160000, 160000 + 64, 160000 + 256, 160000 + 1024, 160000 + 1600, 161024, 163840};
    float *src, *dst;
    if (hipMalloc(&src, (size_t)S * 1600 * 4) != hipSuccess) return 1;
    if (hipMalloc(&dst, (size_t)S * 170000 * 4) != hipSuccess) return 1;
    hipMemset(src, 0, (size_t)S * 1600 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int64_t p : pitches) {
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_scatter, dim3(S / 4), dim3(256), 0, 0, src, dst, p, 0, S);
        const int reps = 50;
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(k_scatter, dim3(S / 4), dim3(256), 0, 0, src, dst, p, (int)((r * 1600) % 150000), S);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("pitch %7ld floats (%7ld B): %6.1f us per tick\n", (long)p, (long)p * 4, 1000.0f * ms / reps);
    }
    return 0;
}
