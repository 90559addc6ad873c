// Probe: where does ds_write_addtid_b32 put its data for a given M0? (scripts/probes)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float* out, uint32_t m0v, int off) {
    __shared__ float s[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) s[i] = -1.0f;
    __syncthreads();
    if (threadIdx.x < 64) {
        float v = (float)threadIdx.x;
        uint32_t sv;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tds_write_addtid_b32 %2 offset:1024\n\ts_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %0"
                     : "=&s"(sv) : "s"(m0v), "v"(v) : "memory");
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) out[i] = s[i];
}
int main() {
    float* d; hipMalloc(&d, 8192 * 4);
    float h[8192];
    uint32_t cases[] = {0u, 4096u, 0xFFFF0000u, 0xFFFF0000u | 4096u, 0x10000u | 4096u, 0xFFFFFFFFu};
    for (uint32_t m : cases) {
        hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, m, 0);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        int first = -1, n = 0;
        for (int i = 0; i < 8192; ++i) if (h[i] != -1.0f) { if (first < 0) first = i; ++n; }
        printf("M0=0x%08x: %d dwords written, first at byte %d, value %g, next %g\n", m, n, first * 4,
               first >= 0 ? h[first] : -1.f, first >= 0 ? h[first + 1] : -1.f);
    }
    return 0;
}
