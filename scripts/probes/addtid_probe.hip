// Probe: ds_write_addtid_b32 placement for a given M0 (with and without the M0 -> LDS
// hazard nop), and __builtin_amdgcn_global_load_lds (4 B) placement (scripts/probes).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float* out, const float* src, uint32_t m0v, int mode) {
    __shared__ float s[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) s[i] = -1.0f;
    __syncthreads();
    if (threadIdx.x < 64) {
        float v = (float)threadIdx.x;
        uint32_t sv;
        if (mode == 0)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tds_write_addtid_b32 %2 offset:1024\n\ts_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %0"
                         : "=&s"(sv) : "s"(m0v), "v"(v) : "memory");
        else if (mode == 1)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tds_write_addtid_b32 %2 offset:1024\n\ts_waitcnt lgkmcnt(0)\n\ts_mov_b32 m0, %0"
                         : "=&s"(sv) : "s"(m0v), "v"(v) : "memory");
        else {
            __builtin_amdgcn_global_load_lds(src + threadIdx.x, (__attribute__((address_space(3))) void*)(s + m0v / 4), 4, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) out[i] = s[i];
}
int main() {
    float *d, *src; hipMalloc(&d, 8192 * 4); hipMalloc(&src, 64 * 4);
    float hs[64]; for (int i = 0; i < 64; ++i) hs[i] = 100.0f + i;
    hipMemcpy(src, hs, sizeof(hs), hipMemcpyHostToDevice);
    float h[8192];
    uint32_t cases[] = {0u, 4096u, 20000u};
    for (int mode = 0; mode < 3; ++mode)
        for (uint32_t m : cases) {
            hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, src, m, mode);
            hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            int first = -1, n = 0;
            for (int i = 0; i < 8192; ++i) if (h[i] != -1.0f) { if (first < 0) first = i; ++n; }
            printf("mode %d M0/base=%u: %d dwords written, first at byte %d, value %g, next %g, last %g\n", mode, m, n,
                   first * 4, first >= 0 ? h[first] : -1.f, first >= 0 ? h[first + 1] : -1.f,
                   first >= 0 ? h[first + n - 1] : -1.f);
        }
    return 0;
}
