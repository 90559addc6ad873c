// LDS broadcast probe: does a ds_read_b128 whose 64 lanes read only 16 (or 1) distinct
// 16-B rows cost less LDS time than one with 64 distinct rows?  8 waves per workgroup, one
// workgroup per CU (the scorer's shape), each wave issuing batches of 8 reads.
// Build: hipcc --offload-arch=gfx950 -O3 lds_broadcast_probe.hip -o lds_broadcast_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void k(float* out, int iters) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4* s = reinterpret_cast<float4*>(smem);
    for (int i = threadIdx.x; i < 8192; i += 512) s[i] = make_float4(i, i + 1, i + 2, i + 3);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // row of this lane: MODE 0: 64 distinct, 1: 16 distinct (lane & 15), 2: one row
    const int row = MODE == 0 ? lane : (MODE == 1 ? (lane & 15) : 0);
    const uint32_t base = (uint32_t)(uintptr_t)(s + 1024 * wave + 9 * row);   // 9: odd row pitch (conflict free)
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
        floatx4 r[8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[c]) : "v"(base), "i"(16 * 64 * c) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int c = 0; c < 8; ++c) acc += r[c];
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main() {
    float* d;
    hipMalloc(&d, 256 * 512 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 4000;
    for (int rep = 0; rep < 2; ++rep)
        for (int m = 0; m < 3; ++m) {
            hipEventRecord(a);
            if (m == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(512), 131072, 0, d, iters);
            if (m == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(512), 131072, 0, d, iters);
            if (m == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(512), 131072, 0, d, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            // per CU: 8 waves x iters x 8 reads of 1 KiB
            const double bytes = 8.0 * iters * 8 * 1024;
            printf("mode %d (%s): %.3f ms, %.1f B/clk/CU at 2.1 GHz\n", m,
                   m == 0 ? "64 distinct rows" : (m == 1 ? "16 distinct rows" : "1 row"), ms,
                   bytes / (ms * 1e-3 * 2.1e9));
        }
    return 0;
}
