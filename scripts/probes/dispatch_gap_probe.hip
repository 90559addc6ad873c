// Dispatch-gap probe: gaps between back-to-back kernels on one stream (read them from a
// rocprofv3 --kernel-trace of this binary) for a second kernel with/without 157 KB of dynamic
// LDS and with/without private scratch, after a first kernel that fills the GPU.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fill(float* p, int n) {   // 8,192 waves writing 64 MB (like the gate)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = (float)i;
}
__global__ __launch_bounds__(512, 1) void k_small(float* p) {
    extern __shared__ float lds[];
    if (threadIdx.x == 0 && p[0] < -1.0f) { lds[0] = 1.0f; p[1] = lds[0]; }
}
__global__ __launch_bounds__(512, 1) void k_scratch(float* p, int k) {
    extern __shared__ float lds[];
    volatile float a[64];
    for (int i = 0; i < 64; ++i) a[i] = p[i & 7];
    if (threadIdx.x == 0 && a[k & 63] < -1.0f) { lds[0] = 1.0f; p[1] = lds[0]; }
}

int main() {
    const int n = 16 << 20;
    float* p;
    if (hipMalloc(&p, n * sizeof(float)) != hipSuccess) return 1;
    hipMemset(p, 0, n * sizeof(float));
    const int big = 157 * 1024;
    hipFuncSetAttribute((const void*)k_small, hipFuncAttributeMaxDynamicSharedMemorySize, big);
    hipFuncSetAttribute((const void*)k_scratch, hipFuncAttributeMaxDynamicSharedMemorySize, big);
    for (int rep = 0; rep < 50; ++rep) {
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, p, n);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, 0, p);        // no LDS, no scratch
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, p, n);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(512), big, 0, p);      // 157 KB LDS
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, p, n);
        hipLaunchKernelGGL(k_scratch, dim3(256), dim3(512), big, 0, p, rep);   // LDS + scratch
    }
    hipDeviceSynchronize();
    printf("done\n");
    hipFree(p);
    return 0;
}
