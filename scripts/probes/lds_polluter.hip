// Diagnostic: leave every CU's LDS (and the VGPRs of the last waves) full of a chosen pattern,
// so a later kernel that reads LDS or registers before writing them sees that pattern instead
// of the benign leftovers of an identical earlier launch (round-6 ring-path miss: wrong values
// only in the first engine after other tests ran).
//   pollute(kind): kind 0 = quiet NaN words, 1 = large finite floats (1e30), 2 = xorshift
//   random words, 3 = small finite floats (0.5 + i * 1e-6).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC lds_polluter.hip -o lds_polluter.so
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t pat(int kind, uint32_t i) {
    switch (kind) {
    case 0: return 0x7FC00000u | (i & 0xFFFu);
    case 1: return __float_as_uint(1e30f);
    case 2: { uint32_t x = i * 2654435761u + 0x9E3779B9u; x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; }
    default: return __float_as_uint(0.5f + (float)(i & 0xFFFF) * 1e-6f);
    }
}

__global__ __launch_bounds__(1024) void k_pollute(int kind, uint32_t* sink) {
    extern __shared__ uint32_t lds[];
    const int n = 160 * 1024 / 4;
    for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = pat(kind, i + 977u * blockIdx.x);
    __syncthreads();
    // registers: 96 live values per lane, combined so none is dead
    uint32_t r[96];
#pragma unroll
    for (int k = 0; k < 96; ++k) r[k] = pat(kind, threadIdx.x * 131u + k + lds[(threadIdx.x * 7 + k) % n]);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 96; ++k) acc ^= r[k] * (k + 1);
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

extern "C" int pollute(int kind) {
    static uint32_t* sink = nullptr;
    if (!sink && hipMalloc(&sink, 4096 * 4) != hipSuccess) return -1;
    hipFuncSetAttribute((const void*)k_pollute, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int rep = 0; rep < 4; ++rep)
        hipLaunchKernelGGL(k_pollute, dim3(256 * 4), dim3(1024), 160 * 1024, 0, kind, sink);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
