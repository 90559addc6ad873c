// Probe: after hipFree, does a new hipMalloc that reuses the virtual range see only its own
// data from every CU?  (round-6 ring-path miss: wrong values appear only in the first engine
// created after a session's earlier tests freed theirs, never in later identical engines, and
// only in the first rows of the new engine's ring.)
// Each round: A = hipMalloc(bytes); every CU writes pattern a into A (TLB entries everywhere);
// hipFree(A); B = hipMalloc(bytes) (usually the same address); hipMemset(B, 0); a kernel on every
// CU writes pattern b into B; a kernel on every CU checks B == b (counts other words, and words
// equal to pattern a: stale mappings).  Sizes vary so the allocator splits and merges ranges.
// Build: hipcc --offload-arch=gfx950 -O3 va_reuse_probe.hip -o va_reuse_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_fill(uint32_t* p, size_t n, uint32_t tag) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = tag ^ (uint32_t)(i * 2654435761u);
}
__global__ void k_check(const uint32_t* p, size_t n, uint32_t tag, uint32_t old_tag, unsigned long long* cnt) {
    unsigned long long bad = 0, stale = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = p[i];
        if (v != (tag ^ (uint32_t)(i * 2654435761u))) {
            ++bad;
            if (v == (old_tag ^ (uint32_t)(i * 2654435761u))) ++stale;
        }
    }
    if (bad) { atomicAdd(&cnt[0], bad); atomicAdd(&cnt[1], stale); }
}
__global__ void k_zero_check(const uint32_t* p, size_t n, unsigned long long* cnt) {
    unsigned long long bad = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (p[i] != 0u) ++bad;
    if (bad) atomicAdd(&cnt[2], bad);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 200;
    unsigned long long* cnt;
    hipMalloc(&cnt, 4 * sizeof(unsigned long long));
    hipMemset(cnt, 0, 4 * sizeof(unsigned long long));
    const size_t sizes[] = {1u << 20, 3u << 20, 20u << 20, 64u << 20, 5u << 20, 160u << 20, 2u << 20};
    int same = 0;
    srand(7);
    for (int r = 0; r < rounds; ++r) {
        const size_t bytes = sizes[r % 7] + 4096 * (size_t)(rand() % 64);
        const size_t n = bytes / 4;
        uint32_t *a, *b;
        hipMalloc(&a, bytes);
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, a, n, 0xA5A50000u + r);
        hipDeviceSynchronize();
        hipFree(a);
        hipMalloc(&b, bytes);
        same += (a == b);
        hipMemset(b, 0, bytes);
        hipLaunchKernelGGL(k_zero_check, dim3(2048), dim3(256), 0, 0, b, n, cnt);
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, b, n, 0x5A5A0000u + r);
        hipLaunchKernelGGL(k_check, dim3(2048), dim3(256), 0, 0, b, n, 0x5A5A0000u + r, 0xA5A50000u + r, cnt);
        hipDeviceSynchronize();
        hipFree(b);
    }
    unsigned long long h[4];
    hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost);
    printf("%d rounds (%d reused the freed address): words not zero after memset %llu; wrong after rewrite %llu "
           "(%llu of them the freed buffer's pattern)\nhip: %s\n",
           rounds, same, h[2], h[0], h[1], hipGetErrorString(hipGetLastError()));
    return 0;
}
