// Probe: can a line zeroed by hipMemsetAsync stay readable as ZERO on some XCD after another
// kernel rewrote it?  (round-6 ring-path miss: the recording build showed the ring scorer read
// four 128-B lines of zeros -- the ring's initial hipMemsetAsync -- where the gate had written
// samples twice since.)  Per round: hipMalloc region; hipMemsetAsync(0) [or our own zero
// kernel]; every XCD reads it (warm); a kernel on XCD w writes pattern; every XCD checks.
// Build: hipcc --offload-arch=gfx950 -O3 memset_stale_probe.hip -o memset_stale_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 15;
}
__global__ void k_zero(uint4* p, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4(0, 0, 0, 0);
}
__global__ void k_read(const uint32_t* p, size_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += p[i];
    if (acc == 0x9E3779B9u) sink[0] = acc;
}
__global__ void k_write_on(uint32_t* p, size_t n, int xcd, uint32_t tag) {
    if (xcc_id() != xcd) return;
    // the blocks on this XCD cover the region (blockIdx / 8 as their index among 8 XCDs' worth)
    const size_t nb = gridDim.x / 8, b = blockIdx.x / 8;
    for (size_t i = b * blockDim.x + threadIdx.x; i < n; i += nb * blockDim.x) p[i] = tag + (uint32_t)i;
}
__global__ void k_check(const uint32_t* p, size_t n, uint32_t tag, unsigned long long* cnt) {
    unsigned long long bad = 0, zero = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = p[i];
        if (v != tag + (uint32_t)i) { ++bad; zero += v == 0; }
    }
    if (bad) { atomicAdd(&cnt[0], bad); atomicAdd(&cnt[1], zero); }
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 100;
    unsigned long long* cnt;
    uint32_t* sink;
    hipMalloc(&cnt, 32);
    hipMalloc(&sink, 64);
    for (int mode = 0; mode < 2; ++mode) {
        hipMemset(cnt, 0, 32);
        int covered = 0;
        for (int r = 0; r < rounds; ++r) {
            const size_t bytes = (size_t)(1 + r % 7) << 20;
            const size_t n = bytes / 4;
            uint32_t* p;
            hipMalloc(&p, bytes);
            if (mode == 0) hipMemsetAsync(p, 0, bytes, 0);
            else hipLaunchKernelGGL(k_zero, dim3(1024), dim3(256), 0, 0, (uint4*)p, bytes / 16);
            hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, 0, p, n, sink);          // every XCD warm
            hipLaunchKernelGGL(k_write_on, dim3(2048), dim3(256), 0, 0, p, n, r % 8, 0x1000u * (r + 1));
            hipLaunchKernelGGL(k_check, dim3(2048), dim3(256), 0, 0, p, n, 0x1000u * (r + 1), cnt);
            hipDeviceSynchronize();
            hipFree(p);
            ++covered;
        }
        unsigned long long h[2];
        hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost);
        printf("%s zero-fill, %d rounds: %llu stale words (%llu of them zero)\n", mode ? "own-kernel" : "hipMemsetAsync",
               covered, h[0], h[1]);
        fflush(stdout);
    }
    printf("hip: %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
