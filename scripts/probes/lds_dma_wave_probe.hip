// LDS-DMA from the 8 waves of a 512-thread workgroup: wave w DMAs 64 dwords (values 1000 w +
// lane) to byte offset 20000 + 13312 w.  Report where each wave's data landed.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(const float* src, int* out) {
    extern __shared__ float s[];
    const int n = 160 * 1024 / 4;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s[i] = -7.0f;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 8192 * 4, 0x00020000);
    const int off = __builtin_amdgcn_readfirstlane(20000 + 13312 * wave);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(s + off / 4), 4,
                                             4 * (1000 * wave + lane), 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int m = 0;
        for (int i = 0; i < n; ++i)
            if (s[i] != -7.0f && m < 1000) { out[2 * m] = i * 4; out[2 * m + 1] = (int)s[i]; ++m; }
        out[2047] = m;
    }
}

int main() {
    static float h[8192];
    for (int i = 0; i < 8192; ++i) h[i] = (float)i;
    float* d; int* o;
    hipMalloc(&d, sizeof(h)); hipMalloc(&o, 2048 * 4);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipMemset(o, 0, 2048 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(512), 160 * 1024, 0, d, o);
    int ho[2048];
    hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
    printf("%d dwords changed\n", ho[2047]);
    for (int m = 0; m < ho[2047]; m += 64) printf("  byte %6d <- src %d (expect wave %d at %d)\n", ho[2 * m], ho[2 * m + 1],
                                                ho[2 * m + 1] / 1000, 20000 + 13312 * (ho[2 * m + 1] / 1000));
    return 0;
}
