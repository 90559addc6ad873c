// Where does an LDS-DMA (buffer_load_dword ... lds) land when its LDS destination is above
// 64 KiB?  Fill 160 KiB of LDS with a sentinel, DMA 64 dwords to byte offsets 16 KiB, 70 000,
// 100 000 and 140 000, then report every dword that changed.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(const float* src, int* out) {
    extern __shared__ float s[];
    const int n = 160 * 1024 / 4;
    for (int i = threadIdx.x; i < n; i += 64) s[i] = -7.0f;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 4096 * 4, 0x00020000);
    const int offs[4] = {16384, 70000, 100000, 140000};
    for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(s + offs[j] / 4), 4,
                                                 4 * (64 * j + threadIdx.x), 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int m = 0;
        for (int i = 0; i < n; ++i)
            if (s[i] != -7.0f && m < 1024) { out[2 * m] = i * 4; out[2 * m + 1] = (int)s[i]; ++m; }
        out[2047] = m;
    }
}

int main() {
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (float)i;
    float* d; int* o;
    hipMalloc(&d, sizeof(h)); hipMalloc(&o, 2048 * 4);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipMemset(o, 0, 2048 * 4);
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 160 * 1024, 0, d, o);
    int ho[2048];
    hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
    printf("%d dwords changed\n", ho[2047]);
    for (int m = 0; m < ho[2047]; m += 16) printf("  byte %6d <- src %d\n", ho[2 * m], ho[2 * m + 1]);
    return 0;
}
