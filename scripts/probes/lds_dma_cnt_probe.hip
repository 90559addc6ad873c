// Does LDS-DMA (buffer_load_dword ... lds) count in lgkmcnt as well as vmcnt?  Time (s_memtime)
// an s_waitcnt lgkmcnt(0) issued right after 48 LDS-DMA instructions (+ one ds_read), against
// an s_waitcnt vmcnt(0) in the same position.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int W>
__global__ void k(const float* src, unsigned long long* out) {
    extern __shared__ float s[];
    for (int i = threadIdx.x; i < 16384; i += 64) s[i] = (float)i;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 1 << 26, 0x00020000);
    const int lane = threadIdx.x;
    for (int j = 0; j < 48; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(s + 64 * j), 4,
                                                 4 * (4096 * j + lane) + 65536 * blockIdx.x, 0, 0, 0);
    const float v = ((volatile float*)s)[12000 + lane];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (W == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const float w = s[64 * 47 + lane];   // DMA destination after both waits
    if (lane == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = (unsigned long long)(v + w); }
}

int main() {
    float* d; unsigned long long* o;
    hipMalloc(&d, 1 << 26); hipMalloc(&o, 1024 * 16);
    hipMemset(d, 0, 1 << 26);
    unsigned long long h[2048];
    for (int W = 0; W < 2; ++W) {
        for (int rep = 0; rep < 2; ++rep) {
            if (W == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(64), 65536, 0, d, o);
            else hipLaunchKernelGGL(k<1>, dim3(256), dim3(64), 65536, 0, d, o);
            hipDeviceSynchronize();
        }
        hipMemcpy(h, o, 256 * 16, hipMemcpyDeviceToHost);
        unsigned long long sum = 0, mx = 0;
        for (int b = 0; b < 256; ++b) { sum += h[2 * b]; mx = h[2 * b] > mx ? h[2 * b] : mx; }
        printf("after 48 LDS-DMA: s_waitcnt %s took mean %llu, max %llu cycles\n", W == 0 ? "lgkmcnt(0)" : "vmcnt(0)  ", sum / 256, mx);
    }
    return 0;
}
