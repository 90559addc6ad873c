// buffer_load_dword ... lds (LDS-DMA through a buffer descriptor): does an out-of-range lane
// write 0 into LDS, like the VGPR form returns 0?  (the scorer's scout / staging would rely on it)
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(const float* src, int n, float* out) {
    __shared__ float s[4 * 64];
    for (int i = threadIdx.x; i < 4 * 64; i += 64) s[i] = -7.0f;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, n * 4, 0x00020000);
    const int lane = threadIdx.x;
    // row 0: in range for lanes < n; row 1: lanes 0..63 at n - 32 + lane (half out of range);
    // row 2: offset -1 (huge unsigned: out of range); row 3: in range
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(s + 0), 4, lane * 4, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(s + 64), 4, (n - 32 + lane) * 4, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(s + 128), 4, -1, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(s + 192), 4, (lane + 5) * 4, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * 64; i += 64) out[i] = s[i];
}

int main() {
    const int n = 100;
    float h[n], o[256];
    for (int i = 0; i < n; ++i) h[i] = 1.0f + i;
    float *d, *dout;
    hipMalloc(&d, n * 4);
    hipMalloc(&dout, 256 * 4);
    hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, n, dout);
    hipMemcpy(o, dout, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        bad += o[l] != h[l];
        const int q = n - 32 + l;
        bad += o[64 + l] != (q < n ? h[q] : 0.0f);
        bad += o[128 + l] != 0.0f;
        bad += o[192 + l] != h[l + 5];
    }
    printf("row1 lanes 30..34: %g %g %g %g %g; row2 lane 0: %g\n", o[94], o[95], o[96], o[97], o[98], o[128]);
    printf("buffer_lds_probe: %s (%d mismatches)\n", bad ? "FAIL" : "OOB lanes write 0", bad);
    return bad != 0;
}
