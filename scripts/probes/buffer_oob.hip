// Probe: does buffer_load_dwordx4 range-check per dword (partial tails) on gfx950?
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const float* p, int n, float* out) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, n * 4, 0x00020000);
    const int l = threadIdx.x;
    // lane l loads 4 dwords starting at float index l*4 - 6 (unaligned starts included)
    int off = (l * 4 - 6) * 4;
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    out[l * 4 + 0] = __builtin_bit_cast(float, v[0]);
    out[l * 4 + 1] = __builtin_bit_cast(float, v[1]);
    out[l * 4 + 2] = __builtin_bit_cast(float, v[2]);
    out[l * 4 + 3] = __builtin_bit_cast(float, v[3]);
}
__global__ void k1(const float* p, int n, float* out) {   // same with a 1-float misalignment
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(p + 1), (short)0, n * 4, 0x00020000);
    const int l = threadIdx.x;
    int off = (l * 4 - 6) * 4;
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    for (int c = 0; c < 4; ++c) out[l * 4 + c] = __builtin_bit_cast(float, v[c]);
}
int main() {
    const int n = 101;
    float h[256];
    for (int i = 0; i < 256; ++i) h[i] = i + 1;
    float *d, *o;
    hipMalloc(&d, 256 * 4); hipMalloc(&o, 256 * 4);
    hipMemcpy(d, h, 256 * 4, hipMemcpyHostToDevice);
    float r[256];
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 0) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, n, o);
        else hipLaunchKernelGGL(k1, dim3(1), dim3(64), 0, 0, d, n, o);
        hipMemcpy(r, o, 256 * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int c = 0; c < 4; ++c) {
                const int q = l * 4 - 6 + c;
                const float want = (q >= 0 && q < n) ? h[q + pass] : 0.0f;
                if (r[l * 4 + c] != want) {
                    if (bad < 12) printf("pass %d lane %d c %d q %d got %g want %g\n", pass, l, c, q, r[l * 4 + c], want);
                    ++bad;
                }
            }
        printf("pass %d (%s): %d mismatches\n", pass, pass ? "unaligned base" : "aligned base", bad);
    }
    return 0;
}
