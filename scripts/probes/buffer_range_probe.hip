// Probe: how does the buffer range check treat a 16-B load that straddles num_records?
// A raw buffer descriptor over n floats (num_records = 4 n bytes); lane l loads 16 B at
// byte offset 4 (n - 4 + l) for l < 8 and prints which of its four dwords came back.
// Build: hipcc --offload-arch=gfx950 -O3 -o buffer_range_probe buffer_range_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void probe(const float* p, int n, float* out) {
    const int l = threadIdx.x;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, n * 4, 0x00020000);
    const int off = 4 * (n - 4 + l);
    const uint4 q = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    out[4 * l + 0] = __uint_as_float(q.x);
    out[4 * l + 1] = __uint_as_float(q.y);
    out[4 * l + 2] = __uint_as_float(q.z);
    out[4 * l + 3] = __uint_as_float(q.w);
    // also a b64 and a b96 at the same offsets
    const uint2 d = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    out[32 + 2 * l] = __uint_as_float(d.x);
    out[32 + 2 * l + 1] = __uint_as_float(d.y);
}

int main() {
    const int n = 64;
    float h[n + 16];
    for (int i = 0; i < n + 16; ++i) h[i] = (float)(i + 1);   // past n: nonzero, so a read shows
    float *d, *o;
    hipMalloc(&d, sizeof(h));
    hipMalloc(&o, 64 * sizeof(float));
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipMemset(o, 0xff, 64 * sizeof(float));
    probe<<<1, 8>>>(d, n, o);
    float r[64];
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    for (int l = 0; l < 8; ++l)
        printf("b128 at sample %d (n = %d): %g %g %g %g   b64: %g %g\n", n - 4 + l, n, r[4 * l], r[4 * l + 1],
               r[4 * l + 2], r[4 * l + 3], r[32 + 2 * l], r[32 + 2 * l + 1]);
    hipFree(d);
    hipFree(o);
    return 0;
}
