// Probe: issue cost of gfx950 f32 VALU forms, one and two waves per SIMD, 8 independent chains
// per lane (distinct operand registers per chain).  Cycles (s_memtime) per wave-instruction.
//   fma3v  v_fma_f32 d, a, b, c      (three VGPR sources)      fmac  v_fmac_f32 d, a, b (VOP2)
//   fmasv  v_fma_f32 d, a, s, c      (one SGPR source)         mul   v_mul_f32 d, a, b
//   add    v_add_f32 d, a, b                                  pkfma v_pk_fma_f32 (three VGPR pairs)
//   pkadd  v_pk_add_f32                                        pkmul v_pk_mul_f32
//   pkfmas v_pk_fma_f32 with op_sel_hi broadcast of one VGPR    mix   fma3v + ds_read_b64 alternating
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int KIND>
__global__ __launch_bounds__(512) void k(float* out, unsigned long long* cyc, int iters, float sv) {
    f2 a[8], b[8], c[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = f2{threadIdx.x * 0.001f + i, i * 0.5f};
        b[i] = f2{1.0001f + i * 1e-6f, 0.9999f};
        c[i] = f2{1e-4f * i, 2e-4f};
    }
    __shared__ f2 lds[512];
    lds[threadIdx.x] = a[0];
    __syncthreads();
    const unsigned lbase = (unsigned)(uintptr_t)lds + 8 * (threadIdx.x & 63);
    f2 acc = {0.f, 0.f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i].x) : "v"(b[i].x), "v"(c[i].x));
                if (KIND == 1) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i].x) : "v"(b[i].x), "v"(c[i].x));
                if (KIND == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i].x) : "s"(sv), "v"(c[i].x));
                if (KIND == 3) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i].x) : "v"(b[i].x));
                if (KIND == 4) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i].x) : "v"(c[i].x));
                if (KIND == 5) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "v"(c[i]));
                if (KIND == 6) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c[i]));
                if (KIND == 7) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
                if (KIND == 8) asm volatile("v_pk_fma_f32 %0, %0, %1, %2 op_sel_hi:[1,0,1]" : "+v"(a[i]) : "v"(b[i]), "v"(c[i]));
                if (KIND == 9) {
                    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i].x) : "v"(b[i].x), "v"(c[i].x));
                    if (i == 0) asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(acc) : "v"(lbase) : "memory");
                }
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = acc.x;
    for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
    if (s == 1234.5f) out[threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
}
typedef void (*kfn)(float*, unsigned long long*, int, float);
int main() {
    float* d;
    unsigned long long* cyc;
    (void)hipMalloc(&d, 4096);
    (void)hipMalloc(&cyc, 8);
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, iters = 4000;
    const char* names[10] = {"fma3v", "fmac", "fmasv", "mul", "add", "pkfma", "pkadd", "pkmul", "pkfma_bcast", "fma+ds_read"};
    kfn fns[10] = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>};
    for (int kind = 0; kind < 10; ++kind)
        for (int wps = 1; wps <= 2; ++wps) {
            const int threads = 256 * wps;
            unsigned long long h = 0;
            hipLaunchKernelGGL(fns[kind], dim3(cus), dim3(threads), 0, 0, d, cyc, 10, 1.0001f);
            (void)hipDeviceSynchronize();
            (void)hipMemset(cyc, 0, 8);
            hipLaunchKernelGGL(fns[kind], dim3(cus), dim3(threads), 0, 0, d, cyc, iters, 1.0001f);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
            const double per_wave = (double)h / ((double)cus * threads / 64);
            const double instr = (double)iters * 64;
            printf("%-12s waves/SIMD %d: %.2f cycles per wave-instruction per wave, %.2f per SIMD\n", names[kind], wps,
                   per_wave / instr, per_wave / instr / wps);
        }
    return 0;
}
