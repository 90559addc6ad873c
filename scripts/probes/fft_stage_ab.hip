// A/B probe: one DFT16 stage of k_score_f32's four-step FFT on the VALU (the scorer's
// radix-4x4 with tan-factored twiddles, one 16-point column per lane) against the same
// 64 columns per wave on the matrix cores (v_mfma_f32_16x16x32_f16 on f16 hi/lo splits:
// Dh Xh + Dh Xl + Dl Xh, the DCT's scheme; 16 columns per MFMA set, 4 sets per wave).
// Both variants start from float32 data in registers and end with float32 results in
// registers, 8 waves per CU as in the scorer.  Reports wave-cycles per DFT16 column and
// the error against a float64 DFT.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o fft_stage_ab fft_stage_ab.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---- VALU DFT16 (as in ewk_mfcc.hip) ------------------------------------------------
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 t0 = make_float2(a0.x + a2.x, a0.y + a2.y), t1 = make_float2(a0.x - a2.x, a0.y - a2.y);
    const float2 t2 = make_float2(a1.x + a3.x, a1.y + a3.y), t3 = make_float2(a1.x - a3.x, a1.y - a3.y);
    a0 = make_float2(t0.x + t2.x, t0.y + t2.y);
    a2 = make_float2(t0.x - t2.x, t0.y - t2.y);
    a1 = make_float2(t1.x + t3.y, t1.y - t3.x);
    a3 = make_float2(t1.x - t3.y, t1.y + t3.x);
}
__device__ __forceinline__ void dft16_stage2(float2 (&x)[16]) {
    constexpr float C1 = 0.92387953251128674f, R2 = 0.70710678118654752f, T = 0.41421356237309505f;
    dft4(x[0], x[1], x[2], x[3]);
    {
        const float2 a0 = x[4], y1 = x[5], y2 = x[6], y3 = x[7];
        const float2 u2 = make_float2(y2.x + y2.y, y2.y - y2.x);
        const float2 t0 = make_float2(fmaf(R2, u2.x, a0.x), fmaf(R2, u2.y, a0.y));
        const float2 t1 = make_float2(fmaf(-R2, u2.x, a0.x), fmaf(-R2, u2.y, a0.y));
        const float2 u1 = make_float2(fmaf(T, y1.y, y1.x), fmaf(-T, y1.x, y1.y));
        const float2 u3 = make_float2(fmaf(T, y3.x, y3.y), fmaf(T, y3.y, -y3.x));
        const float2 v2 = make_float2(u1.x + u3.x, u1.y + u3.y), v3 = make_float2(u1.x - u3.x, u1.y - u3.y);
        x[4] = make_float2(fmaf(C1, v2.x, t0.x), fmaf(C1, v2.y, t0.y));
        x[6] = make_float2(fmaf(-C1, v2.x, t0.x), fmaf(-C1, v2.y, t0.y));
        x[5] = make_float2(fmaf(C1, v3.y, t1.x), fmaf(-C1, v3.x, t1.y));
        x[7] = make_float2(fmaf(-C1, v3.y, t1.x), fmaf(C1, v3.x, t1.y));
    }
    {
        const float2 a0 = x[8], y1 = x[9], y2 = x[10], y3 = x[11];
        const float2 t0 = make_float2(a0.x + y2.y, a0.y - y2.x), t1 = make_float2(a0.x - y2.y, a0.y + y2.x);
        const float2 u1 = make_float2(y1.x + y1.y, y1.y - y1.x);
        const float d3 = y3.y - y3.x, n3 = y3.x + y3.y;
        const float2 v2 = make_float2(u1.x + d3, u1.y - n3), v3 = make_float2(u1.x - d3, u1.y + n3);
        x[8] = make_float2(fmaf(R2, v2.x, t0.x), fmaf(R2, v2.y, t0.y));
        x[10] = make_float2(fmaf(-R2, v2.x, t0.x), fmaf(-R2, v2.y, t0.y));
        x[9] = make_float2(fmaf(R2, v3.y, t1.x), fmaf(-R2, v3.x, t1.y));
        x[11] = make_float2(fmaf(-R2, v3.y, t1.x), fmaf(R2, v3.x, t1.y));
    }
    {
        const float2 a0 = x[12], y1 = x[13], y2 = x[14], y3 = x[15];
        const float d2 = y2.y - y2.x, n2 = y2.x + y2.y;
        const float2 t0 = make_float2(fmaf(R2, d2, a0.x), fmaf(-R2, n2, a0.y));
        const float2 t1 = make_float2(fmaf(-R2, d2, a0.x), fmaf(R2, n2, a0.y));
        const float2 u1 = make_float2(fmaf(T, y1.x, y1.y), fmaf(T, y1.y, -y1.x));
        const float m3 = fmaf(T, y3.y, y3.x), u3y = fmaf(T, y3.x, -y3.y);
        const float2 v2 = make_float2(u1.x - m3, u1.y + u3y), v3 = make_float2(u1.x + m3, u1.y - u3y);
        x[12] = make_float2(fmaf(C1, v2.x, t0.x), fmaf(C1, v2.y, t0.y));
        x[14] = make_float2(fmaf(-C1, v2.x, t0.x), fmaf(-C1, v2.y, t0.y));
        x[13] = make_float2(fmaf(C1, v3.y, t1.x), fmaf(-C1, v3.x, t1.y));
        x[15] = make_float2(fmaf(-C1, v3.y, t1.x), fmaf(C1, v3.x, t1.y));
    }
}
__device__ __forceinline__ void dft16_perm(float2 (&x)[16]) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(x[n2], x[4 + n2], x[8 + n2], x[12 + n2]);
    dft16_stage2(x);
}
__device__ __forceinline__ constexpr int dperm(int k) { return 4 * (k & 3) + (k >> 2); }

// ---- MFMA DFT16 on hi/lo splits --------------------------------------------------------
__device__ __forceinline__ float f16_trunc(float x) { return __uint_as_float(__float_as_uint(x) & 0xFFFFE000u); }
__device__ __forceinline__ uint32_t pk_f16(float a, float b) {
    halfx2 h;
    h.x = (_Float16)a;
    h.y = (_Float16)b;
    return __builtin_bit_cast(uint32_t, h);
}
// B operand (lane (col, g): K = 8g..8g+7 of column col, K = 2 n + re/im) hi/lo from 8 floats
__device__ __forceinline__ void split8(const float (&x)[8], halfx8& hi, halfx8& lo) {
    float h[8], l[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { h[i] = f16_trunc(x[i]); l[i] = x[i] - h[i]; }
    uint4 H = make_uint4(pk_f16(h[0], h[1]), pk_f16(h[2], h[3]), pk_f16(h[4], h[5]), pk_f16(h[6], h[7]));
    uint4 L = make_uint4(pk_f16(l[0], l[1]), pk_f16(l[2], l[3]), pk_f16(l[4], l[5]), pk_f16(l[6], l[7]));
    hi = __builtin_bit_cast(halfx8, H);
    lo = __builtin_bit_cast(halfx8, L);
}
// A = real form of the DFT16 (row m = 2k + re/im, col K = 2n + re/im), split hi/lo; lane
// (row r, g): A[16 T + r][8g + i] for M-tile T.
__device__ void dft_a_operands(int lane, halfx8 (&Ah)[2], halfx8 (&Al)[2]) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int T = 0; T < 2; ++T) {
        float v[8];
        const int m = 16 * T + r, k = m >> 1, c = m & 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int K = 8 * g + i, n = K >> 1, cp = K & 1;
            const double ang = -2.0 * M_PI * (double)((k * n) & 15) / 16.0;
            const double wr = cos(ang), wi = sin(ang);
            // out.re = wr a - wi b ; out.im = wi a + wr b  (a = re, b = im of x[n])
            const double e = c == 0 ? (cp == 0 ? wr : -wi) : (cp == 0 ? wi : wr);
            v[i] = (float)e;
        }
        split8(v, Ah[T], Al[T]);
    }
}

constexpr int kIters = 32;

__global__ __launch_bounds__(512) void k_valu(const float* in, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float2 a[16];
#pragma unroll
    for (int n = 0; n < 16; ++n) a[n] = make_float2(in[(lane * 16 + n) * 2], in[(lane * 16 + n) * 2 + 1]);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
        dft16_perm(a);
        asm volatile("" : "+v"(a[0].x), "+v"(a[5].y), "+v"(a[10].x), "+v"(a[15].y));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
    if (blockIdx.x == 0 && wave == 0) {   // one iteration's result for the precision check
        float2 b[16];
#pragma unroll
        for (int n = 0; n < 16; ++n) b[n] = make_float2(in[(lane * 16 + n) * 2], in[(lane * 16 + n) * 2 + 1]);
        dft16_perm(b);
#pragma unroll
        for (int k = 0; k < 16; ++k) { out[(lane * 16 + k) * 2] = b[dperm(k)].x; out[(lane * 16 + k) * 2 + 1] = b[dperm(k)].y; }
    }
    float s = 0.f;
#pragma unroll
    for (int n = 0; n < 16; ++n) s += a[n].x + a[n].y;
    if (s == 1234.5f) out[0] = s;
}

// 4 sets of 16 columns per wave (64 DFT16s): lane (col, g) holds column col's K-chunk g
// of each set as 8 floats (x[set][8]).
__global__ __launch_bounds__(512) void k_mfma(const float* in, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 15, g = lane >> 4;
    halfx8 Ah[2], Al[2];
    dft_a_operands(lane, Ah, Al);
    float x[4][8];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[s][i] = in[((16 * s + col) * 16) * 2 + 8 * g + i];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            halfx8 Bh, Bl;
            split8(x[s], Bh, Bl);
            floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
            c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[0], Bh, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[1], Bh, c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[0], Bl, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[1], Bl, c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Al[0], Bh, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Al[1], Bh, c1, 0, 0, 0);
            // the outputs (rows 4g..4g+3 of each M-tile) become the next stage's inputs
#pragma unroll
            for (int i = 0; i < 4; ++i) { x[s][i] = c0[i]; x[s][4 + i] = c1[i]; }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
    if (blockIdx.x == 0 && wave == 0) {   // precision: set 0 on the original input
        float y[8];
        for (int i = 0; i < 8; ++i) y[i] = in[(col * 16) * 2 + 8 * g + i];
        halfx8 Bh, Bl;
        split8(y, Bh, Bl);
        floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[0], Bh, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[1], Bh, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[0], Bl, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah[1], Bl, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Al[0], Bh, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(Al[1], Bh, c1, 0, 0, 0);
        // lane (col, g): rows 4g + i (M-tile 0: k = 2g + i/2) and 16 + 4g + i (k = 8 + 2g + i/2)
        for (int i = 0; i < 4; ++i) {
            const int m0 = 4 * g + i, m1 = 16 + 4 * g + i;
            out[(col * 16 + (m0 >> 1)) * 2 + (m0 & 1)] = c0[i];
            out[(col * 16 + (m1 >> 1)) * 2 + (m1 & 1)] = c1[i];
        }
    }
    float sm = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) sm += x[s][i];
    if (sm == 1234.5f) out[0] = sm;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int ncol = 64 * 16;   // 1024 columns (k_valu uses 64 per wave, k_mfma 64 as 4 sets)
    float* h = (float*)malloc(ncol * 2 * sizeof(float));
    srand(7);
    for (int i = 0; i < ncol * 2; ++i) {   // windowed-sample-like values, 5 decades of level
        const double u = (rand() + 0.5) / ((double)RAND_MAX + 1.0), v = (rand() + 0.5) / ((double)RAND_MAX + 1.0);
        const double gsn = sqrt(-2.0 * log(u)) * cos(2.0 * M_PI * v);
        h[i] = (float)(gsn * pow(10.0, -5.0 * (double)((i / 32) % 6) / 5.0));
    }
    float *din, *dout;
    unsigned long long* dc;
    (void)hipMalloc(&din, ncol * 2 * sizeof(float));
    (void)hipMalloc(&dout, ncol * 2 * sizeof(float));
    (void)hipMalloc(&dc, cus * 8 * sizeof(unsigned long long));
    (void)hipMemcpy(din, h, ncol * 2 * sizeof(float), hipMemcpyHostToDevice);
    unsigned long long* hc = (unsigned long long*)malloc(cus * 8 * sizeof(unsigned long long));
    float* ho = (float*)malloc(ncol * 2 * sizeof(float));
    for (int v = 0; v < 2; ++v) {
        for (int rep = 0; rep < 3; ++rep) {
            if (v == 0) hipLaunchKernelGGL(k_valu, dim3(cus), dim3(512), 0, 0, din, dout, dc);
            else hipLaunchKernelGGL(k_mfma, dim3(cus), dim3(512), 0, 0, din, dout, dc);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(hc, dc, cus * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        (void)hipMemcpy(ho, dout, ncol * 2 * sizeof(float), hipMemcpyDeviceToHost);
        double cy = 0;
        for (int i = 0; i < cus * 8; ++i) cy += (double)hc[i];
        cy /= cus * 8;
        // wave-cycles per DFT16 column: each wave does 64 columns per iteration
        const double per_col = cy / kIters / 64.0;
        // precision vs a float64 DFT16 of the same input (first 64 columns for VALU: one per
        // lane; first 16 for MFMA: set 0), max |err| / max |X| per column
        double worst = 0, mean = 0;
        const int nc = v == 0 ? 64 : 16;
        for (int c = 0; c < nc; ++c) {
            double mx = 0, me = 0;
            for (int k = 0; k < 16; ++k) {
                double re = 0, im = 0;
                for (int n = 0; n < 16; ++n) {
                    const double a = h[(c * 16 + n) * 2], b = h[(c * 16 + n) * 2 + 1];
                    const double ang = -2.0 * M_PI * (double)((k * n) % 16) / 16.0;
                    re += a * cos(ang) - b * sin(ang);
                    im += a * sin(ang) + b * cos(ang);
                }
                const double er = ho[(c * 16 + k) * 2] - re, ei = ho[(c * 16 + k) * 2 + 1] - im;
                mx = fmax(mx, sqrt(re * re + im * im));
                me = fmax(me, sqrt(er * er + ei * ei));
            }
            const double rel = mx > 0 ? me / mx : 0;
            worst = fmax(worst, rel);
            mean += rel / nc;
        }
        printf("%s DFT16: %.2f wave-cycles (s_memtime) per 16-point column, 8 waves/CU; "
               "error max|dX|/max|X|: worst %.3g, mean %.3g\n", v == 0 ? "VALU radix-4x4 " : "MFMA f16 hi/lo", per_col,
               worst, mean);
    }
    return 0;
}
