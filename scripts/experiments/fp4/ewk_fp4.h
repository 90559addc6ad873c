// ewk_fp4.h -- a frame pass of the float32 scorer built in round 5: four lanes per frame.
// Measured slower than the product pass ("Round 5") and kept here, out of
// libewk.so; scripts/probes/fp4_probe.hip builds it.
//
// Replaces the FFT + mel + log of WordMatcher.extract_mfcc's librosa call (reference
// easywakeword/wakeword.py:561-563: stft(n_fft=512, hop=160, center=True) -> |.|^2 -> Slaney
// mel -> power_to_db) for 16 consecutive frames per wave: one pass = one 16-frame log-mel tile.
//
// Layout.  lane = p + 16 r: frame p of the pass, row r (a frame's four lanes sit in one column
// of the wave, one per 16-lane row), so every cross-lane step of the FFT and of the mel is a
// row exchange -- v_permlane16_swap (rows 0<->1, 2<->3) and v_permlane32_swap (rows 0<->2,
// 1<->3), no LDS round trip.  The 512-point real frame is 256 complex points z[n] = x[2n] +
// i x[2n+1]; row r holds z[r + 4 n'] (n' < 64, 128 VGPRs of packed (re, im) pairs) and:
//   1. windowed samples from the wave's staged span (LDS, skewed 4 floats per 160 samples so
//      the 32 lanes of a ds_read_b64 hit 64 distinct banks; filled by LDS-DMA, no VGPRs);
//   2. an in-lane DFT64 over n' (4 DFT16 with the window in their first stage, then a
//      W64-twiddled DFT4 with each twiddle factored as m (1 - i f) or m (f - i));
//   3. a transposition by 64 v_permlane16_swap + 64 v_permlane32_swap: quad q of row g then
//      holds Y_s[I_g(q)] of the four source rows s (scripts/fp4_model.py: item());
//   4. W256^(s k'') twiddles and a DFT4 over s: Z[k'' + 64 k'];
//   5. the real-FFT untangle, each bin k and its partner 256 - k in the same lane (the rows'
//      bin sets are closed under k -> 256 - k; row 0's slot pair (0, 15) is special);
//   6. the mel: per-lane partial band sums over the row's 64 bins (every 4-bin block holds one
//      bin of each row, so a band uses the same registers in every row: 229 FMAs, weights per
//      row), a reduce-scatter over the four rows (two swap + add stages per 32-band group),
//      and 10 log10(max(1e-10, .)): row r ends with bands 32 G + 8 r + i in lm[8 G + i],
//      exactly the B operand of k-step G of the DCT's v_mfma_f32_16x16x32_f16 (column = p).
// All complex arithmetic is packed f32 (v_pk_add/mul/fma_f32 with op_sel / neg modifiers):
// one instruction per complex add, two per complex multiply.
#pragma once

#include "../../../easywakeword_amd/csrc/ewk_internal.h"
#include "ewk_fp4_mel.h"
#include "fp4_tables.h"

namespace ewk {
namespace fp4 {

// Phase timing of the pass (scripts/probes/fp4_probe.hip built with -DFP4_TIMING only): the
// s_memtime cycles of each phase, summed in the caller's registers (FP4_TPARAM).
// FP4_SB: a scheduling fence between phases (keeps the scheduler from hoisting a later
// phase's table reads above the current phase's live set).
#ifndef FP4_SB
#define FP4_SB() __builtin_amdgcn_sched_barrier(0)
#endif
#ifdef FP4_TIMING
#define FP4_TS(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define FP4_TPARAM , uint64_t(&tdbg)[8]
#else
#define FP4_TS(v)
#define FP4_TPARAM
#endif

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int FPP = 16;            // frames per wave pass = one log-mel tile
constexpr int SKEW = 4;            // staging: 4 pad floats after every 160 samples
constexpr int BLK = HOP + SKEW;    // 164 staged floats per 160 samples
constexpr int STAGE_BLOCKS = 19;   // 160-sample blocks per pass (15 * 160 + 512 = 2912 samples)
constexpr int STAGE_FLOATS = (STAGE_BLOCKS - 1) * BLK + 64;   // the last block needs its first 32
constexpr int STAGE_BYTES = STAGE_FLOATS * 4;                  // 12,064
static_assert(STAGE_BYTES % 16 == 0, "stage");
static_assert(15 * BLK + 511 + 4 * 3 < STAGE_FLOATS, "frame 15's last sample is staged");

// ---- LDS tables (bytes; copied from Tables by fill_tables) ----------------------------
// Every twiddle is stored in the sign-paired form its packed op reads (m, -m), (f, -f),
// (-s, s, c, c), (-c, c): the negations ride in the VOP3P neg / op_sel modifiers of the whole
// operand, which the compiler folds (it cannot negate one element of a swizzled operand).
constexpr int RP_WIN = 64 * 8 + 16;    // row pitch of win4 [r][n1][a][c] (+16: rows in other banks)
constexpr int RP_TW4 = 16 * 3 * 16 + 16;   // tw4 [g][q][s - 1] = (-s, s, c, c)
constexpr int RP_UTC = 32 * 8 + 16;    // untangle (-cos, cos) [g][pair]
constexpr int RP_UTT = 32 * 8 + 16;    // untangle (tan, tan) [g][pair]
constexpr int RP_MEL = F4_NINC * 4 + 16;
static_assert(RP_MEL % 16 == 0, "mel weight rows");
constexpr int T_WIN = 0;
constexpr int T_TW64 = T_WIN + 4 * RP_WIN;   // [k2][j - 1] = (m, -m, f, -f), k2 = 0..15 (row 0 unused)
constexpr int T_TW4 = T_TW64 + 16 * 48;
constexpr int T_UTC = T_TW4 + 4 * RP_TW4;
constexpr int T_UTT = T_UTC + 4 * RP_UTC;
constexpr int T_MEL = T_UTT + 4 * RP_UTT;
// DCT operand image for v_mfma_f32_16x16x32_f16: D * 2^10 as f16 hi + lo.  Chunk c = 4 G + r
// of a frame holds bands 8 c .. 8 c + 7 (k-step G, lane row r).  Row tile 0 (coefficients
// 0..15): [G][hi/lo][lane] 16-B chunks; row tile 1 (16..19): [G][hi/lo][r][coef & 3] for the
// lanes with (l & 15) < 4, every other lane reads the block's zero chunk.
constexpr int DCT_RT1 = 4 * 2 * 64 * 16;
constexpr int DCT_RT1_STRIDE = 17 * 16;
constexpr int DCT_BYTES = DCT_RT1 + 8 * DCT_RT1_STRIDE;
constexpr int T_DCT = T_MEL + 4 * RP_MEL;
constexpr int TABLE_BYTES = (T_DCT + DCT_BYTES + 15) & ~15;
constexpr float kDctScale = 1024.0f;

// compile-time maps (ewk_internal.h; scripts/fp4_model.py: item, untangle_pairs)
__host__ __device__ constexpr int item(int g, int q) { return f4_item(g, q); }
__host__ __device__ constexpr bool formA(int jk) { return f4_formA(jk); }
__host__ __device__ constexpr int dperm(int k) { return 4 * (k & 3) + (k >> 2); }
// register of DFT64 output k'' = k2 + 16 k1 (in place: block k1, slot dperm(k2))
__host__ __device__ constexpr int yreg(int kk) { return 16 * (kk >> 4) + dperm(kk & 15); }

// ---- packed complex arithmetic -------------------------------------------------------
// Written with vector builtins, not inline asm: the scheduler then knows every instruction's
// latency, and the hazard recognizer its wait states (a VALU write read by a v_permlane swap or
// an MFMA).  A swizzle (.yx, .xx, .yy) becomes op_sel, a negated operand neg_lo/neg_hi.
#define F4_SW(v) __builtin_shufflevector((v), (v), 1, 0)
#define F4_B0(v) __builtin_shufflevector((v), (v), 0, 0)
#define F4_B1(v) __builtin_shufflevector((v), (v), 1, 1)
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// sign constants, kept in VGPRs (an SGPR operand slows a VALU instruction's issue)
struct Konst {
    f2 PM;   // (1, -1)
    f2 TT;   // (tan pi/8, -tan pi/8)
    f2 CC;   // (cos pi/8, -cos pi/8)
    f2 RR;   // (1/sqrt 2, -1/sqrt 2)
};
__device__ __forceinline__ Konst konst() {
    Konst k;
    k.PM = {1.0f, -1.0f};
    k.TT = {0.41421356237309505f, -0.41421356237309505f};
    k.CC = {0.92387953251128674f, -0.92387953251128674f};
    k.RR = {0.70710678118654752f, -0.70710678118654752f};
    asm volatile("" : "+v"(k.PM), "+v"(k.TT), "+v"(k.CC), "+v"(k.RR));
    return k;
}
__device__ __forceinline__ f2 rot_mi(f2 a, f2 b, const Konst& k) { return fma2(F4_SW(b), k.PM, a); }    // a - i b
__device__ __forceinline__ f2 rot_pi(f2 a, f2 b, const Konst& k) { return fma2(F4_SW(b), -k.PM, a); }   // a + i b

__device__ __forceinline__ void dft4(f2& a0, f2& a1, f2& a2, f2& a3, const Konst& k) {
    const f2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
    a0 = t0 + t2;
    a2 = t0 - t2;
    a1 = rot_mi(t1, t3, k);
    a3 = rot_pi(t1, t3, k);
}

// DFT16 in place, radix 4 x 4.  Stage 1, column a (inputs x[a + 4 c], c = 0..3) with the
// window w[c] folded into its first butterflies; stage 2 on the groups x[4 c' .. 4 c' + 3] with
// tan-factored W16 twiddles (W16^1 = C1 (1 - iT), W16^3 = C1 (T - i) = -i C1 (1 + iT), W16^2 =
// R2 (1 - i), W16^6 = R2 (-1 - i)).  On return x[dperm(k)] holds X[k].
__device__ __forceinline__ void dft16_col_win(f2& x0, f2& x1, f2& x2, f2& x3, f2 w0, f2 w1, f2 w2, f2 w3,
                                              const Konst& k) {
    const f2 p2 = x2 * w2, p3 = x3 * w3;
    const f2 t0 = fma2(x0, w0, p2), t1 = fma2(x0, w0, -p2);
    const f2 t2 = fma2(x1, w1, p3), t3 = fma2(x1, w1, -p3);
    x0 = t0 + t2;
    x2 = t0 - t2;
    x1 = rot_mi(t1, t3, k);
    x3 = rot_pi(t1, t3, k);
}
__device__ __forceinline__ void dft16_stage2(f2 (&x)[16], const Konst& k) {
    dft4(x[0], x[1], x[2], x[3], k);
    const f2 C1 = F4_B0(k.CC), R2 = F4_B0(k.RR);
    {   // group 1: W^1, W^2, W^3
        const f2 u2 = rot_mi(x[6], x[6], k);                 // x6 (1 - i)
        const f2 t0 = fma2(R2, u2, x[4]), t1 = fma2(-R2, u2, x[4]);
        const f2 u1 = fma2(F4_SW(x[5]), k.TT, x[5]);         // x5 (1 - iT)
        const f2 u3 = fma2(F4_SW(x[7]), -k.TT, x[7]);        // x7 (1 + iT); W^3 x7 = -i C1 u3
        const f2 v2 = rot_mi(u1, u3, k), v3 = rot_pi(u1, u3, k);
        x[4] = fma2(C1, v2, t0);
        x[6] = fma2(-C1, v2, t0);
        x[5] = fma2(F4_SW(v3), k.CC, t1);                    // t1 - i C1 v3
        x[7] = fma2(F4_SW(v3), -k.CC, t1);                   // t1 + i C1 v3
    }
    {   // group 2: W^2, W^4 = -i, W^6
        const f2 t0 = rot_mi(x[8], x[10], k), t1 = rot_pi(x[8], x[10], k);
        const f2 u1 = rot_mi(x[9], x[9], k);                 // x9 (1 - i)
        const f2 u3 = fma2(F4_SW(x[11]), k.PM, -x[11]);      // x11 (-1 - i)
        const f2 v2 = u1 + u3, v3 = u1 - u3;
        x[8] = fma2(R2, v2, t0);
        x[10] = fma2(-R2, v2, t0);
        x[9] = fma2(F4_SW(v3), k.RR, t1);
        x[11] = fma2(F4_SW(v3), -k.RR, t1);
    }
    {   // group 3: W^3, W^6, W^9 = -C1 (1 - iT)
        const f2 u2 = fma2(F4_SW(x[14]), k.PM, -x[14]);      // x14 (-1 - i)
        const f2 t0 = fma2(R2, u2, x[12]), t1 = fma2(-R2, u2, x[12]);
        const f2 u1 = fma2(F4_SW(x[13]), -k.TT, x[13]);      // x13 (1 + iT); W^3 x13 = -i C1 u1
        const f2 u3 = fma2(F4_SW(x[15]), k.TT, x[15]);       // x15 (1 - iT); W^9 x15 = -C1 u3
        const f2 w = rot_pi(u3, u1, k);                      // u3 + i u1:  v2 = -i u1 - u3 = -w
        const f2 z = rot_mi(u3, u1, k);                      // u3 - i u1:  v3 = -i u1 + u3 = z
        x[12] = fma2(-C1, w, t0);
        x[14] = fma2(C1, w, t0);
        x[13] = fma2(F4_SW(z), k.CC, t1);
        x[15] = fma2(F4_SW(z), -k.CC, t1);
    }
}

// W64^(j k2) u / m: form A, W = m (1 - i f): u (1 - i f);  form B, W = -i m (1 + i f): u (1 + i f).
// F = (f, -f); the form is a constant once the k2 loop is unrolled (the branch folds away).
__device__ __forceinline__ f2 tw_pre(bool A, f2 u, f2 F) { return A ? fma2(F4_SW(u), F, u) : fma2(F4_SW(u), F4_SW(F), u); }
// b + sign * (W u) from u' = tw_pre(u), M = (m, -m)
__device__ __forceinline__ f2 tw_add(bool A, bool plus, f2 b, f2 M, f2 up) {
    if (A) return plus ? fma2(F4_B0(M), up, b) : fma2(F4_B0(M), -up, b);
    return plus ? fma2(F4_SW(up), M, b) : fma2(F4_SW(up), F4_SW(M), b);   // b -/+ i m u' (-M = swapped M)
}
__device__ __forceinline__ f2 tw_mul(bool A, f2 M, f2 up) { return A ? F4_B0(M) * up : F4_SW(up) * M; }

// a (c + i s), W = (-s, s, c, c): (a.x c - a.y s, a.y c + a.x s) = a (c, c) + swap(a) (-s, s)
// (no element-1 broadcast of a computed value: the compiler moves it to a new register first)
__device__ __forceinline__ f2 cmul4(f2 a, f4 W) { return fma2(F4_SW(a), W.xy, a * F4_B0(W.zw)); }

// ---- LDS table fill (once per workgroup) -------------------------------------------------
__device__ __forceinline__ void fill_tables(const Fp4Tables* __restrict__ tab, unsigned char* t, float win_scale, int tid,
                                            int nthreads) {
    for (int i = tid; i < 4 * 64; i += nthreads) {
        const int r = i >> 6, e = i & 63;
        const float2 w = tab->win4[r][e];
        *reinterpret_cast<float2*>(t + T_WIN + r * RP_WIN + 8 * e) = make_float2(w.x * win_scale, w.y * win_scale);
    }
    for (int i = tid; i < 4 * 48; i += nthreads) {
        const int r = i / 48, e = i % 48;
        *reinterpret_cast<float4*>(t + T_TW4 + r * RP_TW4 + 16 * e) = tab->tw4[r][e / 3][e % 3];
    }
    for (int i = tid; i < 16 * 12; i += nthreads) *reinterpret_cast<float*>(t + T_TW64 + 4 * i) = tab->tw64[i / 12][i % 12];
    for (int i = tid; i < 4 * 32; i += nthreads) {
        const int r = i >> 5, j = i & 31;
        *reinterpret_cast<float2*>(t + T_UTC + r * RP_UTC + 8 * j) = tab->utc[r][j];
        *reinterpret_cast<float2*>(t + T_UTT + r * RP_UTT + 8 * j) = tab->utt[r][j];
    }
    for (int i = tid; i < 4 * F4_NINC; i += nthreads)
        *reinterpret_cast<float*>(t + T_MEL + (i / F4_NINC) * RP_MEL + 4 * (i % F4_NINC)) = tab->melw4[i / F4_NINC][i % F4_NINC];
    uint4* sd = reinterpret_cast<uint4*>(t + T_DCT);
    for (int i = tid; i < DCT_BYTES / 16; i += nthreads) {
        int row = -1, c = 0, hl = 0;
        if (i < DCT_RT1 / 16) {
            const int l = i & 63;
            hl = (i >> 6) & 1;
            row = l & 15;
            c = 4 * (i >> 7) + (l >> 4);
        } else {
            const int k = i - DCT_RT1 / 16, blk = k / 17, slot = k % 17;   // blk = G * 2 + hl
            if (slot < 16) {
                row = 16 + (slot & 3);
                c = 4 * (blk >> 1) + (slot >> 2);
                hl = blk & 1;
            }
        }
        uint32_t hw[4];
#pragma unroll
        for (int jj = 0; jj < 8; jj += 2) {
            float v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float d = row >= 0 ? tab->dct[row * NMEL + 8 * c + jj + u] * kDctScale : 0.0f;
                const float h = __uint_as_float(__float_as_uint(d) & 0xFFFFE000u);
                v2[u] = hl ? d - h : h;
            }
            _Float16 a = (_Float16)v2[0], b = (_Float16)v2[1];
            hw[jj >> 1] = (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
        }
        sd[i] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    }
}

// ---- staging: the pass's 2,912 samples -> the wave's LDS span, by LDS-DMA ---------------
// Block b (samples S0 + 160 b ...) goes to floats 164 b .. 164 b + 159; three dword DMAs per
// block write slots [0, 64), [64, 128), [128, 192): in the third, lanes 32-35 land on the pad
// and lanes 36-63 on the next block's slots 0..27 (the same values that block writes again).
// Every lane's sample offset is its own VGPR (negative or past-the-end samples are out of the
// buffer's range and land as 0: stft(center=True, pad_mode='constant')).
__device__ __forceinline__ int stage_lane_part(int j, int lane) {
    return j == 0 ? lane : (j == 1 ? 64 + lane : (lane < 32 ? 128 + lane : (lane < 36 ? 159 : lane + 124)));
}

#define EWK_LDS3(p) ((__attribute__((address_space(3))) void*)(p))

// (rolled loops: unrolled, the compiler hoists all 55 destinations and offsets out of the
// segment loop -- 55 SGPRs and VGPRs live through every pass)
// linear batch: segment = whole buffer descriptor (range [0, L))
__device__ __forceinline__ void stage_dma_linear(__amdgpu_buffer_rsrc_t rsrc, int S0, float* stage, int lane) {
    int v0 = 4 * (S0 + lane), v2 = 4 * (S0 + stage_lane_part(2, lane));
#pragma unroll 1
    for (int b = 0; b < STAGE_BLOCKS - 1; ++b) {
        float* dst = stage + BLK * b;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, EWK_LDS3(dst), 4, v0, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, EWK_LDS3(dst + 64), 4, v0 + 256, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, EWK_LDS3(dst + 128), 4, v2, 0, 0, 0);
        v0 += 4 * HOP;
        v2 += 4 * HOP;
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, EWK_LDS3(stage + BLK * (STAGE_BLOCKS - 1)), 4, v0, 0, 0, 0);
}

// float32 ring (RING 1): segment sample q lives at physical q + start (q < wrap_at) or
// q - wrap_at; samples outside [0, len) read as 0 (offset -1: out of the ring's range)
__device__ __forceinline__ int ring_off(int q, int len, int wrap_at, int start) {
    return (unsigned)q < (unsigned)len ? 4 * (q >= wrap_at ? q - wrap_at : q + start) : -1;
}
__device__ __forceinline__ void stage_dma_ring(__amdgpu_buffer_rsrc_t rsrc, int S0, int len, int wrap_at, int start,
                                               float* stage, int lane) {
    int q0 = S0 + lane, q2 = S0 + stage_lane_part(2, lane);
#pragma unroll 1
    for (int b = 0; b < STAGE_BLOCKS - 1; ++b) {
        float* dst = stage + BLK * b;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, EWK_LDS3(dst), 4, ring_off(q0, len, wrap_at, start), 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, EWK_LDS3(dst + 64), 4, ring_off(q0 + 64, len, wrap_at, start), 0, 0,
                                                 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, EWK_LDS3(dst + 128), 4, ring_off(q2, len, wrap_at, start), 0, 0, 0);
        q0 += HOP;
        q2 += HOP;
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, EWK_LDS3(stage + BLK * (STAGE_BLOCKS - 1)), 4,
                                             ring_off(q0, len, wrap_at, start), 0, 0, 0);
}

// int16 ring (RING 2): through registers (buffer_load_sshort, exact float), no DMA; eight
// loads per lane in flight
__device__ __forceinline__ void stage_i16_ring(__amdgpu_buffer_rsrc_t rsrc, int S0, int len, int wrap_at, int start,
                                               float* stage, int lane) {
    constexpr int N = (STAGE_FLOATS + 63) / 64;
#pragma unroll 1
    for (int c0 = 0; c0 < N; c0 += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int a = 64 * (c0 + u) + lane;                   // staged slot
            const int blk = a / BLK, w = a - BLK * blk;
            const int q = S0 + HOP * blk + (w < HOP ? w : HOP - 1);
            const int off = (unsigned)q < (unsigned)len ? 2 * (q >= wrap_at ? q - wrap_at : q + start) : -1;
            v[u] = (float)(short)__builtin_amdgcn_raw_buffer_load_b16(rsrc, off, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (64 * (c0 + u) + lane < STAGE_FLOATS) stage[64 * (c0 + u) + lane] = v[u];
    }
}

// ---- one pass: 16 frames t0 .. t0 + 15, samples already staged ---------------------------
// Returns the lane's 32 log-mel values (dB, unclamped) of frame t0 + (lane & 15): bands
// 32 G + 8 (lane >> 4) + i in lm[8 G + i].  vmax / vmin: max / min over the lane's values of a
// valid frame (t < T); nanp turns NaN if a band energy is NaN or infinite.  `issue_next` is
// called once the staged samples have been read (the next pass's DMA may then overwrite them).
template <typename NextFn>
__device__ __forceinline__ void pass(const unsigned char* tabs, const float* stage, int lane, bool valid,
                                     float (&lm)[32], float& vmax, float& vmin, float& nanp, NextFn issue_next FP4_TPARAM) {
    FP4_TS(ph0);
    const int p = lane & 15, r = lane >> 4;
    const Konst k = konst();
    f2 D[64];
    // ---- 1+2a: windowed samples and the four DFT16 (over n2, for n1 = 0..3)
    {
        const unsigned char* sb = reinterpret_cast<const unsigned char*>(stage) + 4 * (BLK * p + 2 * r);
        const unsigned char* wb = tabs + T_WIN + RP_WIN * r;
#pragma unroll
        for (int n1 = 0; n1 < 4; ++n1) {
            f2 x[16];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                // volatile: single ds_read_b64 in order (a ds_read2_b64 costs the LDS twice the
                // cycles per byte), consumed column by column
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int np = n1 + 4 * (a + 4 * c);
                    x[a + 4 * c] = *(const __attribute__((address_space(3))) volatile f2*)(sb + 32 * np + 16 * (np / 20));
                }
                // (volatile too: in order with the sample reads, not hoisted above them into spills)
                const f4 wa = *(const __attribute__((address_space(3))) volatile f4*)(wb + 128 * n1 + 32 * a);
                const f4 wc = *(const __attribute__((address_space(3))) volatile f4*)(wb + 128 * n1 + 32 * a + 16);
                dft16_col_win(x[a], x[a + 4], x[a + 8], x[a + 12], wa.xy, wa.zw, wc.xy, wc.zw, k);
            }
            dft16_stage2(x, k);
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) D[16 * n1 + kk] = x[kk];
        }
        // Every staged sample has been read: the next pass's DMA may start.  The DFT16 results
        // are pinned first -- without it the compiler sinks the arithmetic below the DMA loop and
        // keeps the 64 raw samples and 32 window vectors alive across it (spilled).
#pragma unroll
        for (int i = 0; i < 64; i += 8)
            asm volatile("" ::"v"(D[i]), "v"(D[i + 1]), "v"(D[i + 2]), "v"(D[i + 3]), "v"(D[i + 4]), "v"(D[i + 5]),
                         "v"(D[i + 6]), "v"(D[i + 7]));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_next();
    }
    FP4_TS(ph1);
    FP4_SB();
    // ---- 2b: W64^(n1 k2)-twiddled DFT4 over n1: Y[k2 + 16 k1] -> D[16 k1 + dperm(k2)]
    dft4(D[0], D[16], D[32], D[48], k);
    {
        const unsigned char* tb = tabs + T_TW64;
#pragma unroll
        for (int k2 = 1; k2 < 16; ++k2) {
            const f4 e1 = *reinterpret_cast<const f4*>(tb + 48 * k2);        // j = 1: m -m f -f
            const f4 e2 = *reinterpret_cast<const f4*>(tb + 48 * k2 + 16);   // j = 2
            const f4 e3 = *reinterpret_cast<const f4*>(tb + 48 * k2 + 32);   // j = 3
            const bool A1 = formA(k2), A2 = formA(2 * k2), A3 = formA(3 * k2);
            const int sl = dperm(k2);
            f2& b0 = D[sl];
            f2& b1 = D[16 + sl];
            f2& b2 = D[32 + sl];
            f2& b3 = D[48 + sl];
            const f2 u2 = tw_pre(A2, b2, e2.zw), u1 = tw_pre(A1, b1, e1.zw), u3 = tw_pre(A3, b3, e3.zw);
            const f2 t0 = tw_add(A2, true, b0, e2.xy, u2), t1 = tw_add(A2, false, b0, e2.xy, u2);
            const f2 q3 = tw_mul(A3, e3.xy, u3);
            const f2 sm = tw_add(A1, true, q3, e1.xy, u1);      // W u1 + W' u3
            const f2 df = tw_add(A1, true, -q3, e1.xy, u1);     // W u1 - W' u3
            b0 = t0 + sm;
            b2 = t0 - sm;
            b1 = rot_mi(t1, df, k);
            b3 = rot_pi(t1, df, k);
        }
    }
    FP4_TS(ph2);
    FP4_SB();
    // ---- 3: transposition across the four rows (quad q: items I_0..I_3(q))
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        f2& a0 = D[yreg(item(0, q))];
        f2& a1 = D[yreg(item(1, q))];
        f2& a2 = D[yreg(item(2, q))];
        f2& a3 = D[yreg(item(3, q))];
#define EWK_SWAP16(x, y)                                                                                          \
    do {                                                                                                          \
        const auto _r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false); \
        x = __uint_as_float(_r[0]);                                                                               \
        y = __uint_as_float(_r[1]);                                                                               \
    } while (0)
#define EWK_SWAP32(x, y)                                                                                          \
    do {                                                                                                          \
        const auto _r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false); \
        x = __uint_as_float(_r[0]);                                                                               \
        y = __uint_as_float(_r[1]);                                                                               \
    } while (0)
        EWK_SWAP16(a0.x, a1.x); EWK_SWAP16(a0.y, a1.y);
        EWK_SWAP16(a2.x, a3.x); EWK_SWAP16(a2.y, a3.y);
        EWK_SWAP32(a0.x, a2.x); EWK_SWAP32(a0.y, a2.y);
        EWK_SWAP32(a1.x, a3.x); EWK_SWAP32(a1.y, a3.y);
    }
    FP4_TS(ph3);
    FP4_SB();
    // ---- 4: W256^(s k'') and the DFT4 over the source rows s: Z[k'' + 64 k'] -> D[yreg(I_k'(q))]
    {
        const unsigned char* tb = tabs + T_TW4 + RP_TW4 * r;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const f4 w1 = *reinterpret_cast<const f4*>(tb + 48 * q);         // s = 1: (-s, s, c, c)
            const f4 w2 = *reinterpret_cast<const f4*>(tb + 48 * q + 16);    // s = 2
            const f4 w3 = *reinterpret_cast<const f4*>(tb + 48 * q + 32);    // s = 3
            f2& a0 = D[yreg(item(0, q))];
            f2& a1 = D[yreg(item(1, q))];
            f2& a2 = D[yreg(item(2, q))];
            f2& a3 = D[yreg(item(3, q))];
            a1 = cmul4(a1, w1);
            a2 = cmul4(a2, w2);
            a3 = cmul4(a3, w3);
            dft4(a0, a1, a2, a3, k);
        }
    }
    FP4_TS(ph4);
    FP4_SB();
    // ---- 5: untangle: P[slot 4 q + k'] (x 4, folded into the mel weights).  With A = u + conj v,
    // B = u - conj v, E = (t B.x - B.y, t B.y + B.x) and c, t the cos / tan of 2 pi k / 512:
    // P[k] = |A - c E|^2, P[256 - k] = |A + c E|^2.
    float P[64];
    {
        const unsigned char* ucb = tabs + T_UTC + RP_UTC * r;
        const unsigned char* utb = tabs + T_UTT + RP_UTT * r;
        const bool z0 = r == 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const f4 c01 = *reinterpret_cast<const f4*>(ucb + 32 * q);        // (-c, c) of pairs 4q, 4q+1
            const f4 c23 = *reinterpret_cast<const f4*>(ucb + 32 * q + 16);   // pairs 4q+2, 4q+3
            const f4 t01 = *reinterpret_cast<const f4*>(utb + 32 * q);        // (t, t) of pairs 4q, 4q+1
            const f4 t23 = *reinterpret_cast<const f4*>(utb + 32 * q + 16);   // pairs 4q+2, 4q+3
            f2 PP[4];
#pragma unroll
            for (int kp = 0; kp < 4; ++kp) {
                f2 u = D[yreg(item(kp, q))];
                f2 v = D[yreg(item(3 - kp, 15 - q))];
                if (q == 0) {   // row 0: bins 64/192, 32/224, 96/160, 128
                    const f2 uz = kp == 0 ? D[yreg(item(1, 0))] : (kp == 3 ? D[yreg(item(2, 0))] : D[yreg(item(kp - 1, 15))]);
                    const f2 vz = kp == 0 ? D[yreg(item(3, 0))] : (kp == 3 ? D[yreg(item(2, 0))] : D[yreg(item(4 - kp, 15))]);
                    u = z0 ? uz : u;
                    v = z0 ? vz : v;
                }
                const f2 UC = kp == 0 ? c01.xy : (kp == 1 ? c01.zw : (kp == 2 ? c23.xy : c23.zw));
                const f2 TP = kp == 0 ? t01.xy : (kp == 1 ? t01.zw : (kp == 2 ? t23.xy : t23.zw));
                const f2 A = fma2(v, k.PM, u);                     // u + conj v
                const f2 B = fma2(v, -k.PM, u);                    // u - conj v
                const f2 E = fma2(F4_SW(B), -k.PM, B * TP);
                const f2 R = fma2(F4_B0(E), UC, F4_B0(A));         // (A.x - c E.x, A.x + c E.x)
                const f2 I = fma2(F4_B1(E), UC, F4_B1(A));
                PP[kp] = fma2(R, R, I * I);                        // (P[u], P[v])
            }
            if (q == 0) {
                P[0] = PP[0].x;
                P[1] = z0 ? PP[0].x : PP[1].x;
                P[2] = z0 ? PP[3].x : PP[2].x;
                P[3] = z0 ? PP[0].y : PP[3].x;
                P[63] = z0 ? PP[1].y : PP[0].y;   // slot (15, 3)
                P[62] = z0 ? PP[2].y : PP[1].y;
                P[61] = z0 ? PP[2].x : PP[2].y;
                P[60] = z0 ? PP[1].x : PP[3].y;
            } else {
#pragma unroll
                for (int kp = 0; kp < 4; ++kp) {
                    P[4 * q + kp] = PP[kp].x;
                    P[4 * (15 - q) + 3 - kp] = PP[kp].y;
                }
            }
        }
    }
    FP4_TS(ph5);
    FP4_SB();
    // ---- 6: mel partial sums, reduce-scatter over the rows, log
    {
        const unsigned char* mb = tabs + T_MEL + RP_MEL * r;
        float fmx = -INFINITY, fmn = INFINITY;
#pragma unroll
        for (int G = 0; G < 4; ++G) {
            float acc[32];
#pragma unroll
            for (int i = 0; i < 32; ++i) acc[i] = 0.0f;
            f4 nw = *reinterpret_cast<const f4*>(mb + 4 * F4_INC_START[G]);
#pragma unroll
            for (int e0 = F4_INC_START[G]; e0 < F4_INC_START[G + 1]; e0 += 4) {
                const f4 wv = nw;   // requested one chunk ahead
                if (e0 + 4 < F4_INC_START[G + 1]) nw = *reinterpret_cast<const f4*>(mb + 4 * (e0 + 4));
                    const float ww[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (e0 + u < F4_INC_START[G] + F4_INC_COUNT[G])
                        acc[F4_INC_BAND[e0 + u]] = __builtin_fmaf(ww[u], P[F4_INC_SLOT[e0 + u]], acc[F4_INC_BAND[e0 + u]]);
            }
            // stage 1 (rows r, r ^ 2): bands u < 16 stay in rows 0/1, u + 16 in rows 2/3
            float s[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                EWK_SWAP32(acc[u], acc[u + 16]);
                s[u] = acc[u] + acc[u + 16];
            }
            // stage 2 (rows r, r ^ 1): j < 8 stays in even rows, j + 8 in odd rows
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                EWK_SWAP16(s[j], s[j + 8]);
                const float e = s[j] + s[j + 8];
                if (G == 0 && j == 0) nanp = __builtin_fmaf(e, 0.0f, nanp);   // NaN / inf band energy
                // 10 log10(x) = (10 log10 2) log2(x), v_log_f32
                const float db = 3.0102999566398120f * __log2f(fmaxf(1e-10f, e));
                lm[8 * G + j] = db;
                fmx = fmaxf(fmx, db);
                fmn = fminf(fmn, db);
            }
        }
        vmax = fmaxf(vmax, valid ? fmx : -INFINITY);
        vmin = fminf(vmin, valid ? fmn : INFINITY);
    }
#ifdef FP4_TIMING
    FP4_TS(ph6);
    tdbg[0] += ph1 - ph0; tdbg[1] += ph2 - ph1; tdbg[2] += ph3 - ph2;
    tdbg[3] += ph4 - ph3; tdbg[4] += ph5 - ph4; tdbg[5] += ph6 - ph5; tdbg[6] += 1;
#endif
#undef EWK_SWAP16
#undef EWK_SWAP32
}

// ---- DCT of the wave's 16 frames: C[32 x 16] = D[32 x 128] X[128 x 16] ----------------
// X = max(lm, clampv), split in f16 hi/lo (hi = x truncated to 11 bits, lo = f16(x - hi)),
// v_mfma_f32_16x16x32_f16 on Dh Xh + Dh Xl + Dl Xh.  Lane l gets C[4 (l >> 4) + i][l & 15] of
// both row tiles in c[0..3], c[4..7] (the layout of the previous scorer's tile_dct).
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
// hi = v_cvt_pkrtz (round toward zero = the 11-bit truncation over the dB range), lo = f16(x -
// float(hi)) rounded to nearest.  No inline asm here: the values feed the MFMA's B operand
// directly, and a VALU write that an MFMA reads needs wait states the compiler inserts only for
// instructions it can see (an asm v_fma_mix* producer gave launch-to-launch differences).
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& l) {
    const halfx2 hh = __builtin_bit_cast(halfx2, __builtin_amdgcn_cvt_pkrtz(a, b));
    halfx2 ll;
    ll.x = (_Float16)(a - (float)hh.x);
    ll.y = (_Float16)(b - (float)hh.y);
    h = __builtin_bit_cast(uint32_t, hh);
    l = __builtin_bit_cast(uint32_t, ll);
}
#ifndef EWK_DCT_SB
#define EWK_DCT_SB() __builtin_amdgcn_sched_barrier(0)
#endif
__device__ __forceinline__ void dct(const float (&lm)[32], float clampv, const unsigned char* tabs, int lane,
                                    float (&c)[8]) {
    // the pass's tail and these MFMAs are not interleaved (scheduled together, some passes came
    // out with one wrong register: launch-to-launch differences in the log-mel itself)
    EWK_DCT_SB();
    typedef float floatx4 __attribute__((ext_vector_type(4)));
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const int col = lane & 15, g4 = lane >> 4;
    const unsigned char* db = tabs + T_DCT;
    const uint4* a0p = reinterpret_cast<const uint4*>(db) + lane;
    const uint4* a1p = reinterpret_cast<const uint4*>(db + DCT_RT1) + (col < 4 ? 4 * g4 + col : 16);
#pragma unroll
    for (int G = 0; G < 4; ++G) {
        const uint4 A0h = a0p[128 * G], A0l = a0p[128 * G + 64];
        const uint4 A1h = a1p[17 * (2 * G)], A1l = a1p[17 * (2 * G + 1)];
        uint32_t h[4], l[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) split2(fmaxf(lm[8 * G + 2 * k], clampv), fmaxf(lm[8 * G + 2 * k + 1], clampv), h[k], l[k]);
        const uint4 Bh = make_uint4(h[0], h[1], h[2], h[3]), Bl = make_uint4(l[0], l[1], l[2], l[3]);
#define EWK_MF(a, b, acc) \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a), __builtin_bit_cast(halfx8, b), acc, 0, 0, 0)
        EWK_MF(A0h, Bh, acc0); EWK_MF(A1h, Bh, acc1);
        EWK_MF(A0h, Bl, acc0); EWK_MF(A1h, Bl, acc1);
        EWK_MF(A0l, Bh, acc0); EWK_MF(A1l, Bh, acc1);
#undef EWK_MF
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) { c[i] = acc0[i] * (1.0f / kDctScale); c[4 + i] = acc1[i] * (1.0f / kDctScale); }
    // read the accumulators here, in the MFMAs' block: sunk into a caller's conditional block the
    // reads got too few wait states after the last MFMA (launch-to-launch differences)
    asm volatile("" ::"v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6]), "v"(c[7]));
    EWK_DCT_SB();
}

}  // namespace fp4
}  // namespace ewk
