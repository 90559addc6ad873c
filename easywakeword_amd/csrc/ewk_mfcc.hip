// ewk_mfcc.hip -- level-2 matcher: fused MFCC + cosine scorer for ragged segment
// batches on gfx950 (CDNA4).
//
// Replaces WordMatcher.extract_mfcc / calculate_similarity / matches
// (reference easywakeword/wakeword.py:544-639), i.e. librosa 0.11.0
// feature.mfcc(n_mfcc=20, n_fft=512, hop=160) + scipy cosine + the score
// scaling, for many segments per launch.
//
// Design.  Linear batches: one wave = one segment; a persistent grid (one 8-wave
// workgroup per CU sharing the LDS tables) pulls segments from an atomic work counter in
// longest-first order.  Ring events of a streaming tick: one segment per workgroup (its
// tiles spread over the 8 waves) for a few hundred events, one per wave for many.
//   frames  : stft(center=True, pad_mode=constant): frame t covers samples
//             [t*160-256, t*160+256) of the segment, zero outside; T = 1+L//160.
//             Samples come through a buffer descriptor whose range check returns 0
//             outside the segment (the padding); ring segments wrap at the stream ring.
//   staging : a wave pass is 8 frames spanning 1,632 contiguous samples, loaded one
//             pass ahead with coalesced dword loads and stored to LDS with
//             ds_write_addtid_b32.
//   FFT     : 16 lanes per frame, two frames per 16-lane group (8 frames per pass: two
//             independent instruction streams per lane).  The 512-point real frame is
//             packed as 256 complex points z[n] = x[2n] + i x[2n+1]; 256 = 16 x 16
//             four-step FFT: a register DFT16 (window folded into its first stage,
//             tan-factored W16 twiddles), a twiddle, an LDS transpose, a second DFT16,
//             then the real-FFT untangle with each bin and its conjugate partner in the
//             same lane (no cross-lane traffic).
//   mel     : Slaney bands from LDS, fully unrolled with compile-time group widths
//             (band m = j + 16 i; widths {2,2,2,3,4,6,9,12}, weights zero-padded), then
//             10*log10(max(1e-10, .)) via v_log_f32; written to a 16-frame log-mel tile
//             as f16 hi/lo pairs (hi = x truncated to 11 bits, lo = x - hi).
//   DCT     : the only dense GEMM on the path: C[32 x 16] = D[32 x 128] . X[128 x 16]
//             per 16-frame tile on the matrix cores, v_mfma_f32_16x16x32_f16 on the hi/lo
//             splits (Dh Xh + Dh Xl + Dl Xh, f32 accumulation), rows 20..31 zero.
//   top_db  : power_to_db clamps at (segment max - 80 dB), a segment-global coupling.
//             Pass 1 clamps each tile speculatively at the running max - 80 dB (exact
//             once the max is known) and records the stored tile minimum; if the segment
//             min is below the final max - 80 dB, pass 2 recomputes only the tiles whose
//             stored minimum is below it and swaps their contribution in the statistics
//             (nothing is written to global memory but the results).
//   stats   : population mean/std over frames from fp64 shifted sums
//             (d = c - c[frame 0]) -- exact 0 std for identical frames.
//   score   : the reference's own float32 / float64 cosine arithmetic
//             (wakeword.py:611-625 + scipy correlation); NaN kept.  Near-threshold
//             scores are re-scored by k_score_f64 (fp64 path, below).
#include <hip/hip_runtime.h>
#include <math.h>

#include "ewk_internal.h"
#include "ewk_db64.h"   // (the fp64 re-score's 10 log10, ewk_rescore.h)

// s_setprio 1 over the frame-pass LDS phases (window, transposes, mel): -0.4 %
#define EWK_SETPRIO(v) __builtin_amdgcn_s_setprio(v)

// Per-wave phase timing of the linear-batch scorer (debug builds with -DEWK_TIMING only:
// scripts/mb_score.py prints it; the product build compiles none of it).  dbg[k] sums the
// s_memtime cycles of phase k over the wave's segments; the kernel adds them to g_ewk_dbg.
#ifdef EWK_TIMING
#define EWK_DBG_PARAM , uint64_t(&dbg)[kDbgN]
#define EWK_DBG_ARG , dbg
#define EWK_TS(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define EWK_TADD(k, a, b) dbg[k] += (b) - (a)
// frame-pass sub-phases (dbg[12..18]) and passes timed (dbg[19]); tile_passes passes nullptr
#define EWK_PASS_PARAM , uint64_t* pdbg
#define EWK_PASS_ARG(x) , x
#else
#define EWK_DBG_PARAM
#define EWK_DBG_ARG
#define EWK_TS(v)
#define EWK_TADD(k, a, b)
#define EWK_PASS_PARAM
#define EWK_PASS_ARG(x)
#endif
#ifdef EWK_TIMING
constexpr int kDbgN = 20;
#endif

namespace ewk {

#ifdef EWK_TIMING
__device__ unsigned long long g_ewk_dbg[kDbgN];
#endif
// Why segments go to the fp64 re-score (debug builds with -DEWK_LIST_STATS only,
// scripts/list_reasons.py): [0] listed, [1..4] segments meeting each criterion (margin, short,
// nearly stationary, vanishing mean; a segment can meet several), [5..9] their frames.
#ifdef EWK_LIST_STATS
__device__ unsigned long long g_ewk_list[10];
#endif
#ifdef EWK_COOP_DEBUG
// what each wave of the cooperative ring scorer saw, keyed by (stream & 31) * 256 + (tick & 255)
// (scripts/diag_coop.py): the event, its max/min/theta, its shifted sums, the combined stats
constexpr int kCoopKeys = 32 * 256;
__device__ int4 g_coop_ev[kCoopKeys][WAVES];      // stream, ring_start, length, tick
__device__ float4 g_coop_th[kCoopKeys][WAVES];    // wave vmax, wave vmin, theta, nloc
__device__ double g_coop_pd[kCoopKeys][WAVES][60];
__device__ float g_coop_ms[kCoopKeys][40];
__device__ uint4 g_coop_tile[4 * 256][WAVES][512];   // streams 0-3: each wave's last tile before the clamp
#define EWK_COOP_KEY_PARAM , int dkey
#define EWK_COOP_KEY_ARG(k) , (k)
#else
#define EWK_COOP_KEY_PARAM
#define EWK_COOP_KEY_ARG(k)
#endif

typedef float floatx4 __attribute__((ext_vector_type(4)));

// LDS carve (bytes, every offset a multiple of 16).  The per-lane table rows are
// transposed to [lane j][index] with a 144-B (36-dword) row pitch so one
// ds_read_b128 fetches 2 float2 entries and a 16-lane group spans all 64 banks.
// Frames per wave pass: kNF per 16-lane group (kNF = 2: two independent FFTs per lane).
constexpr int kFPP = 4 * kNF;
constexpr int kStageLoads = ((kFPP - 1) * HOP + NFFT + 63) / 64;   // dword loads per lane per pass
// frame fr's FFT scratch starts at scr_frame_off(fr) (ewk_internal.h)
constexpr int kScrFrames = kFPP * SCR_FRAME + 8 * (kNF - 1);
// kNF = 2: a lane's two frames are consecutive (slot (g, f) = frame 2f + g of the pass),
// so the second frame's first 11 sample pairs are the first frame's pairs 5..15 (hop 160 =
// 5 x 32) and only 5 more are read.  The stage is skewed -- sample s at s + 32 floor(s / 320)
// -- so the four lane groups' frames (320 samples apart) land 32 banks apart.
__host__ __device__ constexpr int stg_off(int c) { return 256 * c + 128 * (c / 5); }   // bytes of stage row c
__host__ __device__ constexpr int win_off(int g, int n1) {   // bytes: pair n1 of slot g from the lane's base
    return 4 * (160 * g + 32 * n1 + 32 * ((160 * g + 32 * n1) / 320));
}
constexpr int kStageFloats = stg_off(kStageLoads) / 4;
constexpr int kScrFloats = (kScrFrames > kStageFloats) ? kScrFrames : kStageFloats;
// The per-wave FFT scratch (also the sample staging) comes first in LDS: the M0 base of
// ds_write_addtid_b32 is 16 bits wide, so every wave's scratch must start below 64 KB.
constexpr int SCR_BYTES = (kScrFloats * 4 + 15) & ~15;
constexpr int L_SCR = 0;                                  // [wave] kFPP frames x 272 floats
constexpr int L_TAB = L_SCR + WAVES * SCR_BYTES;
static_assert(L_SCR + (WAVES - 1) * SCR_BYTES < 65536, "ds_write_addtid_b32 bases must fit M0[15:0]");

// LDS carve (bytes, every offset a multiple of 16).  The per-lane table rows are
// transposed to [lane j][index] with a 144-B (36-dword) row pitch so one
// ds_read_b128 fetches 2 float2 entries and a 16-lane group spans all 64 banks.
constexpr int TP = 18;                                    // float2 pitch of a [j][16] table row
constexpr int WP = 52;                                    // float pitch of the [j][48] mel weight row (13 chunks: b128/b64 conflict free)
constexpr int L_WIN2 = L_TAB;                             // [j][n1] = win2[16*n1 + j]
constexpr int L_TW1 = L_WIN2 + 16 * TP * 8;               // [j][k1-1] = tw1[16*k1 + j], k1 = 1..15
constexpr int L_TW2 = L_TW1 + 16 * TP * 8;                // [j][k2] = tw2[j + 16*k2]
constexpr int L_WPAD = L_TW2 + 16 * TP * 8;               // [j][kMelOff[i] + q] = wpad[16*(it0_i + q) + j]
constexpr int L_BLO = L_WPAD + 16 * WP * 4;
constexpr int L_DCT = L_BLO + NMEL * 4;
// DCT operand image for v_mfma_f32_16x16x32_f16: D * 2^10 split into f16 hi + lo (the
// products hi*hi + hi*lo + lo*hi carry ~22 bits).  The tile's k order groups each lane's
// eight bands: k-chunk c (k = 8c .. 8c+7) holds bands c + 16 jj, jj = 0..7, so the
// operand of k-step q for lane l is chunk 4q + (l >> 4).  Row tile 0 (coefficients 0..15):
// [q][hi/lo][lane] 16-B chunks; row tile 1 (coefficients 16..19): [q][hi/lo][l >> 4][l & 3]
// for the lanes with (l & 15) < 4, every other lane reads the block's zero chunk.
constexpr float kDctScale = 1024.0f;
constexpr float kTopDbUnits = 80.0f;   // top_db, in the tile's dB units
constexpr int DCT_RT1 = 4 * 2 * 64 * 16;                  // row tile 1: [q][hi/lo] blocks of 17 chunks
constexpr int DCT_RT1_STRIDE = 17 * 16;                   // 16 data chunks [l >> 4][l & 3] + a zero chunk
constexpr int DCT_BYTES = DCT_RT1 + 8 * DCT_RT1_STRIDE;
constexpr int L_SHARED_END = ((L_DCT + DCT_BYTES) + 15) & ~15;
constexpr int W_TILE = 0;                                 // 16 frame rows x 512 B of f16 hi/lo chunks (tile_chunk)
// per-tile record of the speculative top_db clamp (segment_stats): stored log-mel minima per
// pass, the clamps and the processing order ((passes per tile + 2) x kSpecTiles ints)
constexpr int kSpecTiles = 48;   // tiles of frames 0..767 (7.7 s) are recorded and scout-ordered
constexpr int W_SPEC = W_TILE + 16 * NMEL * 4;
constexpr int kSpecRun = (16 / kFPP) * kSpecTiles;      // spec[kSpecRun + tile]: the tile's clamp
constexpr int kSpecOrder = kSpecRun + kSpecTiles;        // spec[kSpecOrder + k]: k-th tile processed
constexpr int W_BYTES = W_SPEC + (kSpecOrder + kSpecTiles) * 4;
constexpr int L_WG = L_SHARED_END + WAVES * W_BYTES;    // ring mode: segment index + per-wave log-mel max/min
constexpr int LDS_BYTES = L_WG + 16 + 8 * WAVES;
constexpr int kRescoreFrames = 16;
// |mean vector| below which the fp64 path decides (round 5: 32, was 64).  Evidence for 32: the
// float32 score error of streaming events is <= 1.2e-5 above |mean| 32 (profiles/r05_v26_mean_err.txt)
// and 600 segments of four other loud recipes with oracle |mean| in [32, 64) score within 8.6e-6
// (round 6, profiles/r06_v1_mean_band_evidence.json); DESIGN.md numerics.
// easywakeword_amd/_lib.py RESCORE_TINY_MEAN mirrors it.
#ifndef EWK_TINY_MEAN
#define EWK_TINY_MEAN 32.0
#endif
constexpr double kTinyMean = EWK_TINY_MEAN;
                                    // (loud audio, c0 cancelling: DESIGN.md numerics)
// A vanishing-mean segment whose float32 similarity percent p = 100 (0.7 sm + 0.3 ss) is below
// -(kNanMarginA / |mean| + kNanMarginB) scores NaN in the reference too (p ** 1.5 of a negative
// p, wakeword.py:621-625): the float32 pass's error in p is far smaller than that (round 6,
// scripts/nan_margin.py: DESIGN.md numerics), so the fp64 re-score cannot change its score or
// decision and the segment is not listed for it.  (Mirrored by _lib.NAN_MARGIN_A / _B.)
#ifndef EWK_NAN_MARGIN_A
#define EWK_NAN_MARGIN_A 0.5
#endif
constexpr double kNanMarginA = EWK_NAN_MARGIN_A;
constexpr double kNanMarginB = 0.05;
constexpr double kTinyStd = 20.0;   // |std vector| below which the fp64 path decides (bench batch >= 24.8,
                                    // streaming events >= 32.5: scripts/std_norm_dist.py)
static_assert(LDS_BYTES <= 160 * 1024, "the workgroup must fit a CU's LDS");
static_assert(16 % kFPP == 0, "passes must tile the 16-frame log-mel tile");


__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

// Eight ds_read_b128 of consecutive 16-B chunks issued together, and their wait.
// Written as asm so the scheduler cannot sink each read next to its first use (at
// 256 VGPRs it does, and every read then costs a full LDS round trip).
#define EWK_LD128(r, a, c) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[c]) : "v"(a), "i"(16 * (c)) : "memory")
#define EWK_LD128_8(r, addr)                                                                        \
    do {                                                                                           \
        const uint32_t _a = (addr);                                                                \
        EWK_LD128(r, _a, 0); EWK_LD128(r, _a, 1); EWK_LD128(r, _a, 2); EWK_LD128(r, _a, 3);         \
        EWK_LD128(r, _a, 4); EWK_LD128(r, _a, 5); EWK_LD128(r, _a, 6); EWK_LD128(r, _a, 7);         \
    } while (0)
#define EWK_WAIT_8(r)                                                                              \
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), \
                 "+v"(r[5]), "+v"(r[6]), "+v"(r[7]) : : "memory")

__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
    return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}

__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 t0 = make_float2(a0.x + a2.x, a0.y + a2.y);
    const float2 t1 = make_float2(a0.x - a2.x, a0.y - a2.y);
    const float2 t2 = make_float2(a1.x + a3.x, a1.y + a3.y);
    const float2 t3 = make_float2(a1.x - a3.x, a1.y - a3.y);
    a0 = make_float2(t0.x + t2.x, t0.y + t2.y);
    a2 = make_float2(t0.x - t2.x, t0.y - t2.y);
    a1 = make_float2(t1.x + t3.y, t1.y - t3.x);   // t1 - i t3
    a3 = make_float2(t1.x - t3.y, t1.y + t3.x);   // t1 + i t3
}

// Second radix-4 stage of the DFT16 with its W16 twiddles folded into FMAs.  Each
// twiddle is written as a real scale times a (1, tan) factor -- W^1 = C1 (1 - iT),
// W^3 = C1 (T - i), W^9 = C1 (-1 + iT), W^2 = R2 (1 - i), W^6 = R2 (-1 - i), T = tan(pi/8)
// -- the two twiddled inputs of a butterfly pair share the scale, and the scale rides
// in the FMAs of the butterfly outputs: 22 / 20 / 22 instructions for rows k1 = 1 / 2 / 3
// instead of 28 / 24 / 28 (three complex multiplies + a radix-4 butterfly).
__device__ __forceinline__ void dft16_stage2(float2 (&x)[16]) {
    constexpr float C1 = 0.92387953251128674f, R2 = 0.70710678118654752f, T = 0.41421356237309505f;
    dft4(x[0], x[1], x[2], x[3]);
    {   // k1 = 1: twiddles W^1, W^2, W^3
        const float2 a0 = x[4], y1 = x[5], y2 = x[6], y3 = x[7];
        const float2 u2 = make_float2(y2.x + y2.y, y2.y - y2.x);                        // Y2 (1 - i)
        const float2 t0 = make_float2(fmaf(R2, u2.x, a0.x), fmaf(R2, u2.y, a0.y));
        const float2 t1 = make_float2(fmaf(-R2, u2.x, a0.x), fmaf(-R2, u2.y, a0.y));
        const float2 u1 = make_float2(fmaf(T, y1.y, y1.x), fmaf(-T, y1.x, y1.y));       // Y1 (1 - iT)
        const float2 u3 = make_float2(fmaf(T, y3.x, y3.y), fmaf(T, y3.y, -y3.x));       // Y3 (T - i)
        const float2 v2 = make_float2(u1.x + u3.x, u1.y + u3.y), v3 = make_float2(u1.x - u3.x, u1.y - u3.y);
        x[4] = make_float2(fmaf(C1, v2.x, t0.x), fmaf(C1, v2.y, t0.y));
        x[6] = make_float2(fmaf(-C1, v2.x, t0.x), fmaf(-C1, v2.y, t0.y));
        x[5] = make_float2(fmaf(C1, v3.y, t1.x), fmaf(-C1, v3.x, t1.y));                // t1 - i C1 v3
        x[7] = make_float2(fmaf(-C1, v3.y, t1.x), fmaf(C1, v3.x, t1.y));                // t1 + i C1 v3
    }
    {   // k1 = 2: twiddles W^2, W^4 = -i, W^6
        const float2 a0 = x[8], y1 = x[9], y2 = x[10], y3 = x[11];
        const float2 t0 = make_float2(a0.x + y2.y, a0.y - y2.x);                        // a0 + (-i Y2)
        const float2 t1 = make_float2(a0.x - y2.y, a0.y + y2.x);
        const float2 u1 = make_float2(y1.x + y1.y, y1.y - y1.x);                        // Y1 (1 - i)
        const float d3 = y3.y - y3.x, n3 = y3.x + y3.y;                                 // Y3 (-1 - i) = (d3, -n3)
        const float2 v2 = make_float2(u1.x + d3, u1.y - n3), v3 = make_float2(u1.x - d3, u1.y + n3);
        x[8] = make_float2(fmaf(R2, v2.x, t0.x), fmaf(R2, v2.y, t0.y));
        x[10] = make_float2(fmaf(-R2, v2.x, t0.x), fmaf(-R2, v2.y, t0.y));
        x[9] = make_float2(fmaf(R2, v3.y, t1.x), fmaf(-R2, v3.x, t1.y));
        x[11] = make_float2(fmaf(-R2, v3.y, t1.x), fmaf(R2, v3.x, t1.y));
    }
    {   // k1 = 3: twiddles W^3, W^6, W^9
        const float2 a0 = x[12], y1 = x[13], y2 = x[14], y3 = x[15];
        const float d2 = y2.y - y2.x, n2 = y2.x + y2.y;                                 // Y2 (-1 - i) = (d2, -n2)
        const float2 t0 = make_float2(fmaf(R2, d2, a0.x), fmaf(-R2, n2, a0.y));
        const float2 t1 = make_float2(fmaf(-R2, d2, a0.x), fmaf(R2, n2, a0.y));
        const float2 u1 = make_float2(fmaf(T, y1.x, y1.y), fmaf(T, y1.y, -y1.x));       // Y1 (T - i)
        const float m3 = fmaf(T, y3.y, y3.x), u3y = fmaf(T, y3.x, -y3.y);               // Y3 (-1 + iT) = (-m3, u3y)
        const float2 v2 = make_float2(u1.x - m3, u1.y + u3y), v3 = make_float2(u1.x + m3, u1.y - u3y);
        x[12] = make_float2(fmaf(C1, v2.x, t0.x), fmaf(C1, v2.y, t0.y));
        x[14] = make_float2(fmaf(-C1, v2.x, t0.x), fmaf(-C1, v2.y, t0.y));
        x[13] = make_float2(fmaf(C1, v3.y, t1.x), fmaf(-C1, v3.x, t1.y));
        x[15] = make_float2(fmaf(-C1, v3.y, t1.x), fmaf(C1, v3.x, t1.y));
    }
}

// In-place radix-4x4 DFT16.  On return x[4*k1 + k2] holds X[k1 + 4*k2].
__device__ __forceinline__ void dft16_perm(float2 (&x)[16]) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(x[n2], x[4 + n2], x[8 + n2], x[12 + n2]);
    dft16_stage2(x);
}

// dft16_perm of the windowed input (x[n].x w[n].x, x[n].y w[n].y): the window products
// ride in the first stage's FMAs (t0 = fma(x0, w0, x2 w2), t1 = fma(x0, w0, -x2 w2)).
__device__ __forceinline__ void dft16_perm_win(float2 (&x)[16], const float2 (&w)[16]) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
        const float2 x0 = x[n2], x1 = x[4 + n2], x2 = x[8 + n2], x3 = x[12 + n2];
        const float2 w0 = w[n2], w1 = w[4 + n2], w2 = w[8 + n2], w3 = w[12 + n2];
        const float2 p2 = make_float2(x2.x * w2.x, x2.y * w2.y), p3 = make_float2(x3.x * w3.x, x3.y * w3.y);
        const float2 t0 = make_float2(fmaf(x0.x, w0.x, p2.x), fmaf(x0.y, w0.y, p2.y));
        const float2 t1 = make_float2(fmaf(x0.x, w0.x, -p2.x), fmaf(x0.y, w0.y, -p2.y));
        const float2 t2 = make_float2(fmaf(x1.x, w1.x, p3.x), fmaf(x1.y, w1.y, p3.y));
        const float2 t3 = make_float2(fmaf(x1.x, w1.x, -p3.x), fmaf(x1.y, w1.y, -p3.y));
        x[n2] = make_float2(t0.x + t2.x, t0.y + t2.y);
        x[8 + n2] = make_float2(t0.x - t2.x, t0.y - t2.y);
        x[4 + n2] = make_float2(t1.x + t3.y, t1.y - t3.x);   // t1 - i t3
        x[12 + n2] = make_float2(t1.x - t3.y, t1.y + t3.x);  // t1 + i t3
    }
    dft16_stage2(x);
}

// Natural-order accessor of dft16_perm's output: X[k] lives in slot perm(k).
__device__ __forceinline__ constexpr int dperm(int k) { return 4 * (k & 3) + (k >> 2); }


// f16 hi/lo split of a float32: hi = x truncated to f16's 11 significant bits (exact in
// f16 over the dB range), lo = x - hi exactly, stored to f16 with round-to-nearest, so
// float(hi) + float(lo) = x within 2^-22 |x|.
__device__ __forceinline__ float f16_trunc(float x) { return __uint_as_float(__float_as_uint(x) & 0xFFFFE000u); }
typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t pk_f16(float a, float b) {   // v_cvt_pk_f16_f32
    halfx2 h;
    h.x = (_Float16)a;
    h.y = (_Float16)b;
    return __builtin_bit_cast(uint32_t, h);
}
__device__ __forceinline__ float f16_lo(uint32_t p) { return (float)__builtin_bit_cast(halfx2, p).x; }
__device__ __forceinline__ float f16_hi(uint32_t p) { return (float)__builtin_bit_cast(halfx2, p).y; }
// eight log-mel values -> their hi chunk and lo chunk (16 B each)
// hi pair = v_cvt_pkrtz_f16_f32 (round toward zero = the 11-bit truncation over the dB
// range), lo = f16(x - float(hi)) by v_fma_mixlo/mixhi_f16 (the subtraction in f32, exact;
// one rounding to f16): 3 VALU per pair instead of 6.
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& l) {
    h = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
    uint32_t r;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(r) : "v"(a), "v"(h), "v"(b));
    l = r;
}
__device__ __forceinline__ void split8(const float (&x)[8], uint4& hi, uint4& lo) {
    split2(x[0], x[1], hi.x, lo.x);
    split2(x[2], x[3], hi.y, lo.y);
    split2(x[4], x[5], hi.z, lo.z);
    split2(x[6], x[7], hi.w, lo.w);
}
// Byte offset of k-chunk c of frame row r in the log-mel tile: the row's hi chunks fill its
// first 256 B and the lo chunks the next 256 B, chunk c at slot c ^ r, so the 16 rows of a
// DCT operand read (one chunk per row) and the 16 chunks of a row write both cover all
// 64 banks.
__device__ __forceinline__ int tile_chunk(int r, int c) { return 512 * r + 16 * (c ^ r); }

// top_db clamp of a log-mel tile (its flat 8 KB LDS image): lane l takes the chunk pairs
// p = l + 64 u (frame row p >> 4, slot p & 15), rebuilds each value exactly as
// float(hi) + float(lo), clamps it at theta and writes the re-split pair back in place.
__device__ __forceinline__ void clamp_load(const float4* src, int lane, uint4 (&h)[4], uint4 (&l)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int p = lane + 64 * u;
        h[u] = __builtin_bit_cast(uint4, src[32 * (p >> 4) + (p & 15)]);
        l[u] = __builtin_bit_cast(uint4, src[32 * (p >> 4) + 16 + (p & 15)]);
    }
}
__device__ __forceinline__ void clamp_store(float* tile, int lane, const uint4 (&h)[4], const uint4 (&l)[4],
                                            float theta) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t hw[4] = {h[u].x, h[u].y, h[u].z, h[u].w}, lw[4] = {l[u].x, l[u].y, l[u].z, l[u].w};
        float x[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[2 * k] = fmaxf(f16_lo(hw[k]) + f16_lo(lw[k]), theta);
            x[2 * k + 1] = fmaxf(f16_hi(hw[k]) + f16_hi(lw[k]), theta);
        }
        uint4 hh, ll;
        split8(x, hh, ll);
        const int p = lane + 64 * u;
        uint4* dst = reinterpret_cast<uint4*>(tile) + 32 * (p >> 4) + (p & 15);
        dst[0] = hh;
        dst[16] = ll;
    }
}

// FFT transpose image of one pass (one real or imaginary plane): row k1 of frame set g
// holds the 64 lanes' values (16 f + j) contiguously, as ds_write_addtid_b32 stores them
// (address = M0 + offset + 4 lane).  Rows are placed so that the untangle's row reads
// -- lane (f, h, j') fetches rows j' and 16 - j' (8 for j' = 0) of frame set h with
// ds_read_b128 -- hit 16 distinct bank quads in every lane group: the row of (r, h)
// starts at quad (j'(r) & 3) + 8 h (mod 16), rows sorted by that shift.
__host__ __device__ constexpr int tr_off(int r, int h) {
    const int jp = r < 8 ? r : (r == 8 ? 0 : 16 - r);
    const int q = (jp >> 2) + (r >= 8 ? 2 : 0);
    return 64 * (16 * h + 4 * (jp & 3) + q) + 4 * ((jp & 3) + 8 * h);   // floats
}

// Segment samples through a buffer descriptor: the hardware range check returns 0
// outside [0, len) (negative offsets wrap to huge unsigned ones), which is exactly
// stft(center=True, pad_mode='constant').  Ring segments wrap at the stream ring.
// RING: 0 linear float32 batch, 1 float32 ring, 2 int16 ring (EWK_RING_I16: the sample
// is x * 32768; the 1/32768 rides in the window table, a power-of-two scale, so the
// windowed products are bit-identical to the float32 ring's).
template <int RING>
struct SegSrc {
    __amdgpu_buffer_rsrc_t rsrc;   // linear: the segment; ring: the whole stream ring
    int32_t len;
    int32_t wrap_at;               // ring: q >= wrap_at -> physical q + start - ring
    int32_t start;                 // ring: physical index of sample 0
    int32_t ring;
};

constexpr int sample_bytes(int ring) { return ring == 2 ? 2 : 4; }

template <int RING>
__device__ __forceinline__ SegSrc<RING> make_src(const void* p, int64_t start, int64_t ring, int32_t len) {
    SegSrc<RING> v;
    const unsigned char* b = static_cast<const unsigned char*>(p) + (RING ? 0 : start * sample_bytes(RING));
    const uint64_t bu = (uint64_t)b;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bu);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(bu >> 32));
    const void* bb = (const void*)(((uint64_t)hi << 32) | lo);
    const int32_t n = __builtin_amdgcn_readfirstlane(RING ? (int32_t)ring : len);
    v.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)bb, (short)0, n * sample_bytes(RING), 0x00020000);
    v.len = __builtin_amdgcn_readfirstlane(len);
    v.start = __builtin_amdgcn_readfirstlane((int32_t)start);
    v.ring = __builtin_amdgcn_readfirstlane((int32_t)ring);
    v.wrap_at = v.ring - v.start;
    return v;
}

// Coalesced staging loads: lane l fetches samples q0 + 64*c + l, c < kStageLoads.
template <int RING>
__device__ __forceinline__ void stage_load(const SegSrc<RING>& v, int q0, int lane, float (&r)[kStageLoads]) {
#pragma unroll
    for (int c = 0; c < kStageLoads; ++c) {
        const int q = q0 + 64 * c + lane;
        int off;
        if (RING) {
            const int phys = q >= v.wrap_at ? q - v.wrap_at : q + v.start;
            off = (unsigned)q < (unsigned)v.len ? phys * sample_bytes(RING) : -1;
        } else {
            off = q * 4;
        }
        if (RING == 2)   // buffer_load_sshort + v_cvt_f32_i32: the int16 sample, exactly
            r[c] = (float)(short)__builtin_amdgcn_raw_buffer_load_b16(v.rsrc, off, 0, 0);
        else
            r[c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(v.rsrc, off, 0, 0));
    }
}

// 13 lane-contiguous rows of 64 floats with ds_write_addtid_b32 (M0 = stage base, saved
// and restored; s_nop 0 for the M0 -> LDS hazard): half the LDS cycles of ds_write_b32
#define EWK_ST13(o)                                                                                            \
    asm volatile("s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %[base]\n\ts_nop 0\n\t"                              \
                 "ds_write_addtid_b32 %[r0] offset:%[o0]\n\tds_write_addtid_b32 %[r1] offset:%[o1]\n\t"          \
                 "ds_write_addtid_b32 %[r2] offset:%[o2]\n\tds_write_addtid_b32 %[r3] offset:%[o3]\n\t"          \
                 "ds_write_addtid_b32 %[r4] offset:%[o4]\n\tds_write_addtid_b32 %[r5] offset:%[o5]\n\t"          \
                 "ds_write_addtid_b32 %[r6] offset:%[o6]\n\tds_write_addtid_b32 %[r7] offset:%[o7]\n\t"          \
                 "ds_write_addtid_b32 %[r8] offset:%[o8]\n\tds_write_addtid_b32 %[r9] offset:%[o9]\n\t"          \
                 "ds_write_addtid_b32 %[r10] offset:%[o10]\n\tds_write_addtid_b32 %[r11] offset:%[o11]\n\t"      \
                 "ds_write_addtid_b32 %[r12] offset:%[o12]\n\ts_mov_b32 m0, %[sv]"                                 \
                 : [sv] "=&s"(m0save)                                                                          \
                 : [base] "s"(m0base), [r0] "v"(r[o]), [r1] "v"(r[o + 1]), [r2] "v"(r[o + 2]), [r3] "v"(r[o + 3]), \
                   [r4] "v"(r[o + 4]), [r5] "v"(r[o + 5]), [r6] "v"(r[o + 6]), [r7] "v"(r[o + 7]),                \
                   [r8] "v"(r[o + 8]), [r9] "v"(r[o + 9]), [r10] "v"(r[o + 10]), [r11] "v"(r[o + 11]),          \
                   [r12] "v"(r[o + 12]), [o0] "i"(stg_off(o)), [o1] "i"(stg_off(o + 1)), [o2] "i"(stg_off(o + 2)), \
                   [o3] "i"(stg_off(o + 3)), [o4] "i"(stg_off(o + 4)), [o5] "i"(stg_off(o + 5)),                    \
                   [o6] "i"(stg_off(o + 6)), [o7] "i"(stg_off(o + 7)), [o8] "i"(stg_off(o + 8)),                    \
                   [o9] "i"(stg_off(o + 9)), [o10] "i"(stg_off(o + 10)), [o11] "i"(stg_off(o + 11)),                \
                   [o12] "i"(stg_off(o + 12))                                                                     \
                 : "memory")
static_assert(kStageLoads == 26, "stage_store writes two blocks of 13 rows");
__device__ __forceinline__ void stage_store(float* stage, int lane, const float (&r)[kStageLoads]) {
    const uint32_t m0base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)stage);
    uint32_t m0save;
    EWK_ST13(0);
    EWK_ST13(13);
}

constexpr int kMelW[8] = {2, 2, 2, 3, 4, 6, 9, 12};   // per 16-band group (checked on the host)
constexpr int kMelIt0[8] = {0, 2, 4, 6, 9, 13, 19, 28};    // first weight of group i in Tables::wpad
// Each group's weights start on a b64 (widths 2) or b128 boundary of the LDS row so one
// group is fetched with 1-3 wide reads right before it is used.
constexpr int kMelOff[8] = {0, 2, 4, 8, 12, 16, 24, 36};
constexpr int kMelRow = 48;
static_assert(kMelRow <= WP && WP % 4 == 0, "mel weight rows");

// Column writes of one frame set's transpose image (one plane: real or imaginary), with
// ds_write_addtid_b32 (address = M0 + offset + 4 lane).
template <int G>
__device__ __forceinline__ void xpose_write(const float2 (&ag)[16], int half, uint32_t m0base) {
    constexpr int g = G;
    float w[16];
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) w[k1] = half ? ag[dperm(k1)].y : ag[dperm(k1)].x;
    // M0 is compiler-reserved: saved and restored in the same statement; the
    // s_nop covers the M0-write -> LDS-use hazard (without it the stores use the old M0)
    uint32_t m0save;
    asm volatile("s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %[base]\n\ts_nop 0\n\t"
                 "ds_write_addtid_b32 %[w0] offset:%[o0]\n\tds_write_addtid_b32 %[w1] offset:%[o1]\n\t"
                 "ds_write_addtid_b32 %[w2] offset:%[o2]\n\tds_write_addtid_b32 %[w3] offset:%[o3]\n\t"
                 "ds_write_addtid_b32 %[w4] offset:%[o4]\n\tds_write_addtid_b32 %[w5] offset:%[o5]\n\t"
                 "ds_write_addtid_b32 %[w6] offset:%[o6]\n\tds_write_addtid_b32 %[w7] offset:%[o7]\n\t"
                 "ds_write_addtid_b32 %[w8] offset:%[o8]\n\tds_write_addtid_b32 %[w9] offset:%[o9]\n\t"
                 "ds_write_addtid_b32 %[w10] offset:%[o10]\n\tds_write_addtid_b32 %[w11] offset:%[o11]\n\t"
                 "ds_write_addtid_b32 %[w12] offset:%[o12]\n\tds_write_addtid_b32 %[w13] offset:%[o13]\n\t"
                 "ds_write_addtid_b32 %[w14] offset:%[o14]\n\tds_write_addtid_b32 %[w15] offset:%[o15]\n\t"
                 "s_mov_b32 m0, %[sv]"
                 : [sv] "=&s"(m0save)
                 : [base] "s"(m0base), [w0] "v"(w[0]), [w1] "v"(w[1]), [w2] "v"(w[2]), [w3] "v"(w[3]),
                   [w4] "v"(w[4]), [w5] "v"(w[5]), [w6] "v"(w[6]), [w7] "v"(w[7]), [w8] "v"(w[8]),
                   [w9] "v"(w[9]), [w10] "v"(w[10]), [w11] "v"(w[11]), [w12] "v"(w[12]),
                   [w13] "v"(w[13]), [w14] "v"(w[14]), [w15] "v"(w[15]),
                   [o0] "i"(4 * tr_off(0, g)), [o1] "i"(4 * tr_off(1, g)), [o2] "i"(4 * tr_off(2, g)),
                   [o3] "i"(4 * tr_off(3, g)), [o4] "i"(4 * tr_off(4, g)), [o5] "i"(4 * tr_off(5, g)),
                   [o6] "i"(4 * tr_off(6, g)), [o7] "i"(4 * tr_off(7, g)), [o8] "i"(4 * tr_off(8, g)),
                   [o9] "i"(4 * tr_off(9, g)), [o10] "i"(4 * tr_off(10, g)), [o11] "i"(4 * tr_off(11, g)),
                   [o12] "i"(4 * tr_off(12, g)), [o13] "i"(4 * tr_off(13, g)), [o14] "i"(4 * tr_off(14, g)),
                   [o15] "i"(4 * tr_off(15, g))
                 : "memory");
}

// One kFPP-frame pass: frames t0 .. t0 + kFPP - 1, samples already staged in `scr`.
// Writes rows [row0, row0 + kFPP) of the log-mel tile (clamped at clampv) and returns the
// per-lane max/min of the valid (unclamped) log-mel values.  If next_t0 >= 0, the samples
// of the pass starting at frame next_t0 are fetched meanwhile and staged at the end.
// `lo[i]` = first bin of band j + 16 i (per lane, loaded once per kernel).
template <int RING>
__device__ __forceinline__ void frame_pass(const SegSrc<RING>& v, int t0, int T, int row0, int next_t0,
                                           const unsigned char* smem, float* scr, float* tile,
                                           int lane, const int (&lo)[8], float& vmax, float& vmin, float& nanp,
                                           float clampv EWK_PASS_PARAM) {
    EWK_TS(fp0);
    EWK_SETPRIO(1);
    // lane group f = lane>>4 holds frames fr = 4 g + f (g < kNF) of this pass; the
    // kNF frames of a lane are independent instruction streams (ILP for the wave).
    const int f = lane >> 4, j = lane & 15;
    // after the transpose lane (h, j') = (j >> 3, j & 7) owns bin columns rowA = j' and
    // rowB = 16 - j' (8 for j' = 0) of frame 4h + f (scratch scf)
    const int jp = j & 7;
    const int rowA = jp, rowB = jp ? 16 - jp : 8;
    float* scf = scr + scr_frame_off(4 * (j >> 3) + f);
    bool valid[kNF];
    float* sc[kNF];
#pragma unroll
    for (int g = 0; g < kNF; ++g) {
        valid[g] = t0 + 2 * f + g < T;
        sc[g] = scr + scr_frame_off(4 * g + f);
    }

    // ---- window the staged samples: lane j holds z[16*n1 + j] = x[32*n1+2j] + i x[32*n1+2j+1]
    // (single ds_read_b64s: the compiler would pair them into ds_read2_b64, which
    // costs the LDS twice the cycles per byte)
    float2 a[kNF][16];
    floatx4 t4[8];   // twiddle row W256^(j*k1)
    {
        float2 x[kNF][16];
        {
            const uint32_t sa = (uint32_t)(uintptr_t)(scr + 352 * f + 2 * j);
#define EWK_LD64(g, n) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(x[g][n]) : "v"(sa), "i"(win_off(g, n)) : "memory")
            EWK_LD64(0, 0); EWK_LD64(0, 1); EWK_LD64(0, 2); EWK_LD64(0, 3); EWK_LD64(0, 4); EWK_LD64(0, 5);
            EWK_LD64(0, 6); EWK_LD64(0, 7); EWK_LD64(0, 8); EWK_LD64(0, 9); EWK_LD64(0, 10); EWK_LD64(0, 11);
            EWK_LD64(0, 12); EWK_LD64(0, 13); EWK_LD64(0, 14); EWK_LD64(0, 15);
            EWK_LD64(1, 11); EWK_LD64(1, 12); EWK_LD64(1, 13); EWK_LD64(1, 14); EWK_LD64(1, 15);
#undef EWK_LD64
        }
        floatx4 w4[8];   // this lane's window pairs, fetched in the same batch
        EWK_LD128_8(w4, (uint32_t)(uintptr_t)(reinterpret_cast<const float4*>(smem + L_WIN2) + j * (TP / 2)));
        EWK_WAIT_8(w4);
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(x[0][0]), "+v"(x[0][1]), "+v"(x[0][2]), "+v"(x[0][3]), "+v"(x[0][4]), "+v"(x[0][5]),
                       "+v"(x[0][6]), "+v"(x[0][7]), "+v"(x[0][8]), "+v"(x[0][9]), "+v"(x[0][10]), "+v"(x[0][11]),
                       "+v"(x[0][12]), "+v"(x[0][13]), "+v"(x[0][14]), "+v"(x[0][15])
                     :
                     : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(x[1][11]), "+v"(x[1][12]), "+v"(x[1][13]), "+v"(x[1][14]), "+v"(x[1][15])
                     :
                     : "memory");
#pragma unroll
        for (int n = 0; n <= 10; ++n) x[1][n] = x[0][n + 5];   // the shared sample pairs
        float2 wv[16];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            wv[2 * c] = make_float2(w4[c].x, w4[c].y);
            wv[2 * c + 1] = make_float2(w4[c].z, w4[c].w);
        }
        EWK_SETPRIO(0);
        // ---- DFT16 over n1 (window folded into its first stage), twiddle W256^(j*k1)
        // (one twiddle row serves every frame of the lane, requested before the DFT16s)
        EWK_LD128_8(t4, (uint32_t)(uintptr_t)(reinterpret_cast<const float4*>(smem + L_TW1) + j * (TP / 2)));
#pragma unroll
        for (int g = 0; g < kNF; ++g) {
#pragma unroll
            for (int n = 0; n < 16; ++n) a[g][n] = x[g][n];
            dft16_perm_win(a[g], wv);
        }
    }
    lds_order();
    EWK_TS(fp1);
    // next pass's samples: issued before the mel stage (registers are free there),
    // stored to the staging area at the end of the pass
    float pf[kStageLoads];
    {
        EWK_WAIT_8(t4);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const floatx4 w = t4[c];   // k1 = 2c+1, 2c+2
#pragma unroll
            for (int g = 0; g < kNF; ++g) {
                a[g][dperm(2 * c + 1)] = cmul(a[g][dperm(2 * c + 1)], make_float2(w.x, w.y));
                if (c < 7) a[g][dperm(2 * c + 2)] = cmul(a[g][dperm(2 * c + 2)], make_float2(w.z, w.w));
            }
        }
    }
    EWK_TS(fp2);
    EWK_SETPRIO(1);
    // ---- transpose through LDS (real, then imaginary half): lane k1 <- A_{n2}[k1].
    // Row r (16 floats) keeps column n in 4-float chunk (n>>2) ^ ((r>>2)&3): the
    // column writes (ds_write_b32, the frames of a 32-lane half 272 floats apart) and
    // the row reads (ds_read_b128) are both bank-conflict free.
    float2 b[kNF][16];
    {
        const uint32_t m0base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)scr);
        const int offA = tr_off(rowA, j >> 3) + 16 * f, offB = tr_off(rowB, j >> 3) + 16 * f;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
            for (int g = 0; g < kNF; ++g) {
                if (g == 0) xpose_write<0>(a[0], half, m0base);
                else xpose_write<1>(a[1], half, m0base);
            }
            lds_order();
            // lane (h, j') = (j >> 3, j & 7) reads two columns of frame 4h + f: c0 = j' and its
            // conjugate partner 16 - j' (column 8 beside column 0 for j' = 0)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const float4* rd = reinterpret_cast<const float4*>(scr + (s2 ? offB : offA));
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float4 q = rd[c];
                    if (half) {
                        b[s2][4 * c].y = q.x; b[s2][4 * c + 1].y = q.y; b[s2][4 * c + 2].y = q.z; b[s2][4 * c + 3].y = q.w;
                    } else {
                        b[s2][4 * c].x = q.x; b[s2][4 * c + 1].x = q.y; b[s2][4 * c + 2].x = q.z; b[s2][4 * c + 3].x = q.w;
                    }
                }
            }
            lds_order();
        }
    }
    EWK_TS(fp3);
    EWK_SETPRIO(0);
    // ---- DFT16 over n2: Z[j + 16*k2] = b[dperm(k2)]
#pragma unroll
    for (int g = 0; g < kNF; ++g) dft16_perm(b[g]);
    EWK_TS(fp4);
    // ---- untangle + power, two conjugate bins per step, no cross-lane traffic.  For
    // k = c0 + 16 it the partner Zp = Z[256 - k] sits in this lane's other column; with
    // A = Z[k] + conj(Zp), B = Z[k] - conj(Zp), C = i W512^k B:
    //   P'[k] = |2 X[k]|^2 = |A - C|^2,  P'[256 - k] = |A + C|^2.
    // Lanes j' = 1..7: it = 0..15 (it = 16 repeats it = 15).  Lane j' = 0 pairs column
    // 0 with itself (it = 0..8: k = 16 it, 256 - k; it = 0 yields bin 256) and column 8
    // with itself (it = 9..16: k = 8 + 16 (it - 9)).
    {
        const bool z0 = jp == 0;
        // the 17 twiddles of this lane class, fetched up front (9 ds_read_b128): read one
        // step ahead they cost an LDS round trip per step behind that step's writes
        float2 tw[18];
        {
            const float4* t4 = reinterpret_cast<const float4*>(smem + L_TW2) + jp * (TP / 2);   // [j'][it], 17 entries
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                const float4 q = t4[c];
                tw[2 * c] = make_float2(q.x, q.y);
                tw[2 * c + 1] = make_float2(q.z, q.w);
            }
        }
        float* pA0 = scf + rowA;                     // P[k]      at pA0[16 it]       (it <= 15)
        float* pA1 = z0 ? scf - 136 : pA0;           //           lane 0, it >= 9
        float* pA2 = z0 ? scf - 136 : pA0 - 16;      //           it = 16
        float* pB0 = scf - rowA;                     // P[256-k]  at pB0[256 - 16 it]
        float* pB1 = z0 ? scf + 136 : pB0;
        float* pB2 = z0 ? scf + 136 : pB0 + 16;
        // two steps per iteration, their stores grouped by base (pa, pa, pb, pb) so that
        // the stores of consecutive steps merge into ds_write2_b32
#pragma unroll
        for (int it0 = 0; it0 < 17; it0 += 2) {
            float py[2], px[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int it = it0 + u;
                if (it >= 17) break;
                const float2 w = tw[it];   // (cos, tan)(2 pi k / 512)
                const float2 ug = b[0][dperm(it < 16 ? it : 15)];
                const float2 vg = b[1][dperm(it < 16 ? 15 - it : 0)];
                float2 uu, vv;
                if (it <= 8) {
                    uu = ug;
                    const float2 vz = b[0][dperm((16 - it) & 15)];
                    vv = z0 ? vz : vg;
                } else {
                    const float2 uz = b[1][dperm(it - 9)], vz = b[1][dperm(24 - it)];
                    uu = z0 ? uz : ug;
                    vv = z0 ? vz : vg;
                }
                const float ar = uu.x + vv.x, ai = uu.y - vv.y;
                const float br = uu.x - vv.x, bi = uu.y + vv.y;
                // w = (c, t = s / c): C = c (t br - bi, t bi + br), its scale in the output FMAs
                const float er = fmaf(w.y, br, -bi), ei = fmaf(w.y, bi, br);
                const float yr = fmaf(-w.x, er, ar), yi = fmaf(-w.x, ei, ai);
                const float xr = fmaf(w.x, er, ar), xi = fmaf(w.x, ei, ai);
                py[u] = yr * yr + yi * yi;
                px[u] = xr * xr + xi * xi;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int it = it0 + u;
                if (it >= 17) break;
                float* pa = it <= 8 ? pA0 : (it < 16 ? pA1 : pA2);
                pa[16 * it] = py[u];
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int it = it0 + u;
                if (it >= 17) break;
                float* pb = it <= 8 ? pB0 : (it < 16 ? pB1 : pB2);
                pb[256 - 16 * it] = px[u];
            }
        }
        // the zero pad (bins 257..271) the unrolled band loops read past bin 256
        scf[257 + jp] = 0.0f;
        if (jp < 7) scf[265 + jp] = 0.0f;
    }
    lds_order();
    EWK_TS(fp5);
    EWK_SETPRIO(1);
    if (next_t0 >= 0) stage_load(v, next_t0 * HOP - NFFT / 2, lane, pf);
    // ---- mel + log: lane j computes bands m = j + 16*i of its frames (weights shared).
    // The stage's LDS reads go in two batches (band groups 0-5, then 6-7: 19 and 21
    // weights), each followed by its FMAs -- one wait per batch, not one per group.
    float db[kNF][8];
    {
        const float* wrow = reinterpret_cast<const float*>(smem + L_WPAD) + j * WP;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int i0 = hh ? 6 : 0, i1 = hh ? 8 : 6;
            float wv[MEL_ITERS], pv[kNF][MEL_ITERS];
#pragma unroll
            for (int i = i0; i < i1; ++i) {
                if (kMelW[i] <= 2) {
                    const float2 w = *reinterpret_cast<const float2*>(wrow + kMelOff[i]);
                    wv[kMelIt0[i]] = w.x; wv[kMelIt0[i] + 1] = w.y;
                } else {
#pragma unroll
                    for (int c = 0; c < (kMelW[i] + 3) / 4; ++c) {
                        const float4 w = *reinterpret_cast<const float4*>(wrow + kMelOff[i] + 4 * c);
                        const float ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (4 * c + e < kMelW[i]) wv[kMelIt0[i] + 4 * c + e] = ww[e];
                    }
                }
#pragma unroll
                for (int g = 0; g < kNF; ++g) {
                    const float* sp = sc[g] + lo[i];
#pragma unroll
                    for (int q = 0; q < kMelW[i]; ++q) pv[g][kMelIt0[i] + q] = sp[q];
                }
            }
#pragma unroll
            for (int i = i0; i < i1; ++i)
#pragma unroll
                for (int g = 0; g < kNF; ++g) {
                    float acc = 0.0f;
#pragma unroll
                    for (int q = 0; q < kMelW[i]; ++q) acc = fmaf(wv[kMelIt0[i] + q], pv[g][kMelIt0[i] + q], acc);
                    // 10*log10(x) = (10*log10(2)) * log2(x), v_log_f32
                    db[g][i] = 3.0102999566398120f * __log2f(fmaxf(1e-10f, acc));
                    // NaN probe: a NaN sample makes every bin of its frame NaN, which the
                    // amin floor above would hide (fmax returns the number); the reference's
                    // np.maximum propagates it and scores NaN (acc * 0 is NaN for NaN / Inf)
                    if (i == 0) nanp = fmaf(acc, 0.0f, nanp);
                }
        }
    }
    EWK_SETPRIO(0);
    lds_order();
    EWK_TS(fp6);
    // Rows of frames past T keep their (finite: silence gives -100 dB) values: the DCT
    // columns are independent and the statistics skip those frames, so only the frame's
    // max/min needs the validity test, once per frame.  The eight bands of a lane form
    // k-chunk j of its frame row (hi and lo halves, one ds_write_b128 each).
#pragma unroll
    for (int g = 0; g < kNF; ++g) {
        const int r = row0 + 2 * f + g;
        float fmx = db[g][0], fmn = db[g][0], x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            fmx = fmaxf(fmx, db[g][i]);
            fmn = fminf(fmn, db[g][i]);
            x[i] = fmaxf(db[g][i], clampv);   // top_db recompute path; -inf folds away otherwise
        }
        vmax = fmaxf(vmax, valid[g] ? fmx : -INFINITY);
        vmin = fminf(vmin, valid[g] ? fmn : INFINITY);
        uint4 hi, lo;
        split8(x, hi, lo);
        unsigned char* tb = reinterpret_cast<unsigned char*>(tile) + tile_chunk(r, j);
        *reinterpret_cast<uint4*>(tb) = hi;
        *reinterpret_cast<uint4*>(tb + 256) = lo;
    }
    lds_order();
    if (next_t0 >= 0) stage_store(scr, lane, pf);
    lds_order();
#ifdef EWK_TIMING
    EWK_TS(fp7);
    if (pdbg) {
        pdbg[12] += fp1 - fp0; pdbg[13] += fp2 - fp1; pdbg[14] += fp3 - fp2; pdbg[15] += fp4 - fp3;
        pdbg[16] += fp5 - fp4; pdbg[17] += fp6 - fp5; pdbg[18] += fp7 - fp6; pdbg[19] += 1;
    }
#endif
}

// DCT of one 16-frame log-mel tile on the matrix cores: C[32 x 16] = D[32 x 128] X[128 x 16]
// with v_mfma_f32_16x16x32_f16 on the f16 hi/lo splits, three products per k-step
// (Dh Xh + Dh Xl + Dl Xh, f32 accumulation; the dropped Dl Xl is ~2^-22 relative).
// Lane l gets C[row = 4h + r][frame col] of both row tiles (h = l>>4, col = l&15) in
// c[0..3], c[4..7] -- the layout of the f32 16x16x4 MFMA.  The operands of k-step q
// (6 ds_read_b128) are requested one step ahead of its 6 MFMAs.
#define EWK_DCT_RD(dst, addr, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(off) : "memory")
#define EWK_DCT_LOAD(p, q)                                                   \
    do {                                                                     \
        EWK_DCT_RD(Bh[p], bq[q], 0);                                         \
        EWK_DCT_RD(Bl[p], bq[q], 256);                                       \
        EWK_DCT_RD(A0h[p], a0, 2048 * (q));                                  \
        EWK_DCT_RD(A0l[p], a0, 2048 * (q) + 1024);                           \
        EWK_DCT_RD(A1h[p], a1, DCT_RT1_STRIDE * (2 * (q)));                  \
        EWK_DCT_RD(A1l[p], a1, DCT_RT1_STRIDE * (2 * (q) + 1));              \
    } while (0)
#define EWK_DCT_WAIT(p, n)                                                                               \
    asm volatile("s_waitcnt lgkmcnt(" #n ")"                                                             \
                 : "+v"(Bh[p]), "+v"(Bl[p]), "+v"(A0h[p]), "+v"(A0l[p]), "+v"(A1h[p]), "+v"(A1l[p]) \
                 :                                                                                       \
                 : "memory")
#define EWK_MF(a, b, acc) \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a), __builtin_bit_cast(halfx8, b), acc, 0, 0, 0)
#define EWK_DCT_MFMA(p)                                                                        \
    do {                                                                                       \
        EWK_MF(A0h[p], Bh[p], acc0); EWK_MF(A1h[p], Bh[p], acc1);                              \
        EWK_MF(A0h[p], Bl[p], acc0); EWK_MF(A1h[p], Bl[p], acc1);                              \
        EWK_MF(A0l[p], Bh[p], acc0); EWK_MF(A1l[p], Bh[p], acc1);                              \
    } while (0)
__device__ __forceinline__ void tile_dct(const float* tile, const float* s_dct, int lane, float (&c)[8]) {
    const int col = lane & 15, g4 = lane >> 4;
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    // B of k-step q: chunk 4q + g4 of frame row col, at slot (4q + g4) ^ col =
    // 4 (q ^ (col >> 2)) + (g4 ^ (col & 3))
    const uint32_t tb = (uint32_t)(uintptr_t)tile + 512 * col + 16 * (g4 ^ (col & 3));
    uint32_t bq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[q] = tb + 64 * (q ^ (col >> 2));
    const uint32_t db = (uint32_t)(uintptr_t)s_dct;
    const uint32_t a0 = db + 16 * lane;
    const uint32_t a1 = db + DCT_RT1 + 16 * (col < 4 ? 4 * g4 + col : 16);
    floatx4 Bh[2], Bl[2], A0h[2], A0l[2], A1h[2], A1l[2];
    EWK_DCT_LOAD(0, 0);
    EWK_DCT_LOAD(1, 1);
    EWK_DCT_WAIT(0, 6);
    EWK_DCT_MFMA(0);
    EWK_DCT_LOAD(0, 2);
    EWK_DCT_WAIT(1, 6);
    EWK_DCT_MFMA(1);
    EWK_DCT_LOAD(1, 3);
    EWK_DCT_WAIT(0, 6);
    EWK_DCT_MFMA(0);
    EWK_DCT_WAIT(1, 0);
    EWK_DCT_MFMA(1);
    lds_order();
#pragma unroll
    for (int i = 0; i < 4; ++i) { c[i] = acc0[i] * (1.0f / kDctScale); c[4 + i] = acc1[i] * (1.0f / kDctScale); }
}
#undef EWK_DCT_RD
#undef EWK_DCT_LOAD
#undef EWK_DCT_WAIT
#undef EWK_DCT_MFMA
#undef EWK_MF

// fp64 shifted sums of the frame columns that exist (d = c - cref).
__device__ __forceinline__ void stats_add(const float (&c)[8], const float (&cref)[8], bool ok, double (&s1)[8],
                                          double (&s2)[8]) {
    if (ok) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double d = (double)c[i] - (double)cref[i];
            s1[i] += d;
            s2[i] = fma(d, d, s2[i]);
        }
    }
}

// Swap one tile's contribution: remove the unclamped columns `co`, add the clamped `cn`.
__device__ __forceinline__ void stats_replace(const float (&cn)[8], const float (&co)[8], const float (&cref)[8],
                                              bool ok, double (&s1)[8], double (&s2)[8]) {
    if (ok) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double dn = (double)cn[i] - (double)cref[i], dd = (double)co[i] - (double)cref[i];
            s1[i] += dn - dd;
            s2[i] += fma(dn, dn, -dd * dd);
        }
    }
}

// Wave minimum of a float, no LDS: DPP row scan, then the four row results via readlane.
__device__ __forceinline__ float wave_min(float x) {
    x = fminf(x, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), 0x111, 0xf, 0xf, false)));
    x = fminf(x, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), 0x112, 0xf, 0xf, false)));
    x = fminf(x, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), 0x114, 0xf, 0xf, false)));
    x = fminf(x, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), 0x118, 0xf, 0xf, false)));
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 15));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 31));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 47));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
    return fminf(fminf(r0, r1), fminf(r2, r3));
}

// Sum over the 16 lanes of each row (DPP row_shr scan, no LDS); the total lands in lane 15 of the row.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {   // DPP move of a double; lanes without a source read 0
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double row_sum_d(double x) {
    x += dpp_d<0x111>(x);   // row_shr:1
    x += dpp_d<0x112>(x);   // row_shr:2
    x += dpp_d<0x114>(x);   // row_shr:4
    x += dpp_d<0x118>(x);   // row_shr:8
    return x;
}

// Sum over the wave (rows via DPP, then the four row totals via readlane); uniform result.
__device__ __forceinline__ double wave_sum_d(double x) {
    x = row_sum_d(x);
    double t = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        t += __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), 16 * r + 15),
                              __builtin_amdgcn_readlane(__double2loint(x), 16 * r + 15));
    return t;
}

// Sum of a float over the wave (DPP row scans, the row totals via readlane); uniform result.
__device__ __forceinline__ float wave_sum_f(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x112, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x114, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x118, 0xf, 0xf, false));
    return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 15)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 31))) +
           (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 47)) +
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63)));
}

// Wave maximum of a float (see wave_min).
__device__ __forceinline__ float wave_max(float x) { return -wave_min(-x); }

// Reduce the per-lane sums over the 16 frame columns (DPP, totals in lane 15 of each
// row), hand each coefficient's (S1, S2, cref) to lane k = coefficient through the
// wave's scratch `pd` (20 x 3 doubles), and finish there: lane k < 20 returns its mean in
// s1[0] and its population std in s2[0] (one fp64 division + sqrt per lane, not eight).
__device__ __forceinline__ void finish_stats(int T, const float (&cref)[8], double (&s1)[8], double (&s2)[8],
                                             int lane, double* pd) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        s1[i] = row_sum_d(s1[i]);
        s2[i] = row_sum_d(s2[i]);
    }
    if ((lane & 15) == 15) {
        const int h = lane >> 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = 4 * h + r;
            pd[3 * k] = s1[r]; pd[3 * k + 1] = s2[r]; pd[3 * k + 2] = (double)cref[r];
            if (h == 0) {
                const int k2 = 16 + r;
                pd[3 * k2] = s1[4 + r]; pd[3 * k2 + 1] = s2[4 + r]; pd[3 * k2 + 2] = (double)cref[4 + r];
            }
        }
    }
    lds_order();
    if (lane < NMFCC) {
        const double S1 = pd[3 * lane], S2 = pd[3 * lane + 1], r0 = pd[3 * lane + 2];
        const double Td = (double)T;
        const double mean = r0 + S1 / Td;
        double var = (S2 - S1 * S1 / Td) / Td;
        var = var > 0.0 ? var : 0.0;
        s1[0] = mean;
        s2[0] = sqrt(var);
    }
    lds_order();
}

// Zero the kFPP tile rows of one pass (frames past T).
__device__ __forceinline__ void zero_rows(float* tile, int row0, int lane) {
    for (int m = lane; m < kFPP * NMEL; m += 64) tile[row0 * NMEL + m] = 0.0f;
}

// The tiles of one segment that pass 1 left holding a value below the final max - 80 dB
// are recomputed: the stored tile (clamped at its speculative `run`, rebuilt bit for bit
// by the same frame passes) gives the pass-1 DCT columns to remove, the tile clamped at
// theta in LDS the columns to add.  (Parking every tile in global memory for this pass
// instead wrote 10 KB per 16 frames -- 2.3x the algorithmic traffic -- for the ~16 % of
// bench tiles that need it; recomputing those costs the same time.  Parking only the tiles
// the scout ranks within 3 dB of a later one -- 2.8 per bench segment, 0.47 of them fixed --
// lost 1.5 % too: the parking stores hold up the next pass's vmcnt waits, and a reload
// costs 2/3 of a recompute.  profiles/r03_v2_park_ab.txt.  Rebuilding a self-clamped tile's
// stored image exactly -- its clamp at the run before it, then at its own -- so that the
// columns taken out equal the ones put in to the last bit cost 1.3 %, for score changes of
// ~1e-9: the fix-up recomputes at the tile's final run.  A full-coverage scout (Hann-weighted
// frame energies from every sample, scripts/scout_sim.py H8) cut the recomputes from 0.53 to
// 0.11 tiles per bench segment but its loads cost 4x the time saved: r03_v3_scout_ab.txt.)
// Passes of one tile; `mask` bit p selects pass p (the others' rows are zeroed, like the
// rows of frames past T).
constexpr int kPassesPerTile = 16 / kFPP;
constexpr int kAllPasses = (1 << kPassesPerTile) - 1;
template <int RING>
__device__ __forceinline__ void tile_passes(const SegSrc<RING>& v, int tile_i, int T, const unsigned char* smem,
                                            float* scr, float* tile, int lane, const int (&lo)[8], float& mx,
                                            float& mn, float& nanp, float clampv, int mask = kAllPasses) {
    const int npass = (T + kFPP - 1) / kFPP;
    const int p0 = tile_i * kPassesPerTile;
    mask &= npass - p0 >= kPassesPerTile ? kAllPasses : (1 << max(0, npass - p0)) - 1;
    if (mask) {   // stage the tile's first selected pass
        float r[kStageLoads];
        stage_load(v, (p0 + __builtin_ctz(mask)) * kFPP * HOP - NFFT / 2, lane, r);
        stage_store(scr, lane, r);
        lds_order();
    }
#pragma unroll 1
    for (int p = 0; p < kPassesPerTile; ++p) {
        if ((mask >> p) & 1) {
            const int rest = mask >> (p + 1);   // the next selected pass of this tile is prefetched
            frame_pass(v, (p0 + p) * kFPP, T, p * kFPP, rest ? (p0 + p + 1 + __builtin_ctz(rest)) * kFPP : -1,
                       smem, scr, tile, lane, lo, mx, mn, nanp, clampv EWK_PASS_ARG(nullptr));
        } else {   // frames past T, or a pass left out: zero rows (their columns are not used)
            zero_rows(tile, p * kFPP, lane);
        }
    }
    lds_order();
}

// The passes in `mask` of a tile whose stored values (clamped at `run`) include some below
// the final threshold: recomputed bit for bit, their DCT columns swapped from clamped-at-run
// to clamped-at-theta in the shifted sums.  A pass whose stored minimum is >= theta is
// unchanged and skipped (per-pass records, segment_stats).
template <int RING>
__device__ __forceinline__ void fix_tile(const SegSrc<RING>& v, int tile_i, int T, float run, float theta,
                                         const unsigned char* smem, float* scr, float* tile, int lane,
                                         const int (&lo)[8], const float (&cref)[8], double (&s1)[8],
                                         double (&s2)[8], int mask = kAllPasses) {
    const float* s_dct = reinterpret_cast<const float*>(smem + L_DCT);
    float d0 = 0.f, d1 = 0.f, d2 = 0.f;
    tile_passes(v, tile_i, T, smem, scr, tile, lane, lo, d0, d1, d2, run, mask);
    float co[8], cn[8];
    tile_dct(tile, s_dct, lane, co);
    {
        uint4 h[4], l[4];
        clamp_load(reinterpret_cast<const float4*>(tile), lane, h, l);
        clamp_store(tile, lane, h, l, theta);
    }
    lds_order();
    tile_dct(tile, s_dct, lane, cn);
    const int col = lane & 15;
    stats_replace(cn, co, cref, tile_i * 16 + col < T && ((mask >> (col / kFPP)) & 1), s1, s2);
}

// Scout of a segment's tiles (tile t: frames 16t .. 16t + 15): the energy of 4 x 64 of its
// samples (one 64-sample row every 640), wave-reduced; lane t returns the estimate for tile
// t (t < ntile <= 64).  Only a processing-order heuristic: the results do not depend on it.
constexpr int kScoutBatch = 8;   // tiles whose scout loads are in flight together
template <int RING, int NB>
__device__ __forceinline__ void scout_batch(const SegSrc<RING>& v, int t0, int lane, float& e) {
    float x[NB][4];
#pragma unroll
    for (int u = 0; u < NB; ++u) {   // tiles t0 + u (past the segment: range-checked zeros)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int qs = (t0 + u) * 16 * HOP + 640 * q + 64 + lane;
            int off;
            if (RING) {
                const int phys = qs >= v.wrap_at ? qs - v.wrap_at : qs + v.start;
                off = (unsigned)qs < (unsigned)v.len ? phys * sample_bytes(RING) : -1;
            } else {
                off = qs * 4;
            }
            if (RING == 2)
                x[u][q] = (float)(short)__builtin_amdgcn_raw_buffer_load_b16(v.rsrc, off, 0, 0);
            else
                x[u][q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(v.rsrc, off, 0, 0));
        }
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        float a = x[u][0] * x[u][0];
#pragma unroll
        for (int q = 1; q < 4; ++q) a = fmaf(x[u][q], x[u][q], a);
        const float tot = wave_sum_f(a);
        if (lane == t0 + u) e = tot;
    }
}

// Scout of a segment's tiles (tile t: frames 16t .. 16t + 15): the energy of 4 x 64 of its
// samples (one 64-sample row every 640), wave-reduced; lane t returns the estimate for tile
// t (t < ntile <= 64).  Only a processing-order heuristic: the results do not depend on it.
// The loads of 8 tiles are in flight together (one memory round trip per 1.3 s of segment).
// (scripts/scout_sim.py replays the order on the oracle's log-mel: this scout leaves ~7 % of
// the bench's tiles to recompute, none with the true tile maxima; max-of-rows variants and
// twice the loads reach 6.1 %.)
template <int RING>
__device__ __forceinline__ float scout_tiles(const SegSrc<RING>& v, int ntile, int lane) {
    float e = -1.0f;
    for (int t0 = 0; t0 < ntile; t0 += kScoutBatch) {
        // the batch sized to the tiles left (a short segment's scout issues 2 or 4 tiles' loads
        // and reductions, not 8)
        const int left = ntile - t0;
        if (left <= 2) scout_batch<RING, 2>(v, t0, lane, e);
        else if (left <= 4) scout_batch<RING, 4>(v, t0, lane, e);
        else scout_batch<RING, kScoutBatch>(v, t0, lane, e);
    }
    return e;
}

// The next work item of a persistent wave (linear batches, ring mode 2), claimed ahead:
// its index is requested when the current segment's last tile starts, its work-order entry
// when that tile's passes end and its descriptor before the fix-ups, so neither the atomic
// nor the two dependent loads sit between two segments.  (Claiming at the segment start
// instead holds a reservation for a whole segment and costs more at the batch tail.)
struct WorkAhead {
    int state = 0;      // 0 none, 1 index requested (lane 0), 2 index known, 3 described
    bool first = true;  // the wave's first claim: its own index, no atomic
    int idx = 0;
    int seg = 0;
    int64_t start = 0;
    int32_t len = 0;
    int32_t stream = 0;
    int32_t flags = 0;
};
struct WorkCtx {
    const ScoreArgs* a;
    int base, count;
    bool ahead;         // claim the next item during this segment
    int wid, nw;        // this wave's index in the grid, the grid's waves
};

// The first item of every wave is its own index (work items 0 .. nw - 1), the rest come from
// the counter: one device-scope fetch-add address serves ~1 claim per 11 ns, and a launch's
// first claims all arrive together (2,048 of them: ~23 us for the last;
// scripts/probes/atomic_probe.hip).
template <int RING>
__device__ __forceinline__ void work_claim(const WorkCtx& c, WorkAhead& w, int lane) {
    if (w.first) {
        w.idx = c.wid;
        w.first = false;
    } else if (lane == 0) {
        w.idx = c.nw + atomicAdd(c.a->work, 1);
    }
    w.state = 1;
}
template <int RING>
__device__ __forceinline__ void work_order(const WorkCtx& c, WorkAhead& w) {
    w.idx = __shfl(w.idx, 0, 64);
    w.state = 2;
    if (w.idx < c.count) w.seg = c.base + ((!RING && c.a->order) ? c.a->order[w.idx] : w.idx);
}
template <int RING>
__device__ __forceinline__ void work_describe(const WorkCtx& c, WorkAhead& w) {
    w.state = 3;
    if (w.idx >= c.count) return;
    if (RING) {
        const ewk_event ev = c.a->events[w.seg];
        w.start = ev.ring_start;
        w.len = ev.length;
        w.stream = ev.stream;
        w.flags = ev.flags;
    } else {
        w.start = c.a->offsets[w.seg];
        w.len = c.a->lengths[w.seg];
    }
}

// Whole segment for one wave.  spec: this wave's per-tile record in LDS -- the stored
// log-mel minimum of pass p of tile i in spec[kPassesPerTile * i + p], the tile's
// speculative clamp in spec[kSpecRun + i] (tiles past kSpecTiles are stored unclamped and
// always recomputed when theta bites), then the processing order (spec[kSpecOrder + k]).
//
// The top_db clamp (max - 80 dB over the whole segment) is applied speculatively at the
// running max, which each tile updates before its DCT; a tile that already holds the
// segment max needs no fix, so the tiles are processed loudest first by a scout estimate
// (bench batch: 16 % of the tiles recomputed in time order, ~5 % in scout order), and only
// the passes of a tile that hold a value below the final threshold are recomputed.
template <int RING>
__device__ void segment_stats(const SegSrc<RING>& v, const unsigned char* smem, float* scr, float* tile,
                              float* spec, int lane, const int (&lo)[8], double (&s1)[8], double (&s2)[8],
                              float& theta_out, const WorkCtx& wc, WorkAhead& nx EWK_DBG_PARAM) {
    EWK_TS(tq0);
    const float* s_dct = reinterpret_cast<const float*>(smem + L_DCT);
    const int T = 1 + v.len / HOP;
    const int ntile = (T + 15) >> 4;
    const int npass = (T + kFPP - 1) / kFPP;
    const int col = lane & 15;
    int* order = reinterpret_cast<int*>(spec + kSpecOrder);
    const bool ordered = ntile > 1 && ntile <= kSpecTiles;
    if (ordered) {   // loudest-first order: lane t ranks tile t (ties by index)
        float e = scout_tiles(v, ntile, lane);
        e = e == e ? e : 0.0f;   // NaN samples: a total order (unique ranks) all the same
        int rank = 0;
        for (int u = 0; u < ntile; ++u) {
            const float eu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), u));
            rank += (eu > e) || (eu == e && u < lane);
        }
        if (lane < ntile) order[rank] = lane;
        lds_order();
    }
    EWK_TS(tq1);
    EWK_TADD(1, tq0, tq1);
    float cref[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { s1[i] = 0.0; s2[i] = 0.0; cref[i] = 0.0f; }
    float vmax = -INFINITY, vmin = INFINITY, nanp = 0.0f;
    int tile_i = ordered ? order[0] : 0;
    {   // stage the first pass synchronously
        float r[kStageLoads];
        stage_load(v, tile_i * 16 * HOP - NFFT / 2, lane, r);
        stage_store(scr, lane, r);
        lds_order();
    }
    EWK_TS(tq2);
    EWK_TADD(2, tq1, tq2);
    float run = -INFINITY;   // speculative clamp: running max - 80 dB
    for (int k = 0; k < ntile; ++k) {
        EWK_TS(tk0);
        const int next_tile = k + 1 < ntile ? (ordered ? order[k + 1] : k + 1) : -1;
        const bool rec = tile_i < kSpecTiles;
        float tmw = INFINITY;
        if (!rec) run = -INFINITY;
        const bool last = k + 1 == ntile;
        if (last && wc.ahead) work_claim<RING>(wc, nx, lane);
#pragma unroll 1
        for (int p = 0; p < kPassesPerTile; ++p) {
            const int pass = tile_i * kPassesPerTile + p;
            // the next pass to prefetch: this tile's next, else the next tile's first
            const int nxt = p + 1 < kPassesPerTile && pass + 1 < npass ? (pass + 1) * kFPP
                                                                      : (next_tile >= 0 ? next_tile * 16 : -1);
            float tp = INFINITY;
            if (pass < npass)
                frame_pass(v, pass * kFPP, T, p * kFPP, nxt, smem, scr, tile, lane, lo, vmax, tp, nanp, run EWK_PASS_ARG(dbg));
            else   // rows of frames past T: zero (ignored by the statistics)
                zero_rows(tile, p * kFPP, lane);
            const float tpw = wave_min(tp);   // this pass's minimum (its record below)
            tmw = fminf(tmw, tpw);
            if (lane == 0 && rec) spec[kPassesPerTile * tile_i + p] = tpw;
        }
        lds_order();
        EWK_TS(tk1);
        EWK_TADD(3, tk0, tk1);
        if (last && wc.ahead) work_order<RING>(wc, nx);
        // max(max(x, run), final) = max(x, final): a tile stored clamped at the running max
        // (this tile's own values included) is exact unless a later tile raises the max
        const float run2 = rec ? wave_max(vmax) - kTopDbUnits : -INFINITY;
        if (run2 > run && tmw < run2) {   // this tile raised the max over some of its own values
            uint4 h[4], l[4];
            clamp_load(reinterpret_cast<const float4*>(tile), lane, h, l);
            clamp_store(tile, lane, h, l, run2);
            lds_order();
        }
        run = fmaxf(run, run2);
        float c[8];
        tile_dct(tile, s_dct, lane, c);
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cref[i] = __shfl(c[i], lane & 48, 64);
        }
        stats_add(c, cref, tile_i * 16 + col < T, s1, s2);
        vmin = fminf(vmin, tmw);
        if (lane == 0 && rec) {   // stored minima: the pass minima as clamped at the tile's run
#pragma unroll
            for (int p = 0; p < kPassesPerTile; ++p)
                spec[kPassesPerTile * tile_i + p] = fmaxf(spec[kPassesPerTile * tile_i + p], run);
            spec[kSpecRun + tile_i] = run;
        }
        tile_i = next_tile;
        EWK_TS(tk2);
        EWK_TADD(4, tk1, tk2);
    }
    EWK_TS(tq3);
    if (wc.ahead) work_describe<RING>(wc, nx);
    // wave-wide log-mel max
    vmax = wave_max(vmax);
    const float theta = vmax - kTopDbUnits;
    theta_out = theta;
    if (vmin < theta) {
        lds_order();
        for (int cur = 0; cur < ntile; ++cur) {
            const bool rec = cur < kSpecTiles;
            int mask = kAllPasses;
            if (rec) {   // only the passes holding a stored value below theta change
                mask = 0;
#pragma unroll
                for (int p = 0; p < kPassesPerTile; ++p) mask |= (spec[kPassesPerTile * cur + p] < theta ? 1 : 0) << p;
                if (!mask) continue;
            }
#ifdef EWK_TIMING
            dbg[10] += 1;
            dbg[11] += __builtin_popcount(mask);
#endif
            fix_tile(v, cur, T, rec ? spec[kSpecRun + cur] : -INFINITY, theta, smem, scr, tile, lane, lo, cref, s1,
                     s2, mask);
        }
    }
    if (__ballot(nanp != nanp)) {   // NaN input: NaN statistics, NaN score (like the reference)
#pragma unroll
        for (int i = 0; i < 8; ++i) s1[i] = __builtin_nan("");
    }
    EWK_TS(tq4);
    EWK_TADD(5, tq3, tq4);
#ifndef EWK_SKIP_EPI   // (timing experiment only: the statistics' finish and the score skipped)
    finish_stats(T, cref, s1, s2, lane, reinterpret_cast<double*>(scr));
#endif
    EWK_TS(tq5);
    EWK_TADD(6, tq4, tq5);
}


// Ring mode (few segments per tick, latency matters): the workgroup's waves share one
// segment -- wave w takes tiles w, w + WAVES, ... -- and meet twice: for the segment's
// log-mel max (top_db threshold) and to combine their shifted sums.  Wave w's sums are
// shifted by its own first column (cref_w); wave 0 re-centres them on cref_0:
//   S1 = sum_w s1_w + n_w d_w,  S2 = sum_w s2_w + 2 d_w s1_w + n_w d_w^2,  d_w = cref_w - cref_0.
// Leaves mean / std (fp32-rounded) in misc0[0..19], misc0[20..39] (wave 0's scratch).
template <int RING>
__device__ void segment_stats_coop(const SegSrc<RING>& v, unsigned char* smem, float* scr, float* tile,
                                   float* spec, int wave, int lane, const int (&lo)[8], float* misc0,
                                   float& theta_out EWK_COOP_KEY_PARAM) {
    const float* s_dct = reinterpret_cast<const float*>(smem + L_DCT);
    float* wg_mm = reinterpret_cast<float*>(smem + L_WG + 16);   // [WAVES][2] max, min
    const int T = 1 + v.len / HOP;
    const int ntile = (T + 15) >> 4;
    const int nloc = ntile > wave ? (ntile - wave + WAVES - 1) / WAVES : 0;
    const int col = lane & 15;
    double s1[8], s2[8];
    float cref[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { s1[i] = 0.0; s2[i] = 0.0; cref[i] = 0.0f; }
    float vmax = -INFINITY, vmin = INFINITY, nanp = 0.0f;
    // the wave's last tile stays in LDS (unclamped) until the segment max is known, so a
    // segment of <= WAVES tiles (T <= 128) is never recomputed; earlier tiles are clamped
    // speculatively at the running max (segment_stats) and recomputed if theta bites
    float run = -INFINITY, last_min = INFINITY;
    for (int lt = 0; lt < nloc; ++lt) {
        const int tile_i = wave + WAVES * lt;
        const bool last = lt + 1 == nloc;
        const bool rec = !last && lt < kSpecTiles;
        if (!rec) run = -INFINITY;
        float tmin = INFINITY;
        tile_passes(v, tile_i, T, smem, scr, tile, lane, lo, vmax, tmin, nanp, run);
        const float tmw = wave_min(tmin);
        vmin = fminf(vmin, tmw);
#ifdef EWK_COOP_DEBUG
        if (last && dkey < 4 * 256) {
            lds_order();
#pragma unroll
            for (int u = 0; u < 8; ++u) g_coop_tile[dkey][wave][64 * u + lane] = reinterpret_cast<const uint4*>(tile)[64 * u + lane];
        }
#endif
        if (last) { last_min = tmw; break; }
        const float run2 = rec ? wave_max(vmax) - kTopDbUnits : -INFINITY;
        if (run2 > run && tmw < run2) {   // self-clamp (segment_stats)
            uint4 h[4], l[4];
            clamp_load(reinterpret_cast<const float4*>(tile), lane, h, l);
            clamp_store(tile, lane, h, l, run2);
            lds_order();
        }
        run = fmaxf(run, run2);
        float c[8];
        tile_dct(tile, s_dct, lane, c);
        if (lt == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cref[i] = __shfl(c[i], lane & 48, 64);
        }
        stats_add(c, cref, tile_i * 16 + col < T, s1, s2);
        if (lane == 0 && rec) {   // tile-granular records (both passes recomputed when theta bites)
#pragma unroll
            for (int p = 0; p < kPassesPerTile; ++p) spec[kPassesPerTile * lt + p] = fmaxf(tmw, run);
            spec[kSpecRun + lt] = run;
        }
    }
    vmax = wave_max(vmax);
    if (lane == 0) { wg_mm[2 * wave] = vmax; wg_mm[2 * wave + 1] = vmin; }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < WAVES; ++w) { vmax = fmaxf(vmax, wg_mm[2 * w]); vmin = fminf(vmin, wg_mm[2 * w + 1]); }
    const float theta = vmax - kTopDbUnits;
    theta_out = theta;
#ifdef EWK_COOP_DEBUG
    if (lane == 0) g_coop_th[dkey][wave] = make_float4(wg_mm[2 * wave], wg_mm[2 * wave + 1], theta, (float)nloc);
#endif
    if (nloc > 0) {
        const int tile_l = wave + WAVES * (nloc - 1);
        if (last_min < theta) {   // the last tile, still in LDS: clamp at the final threshold
            uint4 h[4], l[4];
            clamp_load(reinterpret_cast<const float4*>(tile), lane, h, l);
            clamp_store(tile, lane, h, l, theta);
            lds_order();
        }
        float c[8];
        tile_dct(tile, s_dct, lane, c);
        if (nloc == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cref[i] = __shfl(c[i], lane & 48, 64);
        }
        stats_add(c, cref, tile_l * 16 + col < T, s1, s2);
        if (vmin < theta) {
            lds_order();
            for (int lt = 0; lt + 1 < nloc; ++lt) {
                const bool rec = lt < kSpecTiles;
                if (rec && !(spec[kPassesPerTile * lt] < theta)) continue;
                fix_tile(v, wave + WAVES * lt, T, rec ? spec[kSpecRun + lt] : -INFINITY, theta, smem, scr, tile,
                         lane, lo, cref, s1, s2);
            }
        }
    }
    if (__ballot(nanp != nanp)) {   // NaN input (segment_stats): the combined sums go NaN
#pragma unroll
        for (int i = 0; i < 8; ++i) s1[i] = __builtin_nan("");
    }
    // this wave's per-coefficient (s1, s2, cref) -> its scratch, as doubles [coef][3]
    double* pd = reinterpret_cast<double*>(scr);
#pragma unroll
    for (int i = 0; i < 8; ++i) { s1[i] = row_sum_d(s1[i]); s2[i] = row_sum_d(s2[i]); }
    if (col == 15) {
        const int h = lane >> 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = 4 * h + r;
            pd[3 * k] = s1[r]; pd[3 * k + 1] = s2[r]; pd[3 * k + 2] = (double)cref[r];
            if (h == 0) {
                const int k2 = 16 + r;
                pd[3 * k2] = s1[4 + r]; pd[3 * k2 + 1] = s2[4 + r]; pd[3 * k2 + 2] = (double)cref[4 + r];
            }
        }
    }
    __syncthreads();
#ifdef EWK_COOP_DEBUG
    if (lane < 60) g_coop_pd[dkey][wave][lane] = pd[lane];
#endif
    if (wave == 0) {
        double mean = 0.0, sd = 0.0;
        if (lane < NMFCC) {
            const double* p0 = reinterpret_cast<const double*>(smem + L_SCR);
            const double r0 = p0[3 * lane + 2];
            double S1 = 0.0, S2 = 0.0;
            for (int w = 0; w < WAVES; ++w) {
                int n = 0;   // valid frames of wave w's tiles
                for (int ti = w; ti < ntile; ti += WAVES) n += min(16, T - 16 * ti);
                if (n == 0) continue;
                const double* pw = reinterpret_cast<const double*>(smem + L_SCR + w * SCR_BYTES);
                const double a1 = pw[3 * lane], a2 = pw[3 * lane + 1], d = pw[3 * lane + 2] - r0;
                S1 += a1 + (double)n * d;
                S2 += a2 + 2.0 * d * a1 + (double)n * d * d;
            }
            const double Td = (double)T;
            mean = r0 + S1 / Td;
            double var = (S2 - S1 * S1 / Td) / Td;
            sd = sqrt(var > 0.0 ? var : 0.0);
        }
        lds_order();
        if (lane < NMFCC) { misc0[lane] = (float)mean; misc0[20 + lane] = (float)sd; }
#ifdef EWK_COOP_DEBUG
        if (lane < NMFCC) { g_coop_ms[dkey][lane] = (float)mean; g_coop_ms[dkey][20 + lane] = (float)sd; }
#endif
        lds_order();
    }
}

// ---- the score, exactly as WordMatcher.calculate_similarity evaluates it --------
// (wakeword.py:611-625 with scipy 1.15 `correlation`: dist = clip(1 - uv/sqrt(uu*vv), 0, 2)).
// The template u is float32 (librosa.load -> float32 MFCCs).  numpy's dot of two
// float32 vectors is float(sum_double(float(a*b))) (cblas_sdot's scalar path for
// n = 20, verified bit for bit against np.dot); a float32 x float64 or float64 dot
// is a float64 dot.  Two candidate dtypes occur in the reference:
//   float64 (streaming: SoundBuffer slices, wakeword.py:428, 509-513): uu is a
//     float32 dot, uv / vv float64, the rest float64;
//   float32 (WordMatcher on float32 audio): every dot float32 and, under NumPy 2
//     scalar promotion, every following operation float32.
__device__ __forceinline__ float sdot20(const float* a, const float* b) {
#pragma clang fp contract(off)
    double acc = 0.0;
    for (int i = 0; i < NMFCC; ++i) acc += (double)(a[i] * b[i]);
    return (float)acc;
}

template <typename T>
__device__ __forceinline__ double ddot20(const float* a, const T* b) {
#pragma clang fp contract(off)
    double acc = 0.0;
    for (int i = 0; i < NMFCC; ++i) acc += (double)a[i] * (double)b[i];
    return acc;
}

template <typename T>
__device__ __forceinline__ double ddot20s(const T* a) {
#pragma clang fp contract(off)
    double acc = 0.0;
    for (int i = 0; i < NMFCC; ++i) acc += (double)a[i] * (double)a[i];
    return acc;
}

__device__ __forceinline__ double clip02(double d) {
    if (d < 0.0) return 0.0;
    if (d > 2.0) return 2.0;
    return d;   // NaN passes through (np.clip)
}

__device__ __forceinline__ float clip02f(float d) {
    if (d < 0.0f) return 0.0f;
    if (d > 2.0f) return 2.0f;
    return d;
}

// Candidate stats in float64 (the streaming dtype).
__device__ double score_f64cand(const float* tm, const float* ts, const double* cm, const double* cs) {
#pragma clang fp contract(off)
    const double uu_m = (double)sdot20(tm, tm), uu_s = (double)sdot20(ts, ts);
    const double sm = 1.0 - clip02(1.0 - ddot20(tm, cm) / sqrt(uu_m * ddot20s(cm)));
    const double ss = 1.0 - clip02(1.0 - ddot20(ts, cs) / sqrt(uu_s * ddot20s(cs)));
    const double combined = sm * 0.7 + ss * 0.3;
    const double percent = combined * 100.0;
    return pow(percent, 1.5) / 10.0;   // (100**0.5) == 10.0 exactly
}

// Candidate stats in float32 (WordMatcher on float32 audio): float32 arithmetic.
__device__ double score_f32cand(const float* tm, const float* ts, const float* cm, const float* cs) {
#pragma clang fp contract(off)
    float sim[2];
    for (int k = 0; k < 2; ++k) {
        const float* u = k ? ts : tm;
        const float* v = k ? cs : cm;
        const float uu = sdot20(u, u), vv = sdot20(v, v), uv = sdot20(u, v);
        const float prod = uu * vv;                       // float32 * float32
        const float root = (float)sqrt((double)prod);      // math.sqrt, back to float32 (NEP 50)
        const float dist = clip02f(1.0f - uv / root);
        sim[k] = 1.0f - dist;
    }
    const float combined = sim[0] * 0.7f + sim[1] * 0.3f;
    const float percent = combined * 100.0f;
    return (double)(powf(percent, 1.5f) / 10.0f);
}


// Fast-path finishes (the fp64 re-score keeps the reference's exact pow / sequential dots).
__device__ __forceinline__ double score_f64_finish(double uu_m, double uu_s, double uv_m, double vv_m, double uv_s,
                                                   double vv_s, double& percent) {
#pragma clang fp contract(off)
    const double sm = 1.0 - clip02(1.0 - uv_m / sqrt(uu_m * vv_m));
    const double ss = 1.0 - clip02(1.0 - uv_s / sqrt(uu_s * vv_s));
    percent = (sm * 0.7 + ss * 0.3) * 100.0;
    return percent * sqrt(percent) / 10.0;   // p**1.5 (NaN for p < 0 like pow)
}

__device__ __forceinline__ double score_f32_finish(float uu_m, float uu_s, float uv_m, float vv_m, float uv_s,
                                                   float vv_s) {
#pragma clang fp contract(off)
    const float dm = clip02f(1.0f - uv_m / (float)sqrt((double)(uu_m * vv_m)));
    const float ds = clip02f(1.0f - uv_s / (float)sqrt((double)(uu_s * vv_s)));
    const float combined = (1.0f - dm) * 0.7f + (1.0f - ds) * 0.3f;
    const float percent = combined * 100.0f;
    return (double)(powf(percent, 1.5f) / 10.0f);
}

#include "ewk_rescore.h"

// Score one segment from its fp32-rounded mean / std (lane k < 20: coefficient k; one wave):
// wave-parallel dots in a fixed butterfly order, lane 0 finishes the score, writes the
// decision and lists the segment for the fp64 re-score (ewk_rescore.h) when the float32
// pipeline cannot decide it alone.  theta_s: the float32 pass's log-mel max - 80 dB.
template <int RING>
__device__ __forceinline__ void score_epilogue(const ScoreArgs& a, float cmf, float csf, float tmf, float tsf,
                                               int lane, int seg, int len, float theta_s) {
    bool near = a.list_all;
    if (a.has_template) {
        double score, std2, mean2, percent = 0.0;
        if (a.cand_f32) {   // float32 candidates: float products, float-rounded dots (sdot)
            const float uv_m = (float)wave_sum_d((double)(tmf * cmf)), vv_m = (float)wave_sum_d((double)(cmf * cmf));
            const float uv_s = (float)wave_sum_d((double)(tsf * csf)), vv_s = (float)wave_sum_d((double)(csf * csf));
            score = score_f32_finish(a.uu_m32, a.uu_s32, uv_m, vv_m, uv_s, vv_s);
            std2 = vv_s;
            mean2 = vv_m;
        } else {
            const double uv_m = wave_sum_d((double)tmf * (double)cmf), vv_m = wave_sum_d((double)cmf * (double)cmf);
            const double uv_s = wave_sum_d((double)tsf * (double)csf), vv_s = wave_sum_d((double)csf * (double)csf);
            score = score_f64_finish((double)a.uu_m32, (double)a.uu_s32, uv_m, vv_m, uv_s, vv_s, percent);
            std2 = vv_s;
            mean2 = vv_m;
        }
        if (lane == 0) {
            const int match = score >= a.threshold;
            // fp64 re-score: decisions within the margin of the threshold; very short segments
            // (T <= kRescoreFrames) whose 2..16-frame std vectors are too ill-conditioned for the
            // float32 pipeline to meet 1e-4; nearly stationary segments (0 < |std| < kTinyStd:
            // steady noise, or a few bins above the -100 dB floor: std vectors of norm ~1e-2..20
            // whose direction the float32 rounding of the MFCCs (~3e-5 absolute) moves by up to
            // ~3e-4 in the score; scripts/fuzz_err.py over 12 x 200 fuzz segments found 1.3e-4 at
            // |std| = 8); and loud segments whose MFCC mean vector nearly vanishes (|mean| <
            // kTinyMean: c0's positive and negative frames cancel, the float32 log-mel error
            // becomes a direction error, up to 3.6e-4 in the score; DESIGN.md numerics).  An
            // exactly constant segment keeps its NaN (zero std; the reference's own value there
            // is a rounding artefact).
            // (float64 candidates only: a vanishing-mean segment that is NaN beyond the float32 error)
            const bool sure_nan = !a.cand_f32 && percent < -(kNanMarginA / sqrt(mean2) + kNanMarginB);
            near = near || fabs(score - a.threshold) < a.rescore_margin || (1 + len / HOP) <= kRescoreFrames ||
                   (std2 > 0.0 && std2 < kTinyStd * kTinyStd) || (mean2 < kTinyMean * kTinyMean && !sure_nan);
#ifdef EWK_LIST_STATS
            if (near) {
                const unsigned long long T = 1 + len / HOP;
                const bool why[4] = {fabs(score - a.threshold) < a.rescore_margin, (int)T <= kRescoreFrames,
                                     std2 > 0.0 && std2 < kTinyStd * kTinyStd, mean2 < kTinyMean * kTinyMean && !sure_nan};
                atomicAdd(&g_ewk_list[0], 1ull);
                atomicAdd(&g_ewk_list[5], T);
                for (int k = 0; k < 4; ++k)
                    if (why[k]) { atomicAdd(&g_ewk_list[1 + k], 1ull); atomicAdd(&g_ewk_list[6 + k], T); }
            }
#endif
            if (RING) {
                a.events[seg].score = score;
                a.events[seg].match = match;
            } else {
                a.out_score[seg] = score;
                if (a.out_match) a.out_match[seg] = (uint8_t)match;
            }
        }
    }
    if (lane == 0 && near && a.rs_slots) rs_list(a, seg, len, theta_s);   // drained by the re-score launch
}


// MODE 0: linear batch; 1: ring events, one segment per workgroup (cooperative); 2: ring
// events, one segment per wave from the work counter.  S16: int16 rings (EWK_RING_I16).
template <int MODE, int S16>
__global__ __launch_bounds__(64 * WAVES, 1) void k_score_f32(const Tables* __restrict__ tab, ScoreArgs a) {
    constexpr int RING = MODE == 0 ? 0 : (S16 ? 2 : 1);
    const void* ring_base = S16 ? (const void*)a.pcm16 : (const void*)a.pcm;   // ring modes
    constexpr float kWinScale = S16 ? 1.0f / 32768.0f : 1.0f;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // ring mode: the event window and this workgroup's first event, requested before the
    // table fill so their latency overlaps it
    int r_base = 0, r_count = 0;
    ewk_event r_ev = {};
    if (RING) {
        // counters in wrapping count space; slots relative to the bank's epoch base (a watermark
        // left behind an epoch -- no template while its events arrived -- restarts at slot 0)
        r_base = max(0, (int)((uint32_t)*a.ev_base - (uint32_t)a.ev_base0));
        r_count = min((int)((uint32_t)*a.n_events - (uint32_t)a.ev_base0), a.n_seg) - r_base;
        if ((int)blockIdx.x < r_count) r_ev = a.events[r_base + blockIdx.x];
        // one segment per workgroup: a workgroup without one skips the table fill (most of
        // a quiet tick's 256 workgroups)
        if (MODE == 1 && (int)blockIdx.x >= r_count) return;   // (k_rescore_ring ends the tick)
    }
    // ---- cooperative table load (global -> LDS), per-lane rows transposed
    {
        float2* sw2 = reinterpret_cast<float2*>(smem + L_WIN2);
        float2* st1 = reinterpret_cast<float2*>(smem + L_TW1);
        float2* st2 = reinterpret_cast<float2*>(smem + L_TW2);
        for (int i = threadIdx.x; i < 256; i += blockDim.x) {
            const int j = i & 15, n = i >> 4;   // win2[16n + j], tw1[16n + j], tw2[j + 16n]
            sw2[j * TP + n] = make_float2(tab->win2[i].x * kWinScale, tab->win2[i].y * kWinScale);
            if (n > 0) st1[j * TP + n - 1] = tab->tw1[i];
        }
        // [j'][it] = (cos, tan) of tw2[k] for the bin k that lane class j' untangles at step it
        for (int i = threadIdx.x; i < 8 * 17; i += blockDim.x) {
            const int jp = i / 17, it = i % 17;
            const int k = jp ? jp + 16 * (it < 16 ? it : 15) : (it <= 8 ? 16 * it : 8 + 16 * (it - 9));
            const float2 cs = tab->tw2[k];   // (c, t): c = cos is never 0 in float (k = 128: 6.1e-17)
            st2[jp * TP + it] = make_float2(cs.x, cs.y / cs.x);
        }
        int* sb = reinterpret_cast<int*>(smem + L_BLO);
        for (int i = threadIdx.x; i < NMEL; i += blockDim.x) sb[i] = tab->band_lo[i];
        float* sw = reinterpret_cast<float*>(smem + L_WPAD);
        for (int i = threadIdx.x; i < 16 * WP; i += blockDim.x) {
            const int j = i / WP, o = i % WP;
            float w = 0.0f;
#pragma unroll
            for (int g = 0; g < 8; ++g)
                if (o >= kMelOff[g] && o < kMelOff[g] + kMelW[g]) w = tab->wpad[(kMelIt0[g] + o - kMelOff[g]) * 16 + j];
            sw[i] = w;
        }
        // the f16 hi/lo DCT operand chunks (kDctScale keeps the lo parts normal)
        uint4* sd = reinterpret_cast<uint4*>(smem + L_DCT);
        for (int i = threadIdx.x; i < DCT_BYTES / 16; i += blockDim.x) {
            int row = -1, c = 0, hl = 0;
            if (i < DCT_RT1 / 16) {
                const int l = i & 63;
                hl = (i >> 6) & 1;
                row = l & 15;
                c = 4 * (i >> 7) + (l >> 4);
            } else {
                const int k = i - DCT_RT1 / 16, blk = k / 17, slot = k % 17;   // blk = q * 2 + hl
                if (slot < 16) {
                    row = 16 + (slot & 3);
                    c = 4 * (blk >> 1) + (slot >> 2);
                    hl = blk & 1;
                }
            }
            float v[8];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const float d = row >= 0 ? tab->dct[row * NMEL + c + 16 * jj] * kDctScale : 0.0f;
                const float h = f16_trunc(d);
                v[jj] = hl ? d - h : h;
            }
            sd[i] = make_uint4(pk_f16(v[0], v[1]), pk_f16(v[2], v[3]), pk_f16(v[4], v[5]), pk_f16(v[6], v[7]));
        }
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int base = 0, count = a.n_seg;
    if (RING) {
        base = r_base;
        count = r_count;
    }
    unsigned char* wbase = smem + L_SHARED_END + wave * W_BYTES;
    float* scr = reinterpret_cast<float*>(smem + L_SCR + wave * SCR_BYTES);
    float* tile = reinterpret_cast<float*>(wbase + W_TILE);
    float* spec = reinterpret_cast<float*>(wbase + W_SPEC);
    int lo[8];   // first bin of this lane's bands j + 16 i
    {
        const int* sb = reinterpret_cast<const int*>(smem + L_BLO);
#pragma unroll
        for (int i = 0; i < 8; ++i) lo[i] = sb[(lane & 15) + 16 * i];
    }
    // persistent waves pull segments from a work counter (ragged lengths balance)
    // the template is loop-invariant: fetched once, off every segment's critical path.
    // (Reserving the next work item ahead was tried: the tail imbalance costs more.)
    const bool act = lane < NMFCC;
    const float tmf = (a.has_template && act) ? a.tmpl[lane] : 0.0f;
    const float tsf = (a.has_template && act) ? a.tmpl[NMFCC + lane] : 0.0f;
    // Ring mode, MODE 1 (a tick of ~10^3-10^4 streams: a few hundred segments, latency
    // bound): one segment per workgroup at a time, its tiles spread over the waves.  MODE 2
    // (10^5-10^6 streams: enough events to keep every wave busy) falls through: the waves
    // take whole segments from the work counter, like a linear batch.
    if (MODE == 1) {
        int* wg_idx = reinterpret_cast<int*>(smem + L_WG);
        float* misc0 = reinterpret_cast<float*>(smem + L_SCR);   // wave 0's FFT scratch (epilogue only)
        // first segment by workgroup index (its event was requested before the table fill),
        // later ones from the work counter (a burst tick's segments balance over the grid)
        for (int idx = blockIdx.x; idx < count;) {
            __syncthreads();   // wave 0's scratch (misc0) and wg_idx are free again
            // the next index is reserved now, its atomic's latency hidden under this segment
            int nxt = 0;
            if (threadIdx.x == 0) nxt = (int)gridDim.x + atomicAdd(a.work, 1);
            const int seg = base + idx;
            const ewk_event ev = idx == (int)blockIdx.x ? r_ev : a.events[seg];
            if (!(ev.flags & EWK_EV_SKIPPED)) {
                const SegSrc<RING> v = make_src<RING>(
                    static_cast<const unsigned char*>(ring_base) + (int64_t)ev.stream * a.ring_len * sample_bytes(RING),
                    ev.ring_start, a.ring_len, ev.length);
                float theta_s;
#ifdef EWK_COOP_DEBUG
                const int dkey = (ev.stream & 31) * 256 + (int)(ev.tick & 255);
                if (lane == 0) g_coop_ev[dkey][wave] = make_int4(ev.stream, (int)ev.ring_start, ev.length, (int)ev.tick);
#endif
                segment_stats_coop(v, smem, scr, tile, spec, wave, lane, lo, misc0, theta_s EWK_COOP_KEY_ARG(dkey));
                if (wave == 0 && (a.has_template || a.list_all))
                    score_epilogue<RING>(a, act ? misc0[lane] : 0.0f, act ? misc0[20 + lane] : 0.0f, tmf, tsf, lane,
                                         seg, v.len, theta_s);
            }
            if (threadIdx.x == 0) wg_idx[0] = nxt;
            __syncthreads();
            idx = wg_idx[0];
        }
        return;   // k_rescore_ring drains the re-score list and ends the tick
    }
#ifdef EWK_TIMING
    uint64_t dbg[kDbgN] = {};
#endif
    const WorkCtx wc = {&a, base, count, true, (int)blockIdx.x * WAVES + wave, (int)gridDim.x * WAVES};
    WorkAhead nx;
    for (;;) {
        EWK_TS(tw0);
        if (nx.state != 3) {   // nothing claimed ahead (first segment, or after a skipped event)
            work_claim<RING>(wc, nx, lane);
            work_order<RING>(wc, nx);
            work_describe<RING>(wc, nx);
        }
        nx.state = 0;
        if (nx.idx >= count) break;
        const int seg = nx.seg;
        int64_t ring = 0;
        const void* p;
        if (RING) {
            if (nx.flags & EWK_EV_SKIPPED) continue;
            p = static_cast<const unsigned char*>(ring_base) + (int64_t)nx.stream * a.ring_len * sample_bytes(RING);
            ring = a.ring_len;
        } else {
            p = a.pcm;
        }
        const SegSrc<RING> v = make_src<RING>(p, nx.start, ring, nx.len);
        EWK_TS(tw1);
        EWK_TADD(0, tw0, tw1);

        double st1[8], st2[8];
        float theta_s;
        segment_stats(v, smem, scr, tile, spec, lane, lo, st1, st2, theta_s, wc, nx EWK_DBG_ARG);
        EWK_TS(tw2);

        // ---- lane k < 20 holds coefficient k's mean / std (fp32-rounded like the reference's)
        const float cmf = act ? (float)st1[0] : 0.0f, csf = act ? (float)st2[0] : 0.0f;
        if (act && !RING) {
            if (a.out_mean) a.out_mean[(int64_t)seg * NMFCC + lane] = cmf;
            if (a.out_std) a.out_std[(int64_t)seg * NMFCC + lane] = csf;
        }
#ifndef EWK_SKIP_EPI
        if (a.has_template || a.list_all) score_epilogue<RING>(a, cmf, csf, tmf, tsf, lane, seg, v.len, theta_s);
#else
        if (lane == 0 && !RING) a.out_score[seg] = cmf + csf;
#endif
        lds_order();
        EWK_TS(tw3);
        EWK_TADD(7, tw2, tw3);
#ifdef EWK_TIMING
        dbg[9] += 1;
#endif
    }   // work loop
#ifdef EWK_TIMING
    dbg[8] += 1;
    if (lane == 0)
        for (int k = 0; k < kDbgN; ++k) atomicAdd(&g_ewk_dbg[k], (unsigned long long)dbg[k]);
#endif
    // (the fp64 list is drained by k_rescore_linear / k_rescore_ring, launched after this kernel)
}

#ifdef EWK_RS_TIMING
}  // namespace ewk
extern "C" int ewk_debug_rs(unsigned long long* out) {   // read and reset (debug builds only)
    unsigned long long z[16] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ewk::g_rs_dbg), sizeof(z)) != hipSuccess) return -3;
    if (hipMemcpyToSymbol(HIP_SYMBOL(ewk::g_rs_dbg), z, sizeof(z)) != hipSuccess) return -3;
    return 0;
}
extern "C" int ewk_debug_rs_ph(unsigned long long* out) {   // chunk sub-phase cycles (debug builds only)
    unsigned long long z[8] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ewk::g_rs_ph), sizeof(z)) != hipSuccess) return -3;
    if (hipMemcpyToSymbol(HIP_SYMBOL(ewk::g_rs_ph), z, sizeof(z)) != hipSuccess) return -3;
    return 0;
}
namespace ewk {
#endif

#ifdef EWK_COOP_DEBUG
}  // namespace ewk
extern "C" int ewk_debug_coop(void* ev, void* th, void* pd, void* ms) {   // debug builds only
    if (hipMemcpyFromSymbol(ev, HIP_SYMBOL(ewk::g_coop_ev), sizeof(ewk::g_coop_ev)) != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(th, HIP_SYMBOL(ewk::g_coop_th), sizeof(ewk::g_coop_th)) != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(pd, HIP_SYMBOL(ewk::g_coop_pd), sizeof(ewk::g_coop_pd)) != hipSuccess) return -3;
    if (hipMemcpyFromSymbol(ms, HIP_SYMBOL(ewk::g_coop_ms), sizeof(ewk::g_coop_ms)) != hipSuccess) return -3;
    return 0;
}
extern "C" int ewk_debug_coop_tile(int key, void* out) {   // one key's [WAVES][512] uint4 (debug builds only)
    if (key < 0 || key >= 4 * 256) return -1;
    const size_t one = sizeof(ewk::g_coop_tile[0]);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ewk::g_coop_tile), one, (size_t)key * one) != hipSuccess) return -3;
    return 0;
}
namespace ewk {
#endif

#ifdef EWK_LIST_STATS
}  // namespace ewk
extern "C" int ewk_debug_list(unsigned long long* out) {   // read and reset (debug builds only)
    unsigned long long z[10] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ewk::g_ewk_list), sizeof(z)) != hipSuccess) return -3;
    if (hipMemcpyToSymbol(HIP_SYMBOL(ewk::g_ewk_list), z, sizeof(z)) != hipSuccess) return -3;
    return 0;
}
namespace ewk {
#endif

#ifdef EWK_TIMING
}  // namespace ewk
extern "C" int ewk_debug_timing(unsigned long long* out) {   // read and reset (debug builds only)
    unsigned long long z[kDbgN] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ewk::g_ewk_dbg), sizeof(z)) != hipSuccess) return -3;
    if (hipMemcpyToSymbol(HIP_SYMBOL(ewk::g_ewk_dbg), z, sizeof(z)) != hipSuccess) return -3;
    return 0;
}
namespace ewk {
#endif

// Event-count snapshot taken on the gate's stream right after a gate launch: the
// scoring pass that overlaps the next gate scores exactly the events of its own tick.
__global__ void k_snapshot(const int32_t* src, int32_t* dst) { *dst = *src; }

hipError_t launch_snapshot(const int32_t* src, int32_t* dst, hipStream_t s) {
    hipLaunchKernelGGL(k_snapshot, dim3(1), dim3(1), 0, s, src, dst);
    return hipGetLastError();
}

// Poll mirror of an event bank: its four counters and its first min(queued, chunk) events,
// written straight into pinned host memory after the push's last scoring pass (stream-
// ordered, so every score is final).  The host polls it after one event wait instead of
// two D2H copies on a second stream (blit kernels that queue for CU slots behind the next
// gate) and a stream synchronisation.  host: [16 B counters][chunk events], 16-B aligned.
__global__ __launch_bounds__(256) void k_bank_mirror(const int32_t* __restrict__ evc, const ewk_event* __restrict__ ev,
                                                     uint32_t base0, int32_t cap, int32_t chunk,
                                                     unsigned char* __restrict__ host) {
    const uint4 c = *reinterpret_cast<const uint4*>(evc);
    const int32_t n = (int32_t)min(min((uint32_t)(c.x - base0), (uint32_t)cap), (uint32_t)chunk);
    if (threadIdx.x == 0) *reinterpret_cast<uint4*>(host) = c;
    static_assert(sizeof(ewk_event) % 16 == 0, "events copied in 16-B pieces");
    const uint4* src = reinterpret_cast<const uint4*>(ev);
    uint4* dst = reinterpret_cast<uint4*>(host + 16);
    const int nq = n * (int)(sizeof(ewk_event) / 16);
    for (int i = threadIdx.x; i < nq; i += blockDim.x) dst[i] = src[i];
}

hipError_t launch_bank_mirror(const int32_t* evc, const ewk_event* ev, uint32_t base0, int32_t cap, int32_t chunk,
                              unsigned char* host, hipStream_t s) {
    hipLaunchKernelGGL(k_bank_mirror, dim3(1), dim3(256), 0, s, evc, ev, base0, cap, chunk, host);
    return hipGetLastError();
}

// Longest-first work order for a linear batch (LPT: the persistent waves' last
// segments are the shortest, so the grid drains evenly): 64 buckets of the segment's pass
// count, longest first; the order within a bucket is arbitrary (each segment's result
// does not depend on it).
constexpr int kLptBuckets = 64;
__device__ __forceinline__ int lpt_bucket(int32_t len) {   // longest first: bucket 0 = most passes
    const int np = (1 + max(len, 0) / HOP + kFPP - 1) / kFPP;
    return kLptBuckets - 1 - min(np, kLptBuckets - 1);
}

// Grid-parallel LPT order: pass 1 adds each workgroup's bucket histogram of its slice to
// the global totals; pass 2 (every workgroup redoes the 64-bucket exclusive scan) reserves a
// contiguous run per bucket with one atomic on that bucket's cursor and scatters its
// indices.  cnt = order + n: [0, 64) totals, [64, 128) cursors (zeroed before pass 1).
constexpr int kLptBlock = 256;
__global__ __launch_bounds__(kLptBlock) void k_lpt_hist(const int32_t* __restrict__ lengths, int32_t n,
                                                        int32_t* __restrict__ cnt) {
    __shared__ int h[kLptBuckets];
    if (threadIdx.x < kLptBuckets) h[threadIdx.x] = 0;
    __syncthreads();
    for (int i = blockIdx.x * kLptBlock + threadIdx.x; i < n; i += gridDim.x * kLptBlock)
        atomicAdd(&h[lpt_bucket(lengths[i])], 1);
    __syncthreads();
    if (threadIdx.x < kLptBuckets && h[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(kLptBlock) void k_lpt_scatter(const int32_t* __restrict__ lengths, int32_t n,
                                                           int32_t* __restrict__ order, int32_t* __restrict__ cnt,
                                                           int32_t* __restrict__ work, int32_t* __restrict__ rs_ctl) {
    __shared__ int h[kLptBuckets], base[kLptBuckets];
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // the scorer's counters (no fill launches)
        *work = 0;
        for (int i = 0; i < kRsCtl; ++i) rs_ctl[i] = 0;
    }
    if (threadIdx.x < kLptBuckets) h[threadIdx.x] = 0;
    __syncthreads();
    for (int i = blockIdx.x * kLptBlock + threadIdx.x; i < n; i += gridDim.x * kLptBlock)
        atomicAdd(&h[lpt_bucket(lengths[i])], 1);
    __syncthreads();
    if (threadIdx.x < kLptBuckets) {   // one wave: lane = bucket
        const int b = threadIdx.x, tot = cnt[b];
        int incl = tot;
        for (int d = 1; d < kLptBuckets; d <<= 1) {
            const int t = __shfl_up(incl, d, 64);
            if (b >= d) incl += t;
        }
        base[b] = (incl - tot) + (h[b] ? atomicAdd(&cnt[kLptBuckets + b], h[b]) : 0);
        h[b] = 0;
    }
    __syncthreads();
    for (int i = blockIdx.x * kLptBlock + threadIdx.x; i < n; i += gridDim.x * kLptBlock) {
        const int b = lpt_bucket(lengths[i]);
        order[base[b] + atomicAdd(&h[b], 1)] = i;
    }
}

int score_grid(int n_seg, int ring_mode) {
    return ring_mode ? kScoreGridRing : max(1, min((n_seg + WAVES - 1) / WAVES, kScoreGridMax));
}

hipError_t launch_score_f32(const Tables* d_tab, const ScoreArgs& a, int ring_mode, hipStream_t s) {
    if (a.n_seg <= 0) return hipSuccess;
    const int grid = score_grid(a.n_seg, ring_mode);
    if (ring_mode) {   // ring mode: the last workgroup out re-arms the counters after each tick
        if (ring_mode == 2 && a.pcm16) hipLaunchKernelGGL((k_score_f32<2, 1>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, s, d_tab, a);
        else if (ring_mode == 2) hipLaunchKernelGGL((k_score_f32<2, 0>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, s, d_tab, a);
        else if (a.pcm16) hipLaunchKernelGGL((k_score_f32<1, 1>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, s, d_tab, a);
        else hipLaunchKernelGGL((k_score_f32<1, 0>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, s, d_tab, a);
    } else {
        ScoreArgs b = a;
        // the order only matters once the waves queue several segments each
        if (a.order && a.n_seg > 2 * grid * WAVES) {
            int32_t* cnt = a.order + a.n_seg;
            hipError_t e = hipMemsetAsync(cnt, 0, 2 * kLptBuckets * sizeof(int32_t), s);
            if (e != hipSuccess) return e;
            const int g = std::min(256, (a.n_seg + kLptBlock - 1) / kLptBlock);
            hipLaunchKernelGGL(k_lpt_hist, dim3(g), dim3(kLptBlock), 0, s, a.lengths, a.n_seg, cnt);
            hipLaunchKernelGGL(k_lpt_scatter, dim3(g), dim3(kLptBlock), 0, s, a.lengths, a.n_seg, a.order, cnt, a.work,
                               a.rs_ctl);
        } else {
            b.order = nullptr;
            hipError_t e = hipMemsetAsync(a.work, 0, sizeof(int32_t), s);
            if (e == hipSuccess) e = hipMemsetAsync(a.rs_ctl, 0, kRsCtl * sizeof(int32_t), s);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((k_score_f32<0, 0>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, s, d_tab, b);
    }
    return hipGetLastError();
}

hipError_t launch_rescore_linear(const ScoreArgs& a, hipStream_t s) {
    if (a.n_seg <= 0 || !a.rs_slots) return hipSuccess;
    hipLaunchKernelGGL(k_rescore_linear, dim3(kScoreGridMax), dim3(64 * RS_NW), RS_LDS, s, a);
    return hipGetLastError();
}

// After every ring-mode scorer launch (also without a template: the tick end re-arms the
// counters and advances the watermark).
hipError_t launch_rescore_ring(const ScoreArgs& a, hipStream_t s) {
    if (a.n_seg <= 0) return hipSuccess;
    if (a.pcm16) hipLaunchKernelGGL(k_rescore_ring<2>, dim3(kScoreGridRing), dim3(64 * RS_NW), RS_LDS, s, a);
    else hipLaunchKernelGGL(k_rescore_ring<1>, dim3(kScoreGridRing), dim3(64 * RS_NW), RS_LDS, s, a);
    return hipGetLastError();
}

}  // namespace ewk

