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
//   pass    : 16 frames per wave = one log-mel tile, four lanes per frame (ewk_fp4.h):
//             the tile's 2,912 samples staged in LDS by LDS-DMA one pass ahead, an in-register
//             FFT whose cross-lane steps are v_permlane16/32_swap row exchanges, the untangle
//             in-lane, mel partial sums reduced over the frame's four lanes, log.
//   DCT     : the only dense GEMM on the path: C[32 x 16] = D[32 x 128] . X[128 x 16]
//             per tile on the matrix cores, v_mfma_f32_16x16x32_f16 on f16 hi/lo splits
//             (Dh Xh + Dh Xl + Dl Xh, f32 accumulation), operands B straight from the pass's
//             registers, rows 20..31 zero.
//   top_db  : power_to_db clamps at (segment max - 80 dB), a segment-global coupling.
//             Tiles are processed loudest first (a scout) and each is clamped at the
//             running max - 80 dB (exact once the max is known); at the end only the tiles
//             whose stored minimum is below the final max - 80 dB are recomputed and their
//             contribution swapped in the statistics (nothing is written to global memory
//             but the results).
//   stats   : population mean/std over frames from fp64 shifted sums
//             (d = c - c[frame 0]) -- exact 0 std for identical frames.
//   score   : the reference's own float32 / float64 cosine arithmetic
//             (wakeword.py:611-625 + scipy correlation); NaN kept.  Near-threshold
//             scores are re-scored by the fp64 path (ewk_rescore.h).
#include <hip/hip_runtime.h>
#include <math.h>

#include "ewk_fp4.h"
#include "ewk_internal.h"

// Per-wave phase timing of the linear-batch scorer (debug builds with -DEWK_TIMING only:
// scripts/mb_score.py prints it; the product build compiles none of it).  dbg[k] sums the
// s_memtime cycles of phase k over the wave's segments; the kernel adds them to g_ewk_dbg.
#ifdef EWK_TIMING
#define EWK_DBG_PARAM , uint64_t(&dbg)[kDbgN]
#define EWK_DBG_ARG , dbg
#define EWK_TS(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define EWK_TADD(k, a, b) dbg[k] += (b) - (a)
#else
#define EWK_DBG_PARAM
#define EWK_DBG_ARG
#define EWK_TS(v)
#define EWK_TADD(k, a, b)
#endif
#ifdef EWK_TIMING
constexpr int kDbgN = 20;
#endif

namespace ewk {

#ifdef EWK_TIMING
__device__ unsigned long long g_ewk_dbg[kDbgN];
#endif

typedef float floatx4 __attribute__((ext_vector_type(4)));

// LDS carve (bytes, every offset a multiple of 16): the pass tables (ewk_fp4.h), then per
// wave: the staged samples of one pass (filled by LDS-DMA), a 480-B scratch for the
// statistics (finish_stats, the cooperative ring mode's sums) and the top_db records.
constexpr int kFPP = fp4::FPP;                             // frames per pass = per tile
constexpr int L_TAB = 0;
constexpr int L_WAVES = fp4::TABLE_BYTES;
constexpr int W_STAGE = 0;
constexpr int W_PD = W_STAGE + fp4::STAGE_BYTES;            // 20 x 3 doubles
// per-tile record of the speculative top_db clamp (segment_stats): the stored log-mel minimum,
// the clamp and the processing order (3 x kSpecTiles ints)
constexpr int kSpecTiles = 64;   // tiles of frames 0..1023 (10.2 s) are recorded and scout-ordered
constexpr int W_SPEC = W_PD + 480;
constexpr int kSpecRun = kSpecTiles;                       // spec[kSpecRun + tile]: the tile's clamp
constexpr int kSpecOrder = kSpecRun + kSpecTiles;          // spec[kSpecOrder + k]: k-th tile processed
constexpr int W_BYTES = W_SPEC + (kSpecOrder + kSpecTiles) * 4;
constexpr int L_WG = L_WAVES + WAVES * W_BYTES;            // ring mode: segment index + per-wave log-mel max/min
constexpr int LDS_BYTES = L_WG + 16 + 8 * WAVES;
constexpr int kRescoreFrames = 16;
constexpr double kTinyMean = 64.0;  // |mean vector| below which the fp64 path decides
                                    // (loud audio, c0 cancelling: DESIGN.md numerics)
constexpr double kTinyStd = 20.0;   // |std vector| below which the fp64 path decides (bench batch >= 24.8,
                                    // streaming events >= 32.5: scripts/std_norm_dist.py)
constexpr float kTopDbUnits = 80.0f;   // top_db, in the tile's dB units
static_assert(LDS_BYTES <= 160 * 1024, "the workgroup must fit a CU's LDS");
static_assert(W_BYTES % 16 == 0 && fp4::TABLE_BYTES % 16 == 0, "LDS carve alignment");
static_assert(kSpecTiles <= 64, "the scout ranks one tile per lane");

__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

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

// Stage tile `tile` (frames 16 tile .. 16 tile + 15, samples 2,560 tile - 256 ..) into the
// wave's span: LDS-DMA for float32 sources (no VGPRs, lands while the current pass computes),
// registers for int16 rings.
template <int RING>
__device__ __forceinline__ void stage_tile(const SegSrc<RING>& v, int tile, float* stage, int lane) {
    const int S0 = tile * kFPP * HOP - NFFT / 2;
    if (RING == 0) fp4::stage_dma_linear(v.rsrc, S0, stage, lane);
    else if (RING == 1) fp4::stage_dma_ring(v.rsrc, S0, v.len, v.wrap_at, v.start, stage, lane);
    else fp4::stage_i16_ring(v.rsrc, S0, v.len, v.wrap_at, v.start, stage, lane);
}
// the staged samples have landed (LDS-DMA counts in vmcnt; the int16 path's stores are
// ordered before the pass's reads by the wave's in-order LDS queue)
__device__ __forceinline__ void stage_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

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
};

template <int RING>
__device__ __forceinline__ void work_claim(const WorkCtx& c, WorkAhead& w, int lane) {
    if (lane == 0) w.idx = atomicAdd(c.a->work, 1);
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

// The tile of one segment that pass 1 left holding a value below the final max - 80 dB is
// recomputed (the same pass, bit-identical values): the DCT of its values clamped at its
// speculative `run` gives the pass-1 columns to remove, clamped at theta the columns to add.
// (Rounds 1-4 measured the alternatives: parking every tile in global memory, parking only
// the tiles the scout ranks close to a later one, exact fix-ups of self-clamped tiles, a
// full-coverage scout -- each cost more than the recomputes it saved)
template <int RING>
__device__ __forceinline__ void fix_tile(const SegSrc<RING>& v, int tile_i, int T, float run, float theta,
                                         const unsigned char* tabs, float* stage, int lane, const float (&cref)[8],
                                         double (&s1)[8], double (&s2)[8]) {
    stage_tile(v, tile_i, stage, lane);
    stage_wait();
    float lm[32], d0 = -INFINITY, d1 = INFINITY, d2 = 0.0f;
    fp4::pass(tabs, stage, lane, true, lm, d0, d1, d2, [] {});
    float co[8], cn[8];
    fp4::dct(lm, run, tabs, lane, co);
    fp4::dct(lm, theta, tabs, lane, cn);
    stats_replace(cn, co, cref, tile_i * kFPP + (lane & 15) < T, s1, s2);
}

// Whole segment for one wave.  spec: this wave's per-tile record in LDS -- the stored
// log-mel minimum of tile i in spec[i], its speculative clamp in spec[kSpecRun + i] (tiles
// past kSpecTiles are stored unclamped and always recomputed when theta bites), then the
// processing order (spec[kSpecOrder + k]).
//
// The top_db clamp (max - 80 dB over the whole segment) is applied speculatively at the
// running max, which each tile updates before its DCT; a tile that already holds the
// segment max needs no fix, so the tiles are processed loudest first by a scout estimate
// (bench batch: 16 % of the tiles recomputed in time order, ~5 % in scout order).  Each
// tile's samples are staged by LDS-DMA while the previous tile computes.
template <int RING>
__device__ void segment_stats(const SegSrc<RING>& v, const unsigned char* tabs, float* stage, float* spec, double* pd,
                              int lane, double (&s1)[8], double (&s2)[8], float& theta_out, const WorkCtx& wc,
                              WorkAhead& nx EWK_DBG_PARAM) {
    EWK_TS(tq0);
    const int T = 1 + v.len / HOP;
    const int ntile = (T + kFPP - 1) / kFPP;
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
    stage_tile(v, tile_i, stage, lane);
    float run = -INFINITY;   // speculative clamp: running max - 80 dB
    for (int k = 0; k < ntile; ++k) {
        EWK_TS(tk0);
        const int next_tile = k + 1 < ntile ? (ordered ? order[k + 1] : k + 1) : -1;
        const bool rec = tile_i < kSpecTiles;
        if (!rec) run = -INFINITY;
        const bool last = k + 1 == ntile;
        if (last && wc.ahead) work_claim<RING>(wc, nx, lane);
        stage_wait();
        float lm[32], tp = INFINITY;
#ifdef EWK_FP4_SYNC   // debug: synchronous staging, no prefetch
        fp4::pass(tabs, stage, lane, tile_i * kFPP + col < T, lm, vmax, tp, nanp, [] {});
        if (next_tile >= 0) stage_tile(v, next_tile, stage, lane);
#else
        fp4::pass(tabs, stage, lane, tile_i * kFPP + col < T, lm, vmax, tp, nanp, [&] {
            if (next_tile >= 0) stage_tile(v, next_tile, stage, lane);
        });
#endif
        const float tmw = wave_min(tp);   // this tile's minimum (its record below)
        EWK_TS(tk1);
        EWK_TADD(3, tk0, tk1);
        if (last && wc.ahead) work_order<RING>(wc, nx);
        // max(max(x, run), final) = max(x, final): a tile stored clamped at the running max
        // (this tile's own values included) is exact unless a later tile raises the max
        const float run2 = rec ? wave_max(vmax) - kTopDbUnits : -INFINITY;
        run = fmaxf(run, run2);
        float c[8];
        fp4::dct(lm, run, tabs, lane, c);
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cref[i] = __shfl(c[i], lane & 48, 64);
        }
        stats_add(c, cref, tile_i * kFPP + col < T, s1, s2);
        vmin = fminf(vmin, tmw);
        if (lane == 0 && rec) {   // stored minimum: the tile's minimum as clamped at its run
            spec[tile_i] = fmaxf(tmw, run);
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
            if (rec && !(spec[cur] < theta)) continue;   // no stored value below theta
#ifdef EWK_TIMING
            dbg[10] += 1;
#endif
            fix_tile(v, cur, T, rec ? spec[kSpecRun + cur] : -INFINITY, theta, tabs, stage, lane, cref, s1, s2);
        }
    }
    if (__ballot(nanp != nanp)) {   // NaN input: NaN statistics, NaN score (like the reference)
#pragma unroll
        for (int i = 0; i < 8; ++i) s1[i] = __builtin_nan("");
    }
    EWK_TS(tq4);
    EWK_TADD(5, tq3, tq4);
    finish_stats(T, cref, s1, s2, lane, pd);
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
__device__ void segment_stats_coop(const SegSrc<RING>& v, unsigned char* smem, float* stage, float* spec, double* pd,
                                   int wave, int lane, float* misc0, float& theta_out) {
    const unsigned char* tabs = smem + L_TAB;
    float* wg_mm = reinterpret_cast<float*>(smem + L_WG + 16);   // [WAVES][2] max, min
    const int T = 1 + v.len / HOP;
    const int ntile = (T + kFPP - 1) / kFPP;
    const int nloc = ntile > wave ? (ntile - wave + WAVES - 1) / WAVES : 0;
    const int col = lane & 15;
    double s1[8], s2[8];
    float cref[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { s1[i] = 0.0; s2[i] = 0.0; cref[i] = 0.0f; }
    float vmax = -INFINITY, vmin = INFINITY, nanp = 0.0f;
    // the wave's last tile stays in registers (unclamped) until the segment max is known, so
    // a segment of <= WAVES tiles (T <= 128) is never recomputed; earlier tiles are clamped
    // speculatively at the running max (segment_stats) and recomputed if theta bites
    float run = -INFINITY, last_min = INFINITY;
    float lm[32];
    if (nloc > 0) stage_tile(v, wave, stage, lane);
    for (int lt = 0; lt < nloc; ++lt) {
        const int tile_i = wave + WAVES * lt;
        const bool last = lt + 1 == nloc;
        const bool rec = !last && lt < kSpecTiles;
        if (!rec) run = -INFINITY;
        float tmin = INFINITY;
        stage_wait();
        fp4::pass(tabs, stage, lane, tile_i * kFPP + col < T, lm, vmax, tmin, nanp, [&] {
            if (!last) stage_tile(v, tile_i + WAVES, stage, lane);
        });
        const float tmw = wave_min(tmin);
        vmin = fminf(vmin, tmw);
        if (last) { last_min = tmw; break; }
        const float run2 = rec ? wave_max(vmax) - kTopDbUnits : -INFINITY;
        run = fmaxf(run, run2);
        float c[8];
        fp4::dct(lm, run, tabs, lane, c);
        if (lt == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cref[i] = __shfl(c[i], lane & 48, 64);
        }
        stats_add(c, cref, tile_i * kFPP + col < T, s1, s2);
        if (lane == 0 && rec) {
            spec[lt] = fmaxf(tmw, run);
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
    (void)last_min;
    if (nloc > 0) {
        const int tile_l = wave + WAVES * (nloc - 1);
        float c[8];
        fp4::dct(lm, theta, tabs, lane, c);   // the last tile, still in registers: clamped at the final threshold
        if (nloc == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cref[i] = __shfl(c[i], lane & 48, 64);
        }
        stats_add(c, cref, tile_l * kFPP + col < T, s1, s2);
        if (vmin < theta) {
            lds_order();
            for (int lt = 0; lt + 1 < nloc; ++lt) {
                const bool rec = lt < kSpecTiles;
                if (rec && !(spec[lt] < theta)) continue;
                fix_tile(v, wave + WAVES * lt, T, rec ? spec[kSpecRun + lt] : -INFINITY, theta, tabs, stage, lane, cref,
                         s1, s2);
            }
        }
    }
    if (__ballot(nanp != nanp)) {   // NaN input (segment_stats): the combined sums go NaN
#pragma unroll
        for (int i = 0; i < 8; ++i) s1[i] = __builtin_nan("");
    }
    // this wave's per-coefficient (s1, s2, cref) -> its scratch, as doubles [coef][3]
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
    if (wave == 0) {
        double mean = 0.0, sd = 0.0;
        if (lane < NMFCC) {
            const double* p0 = reinterpret_cast<const double*>(smem + L_WAVES + W_PD);
            const double r0 = p0[3 * lane + 2];
            double S1 = 0.0, S2 = 0.0;
            for (int w = 0; w < WAVES; ++w) {
                int n = 0;   // valid frames of wave w's tiles
                for (int ti = w; ti < ntile; ti += WAVES) n += min(kFPP, T - kFPP * ti);
                if (n == 0) continue;
                const double* pw = reinterpret_cast<const double*>(smem + L_WAVES + w * W_BYTES + W_PD);
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
                                                   double vv_s) {
#pragma clang fp contract(off)
    const double sm = 1.0 - clip02(1.0 - uv_m / sqrt(uu_m * vv_m));
    const double ss = 1.0 - clip02(1.0 - uv_s / sqrt(uu_s * vv_s));
    const double percent = (sm * 0.7 + ss * 0.3) * 100.0;
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
        double score, std2, mean2;
        if (a.cand_f32) {   // float32 candidates: float products, float-rounded dots (sdot)
            const float uv_m = (float)wave_sum_d((double)(tmf * cmf)), vv_m = (float)wave_sum_d((double)(cmf * cmf));
            const float uv_s = (float)wave_sum_d((double)(tsf * csf)), vv_s = (float)wave_sum_d((double)(csf * csf));
            score = score_f32_finish(a.uu_m32, a.uu_s32, uv_m, vv_m, uv_s, vv_s);
            std2 = vv_s;
            mean2 = vv_m;
        } else {
            const double uv_m = wave_sum_d((double)tmf * (double)cmf), vv_m = wave_sum_d((double)cmf * (double)cmf);
            const double uv_s = wave_sum_d((double)tsf * (double)csf), vv_s = wave_sum_d((double)csf * (double)csf);
            score = score_f64_finish((double)a.uu_m32, (double)a.uu_s32, uv_m, vv_m, uv_s, vv_s);
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
            near = near || fabs(score - a.threshold) < a.rescore_margin || (1 + len / HOP) <= kRescoreFrames ||
                   (std2 > 0.0 && std2 < kTinyStd * kTinyStd) || mean2 < kTinyMean * kTinyMean;
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
    // ---- cooperative table load (global -> LDS)
    fp4::fill_tables(tab, smem + L_TAB, kWinScale, threadIdx.x, blockDim.x);
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int base = 0, count = a.n_seg;
    if (RING) {
        base = r_base;
        count = r_count;
    }
    // the wave's LDS (a wave-uniform base: the LDS-DMA destination lives in M0)
    unsigned char* wbase = smem + L_WAVES + __builtin_amdgcn_readfirstlane(wave * W_BYTES);
    float* stage = reinterpret_cast<float*>(wbase + W_STAGE);
    double* pd = reinterpret_cast<double*>(wbase + W_PD);
    float* spec = reinterpret_cast<float*>(wbase + W_SPEC);
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
        float* misc0 = reinterpret_cast<float*>(smem + L_WAVES + W_PD);   // wave 0's scratch (epilogue only)
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
                segment_stats_coop(v, smem, stage, spec, pd, wave, lane, misc0, theta_s);
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
    const WorkCtx wc = {&a, base, count, true};
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
        segment_stats(v, smem + L_TAB, stage, spec, pd, lane, st1, st2, theta_s, wc, nx EWK_DBG_ARG);
        EWK_TS(tw2);

        // ---- lane k < 20 holds coefficient k's mean / std (fp32-rounded like the reference's)
        const float cmf = act ? (float)st1[0] : 0.0f, csf = act ? (float)st2[0] : 0.0f;
        if (act && !RING) {
            if (a.out_mean) a.out_mean[(int64_t)seg * NMFCC + lane] = cmf;
            if (a.out_std) a.out_std[(int64_t)seg * NMFCC + lane] = csf;
        }
        if (a.has_template || a.list_all) score_epilogue<RING>(a, cmf, csf, tmf, tsf, lane, seg, v.len, theta_s);
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

