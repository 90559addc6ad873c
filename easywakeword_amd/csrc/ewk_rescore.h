// ewk_rescore.h -- the fp64 re-score of the segments the float32 pass cannot decide alone
// (near the threshold, very short, nearly stationary, or with a vanishing MFCC mean vector:
// see score_epilogue), run by a launch right after the scorer (k_rescore_linear,
// k_rescore_ring).  Included by ewk_mfcc.hip after the score arithmetic; device code only.
//
// This is the float64 candidate path of the reference (wakeword.py:509-513 hands float64 ring
// slices to WordMatcher.extract_mfcc, wakeword.py:544-567 -> librosa 0.11.0 feature.mfcc with
// complex128 stft, float32 Slaney weights, float64 power_to_db and DCT, numpy mean / std).
//
// Work split.  A listed segment is a slot; its frames are cut into 8-frame chunks whose part
// records are consecutive in a pool (the lister reserves them with one atomic and writes each
// record's slot index).  Every wave of the re-score launch claims part record g with one atomic
// on a shared cursor, runs that chunk and counts it done on its slot; the wave finishing a
// slot's last chunk merges the slot.  The part records live in uncached memory, so a record
// written by one wave is read by another on any XCD without an L2 write-back or invalidate
// (round 4: an agent-scope acquire per scanned slot invalidated the XCD's L2 on every claim,
// and a burst tick took 5 ms).  One chunk = one wave, one frame at a time over its 64 lanes:
//   samples -> windowed z[n] = w[2n] x[2n] + i w[2n+1] x[2n+1] (lane j: n = j + 64 r)
//   -> radix-4 Stockham FFT (Ns = 1, 4, 16, 64; LDS between iterations, natural order out)
//   -> real-FFT untangle + power (partner bin 256 - k through LDS) -> Slaney bands over each
//   band's packed support -> 10 log10(max(1e-10, .)) into the chunk's log-mel tile.
// top_db couples every frame to the segment's max; the chunk does not know it yet.  So the
// DCT is split by a speculative clamp theta_s (the float32 pass's max - 80 dB):
//   c_k = A_k + theta B_k,  A_k = sum_{x >= theta} D_km x_m,  B_k = sum_{x < theta} D_km,
// exact for the true theta as long as no value lies within kRsWindow of theta_s (then the
// classification x >= theta_s equals x >= theta); a chunk holding such a value is recomputed
// with the exact theta by the wave that finishes the slot (rare: ~1 chunk in 1,000-5,000).
// The chunk's sums (shifted by its first frame: identical frames give an exact 0 std) go to
// a part record; the finishing wave merges the parts in chunk order as polynomials in theta,
// so the result does not depend on which waves ran which chunks (MODE 0, 1, 2 and the
// serial fallback give the same bits).
//
// scripts/f64_chunk_model.py is the numpy model of these index maps and algebra.

// Drain counters of a -DEWK_RS_TIMING debug build (scripts/rescore_ring_probe.py reads them
// with ewk_debug_rs); the product build compiles none of it.
#ifdef EWK_RS_TIMING
__device__ unsigned long long g_rs_dbg[16];
#define EWK_RS_ADD(k, v) (void)atomicAdd(&g_rs_dbg[k], (unsigned long long)(v))
#define EWK_RS_MAX(k, v) (void)atomicMax(&g_rs_dbg[k], (unsigned long long)(v))
// chunk sub-phases (s_memtime cycles summed over chunks): 0 samples + window, 1 FFT stages,
// 2 untangle + power, 3 mel + log10, 4 DCT, 5 sums + flags, 6 chunks, 7 frame groups
// (summed in registers, flushed once per chunk: an atomic inside the frame loop would put a
// memory round trip into the next sample wait)
__device__ unsigned long long g_rs_ph[8];
#define EWK_RS_TS(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define EWK_RS_PH(k, a, b) (rph[k] += (b) - (a))
#define EWK_RS_PARAM , unsigned long long(&rph)[8]
#define EWK_RS_ARG , rph
#else
#define EWK_RS_ADD(k, v) ((void)0)
#define EWK_RS_MAX(k, v) ((void)0)
#define EWK_RS_TS(v)
#define EWK_RS_PH(k, a, b) ((void)0)
#define EWK_RS_PARAM
#define EWK_RS_ARG
#endif

// dB.  Measured (scripts/rs_window_probe.py, every segment of the bench batch at three lengths and
// of four other recipes listed: ~210,000 segments): |theta - theta_s| <= 1.98e-5 dB, so 2e-4 keeps a
// 10x margin; a wider window only recomputes more chunks (1e-3: 61 of 16,358 bench chunks,
// 516 of 16,376 stationary ones), a slot beyond it redoes every chunk (correct, slower).
#ifndef EWK_RS_WINDOW
#define EWK_RS_WINDOW 2e-4
#endif
constexpr double kRsWindow = EWK_RS_WINDOW;
constexpr double kRsTopDb = 80.0;

// What the drain needs of ScoreArgs, copied in score_tail: the drain is a real call (its
// registers are its own), and a reference to the kernel's own ScoreArgs would make the
// compiler copy the whole kernarg block to scratch and read every field from there in the
// float32 hot loop as well.
struct RsArgs {
    const float* pcm;
    const int16_t* pcm16;
    const int64_t* offsets;
    const int32_t* lengths;
    ewk_event* events;
    int64_t ring_len;
    const float* tmpl;
    double threshold;
    int32_t has_template;
    int32_t cand_f32;
    int32_t* rs_ctl;
    RsSlot* rs_slots;
    int32_t* rs_serial;
    RsPart* rs_parts;
    int32_t rs_cap;
    int32_t rs_part_cap;
    double* out_score;
    uint8_t* out_match;
    double* out_mean64;
    double* out_std64;
    const Tables64* tab64;
};

__device__ __forceinline__ RsArgs rs_args(const ScoreArgs& a) {
    RsArgs r;
    r.pcm = a.pcm; r.pcm16 = a.pcm16; r.offsets = a.offsets; r.lengths = a.lengths; r.events = a.events;
    r.ring_len = a.ring_len; r.tmpl = a.tmpl; r.threshold = a.threshold; r.has_template = a.has_template;
    r.cand_f32 = a.cand_f32; r.rs_ctl = a.rs_ctl; r.rs_slots = a.rs_slots; r.rs_parts = a.rs_parts;
    r.rs_serial = a.rs_serial; r.rs_part_cap = a.rs_part_cap;
    r.rs_cap = a.rs_cap; r.out_score = a.out_score; r.out_match = a.out_match; r.out_mean64 = a.out_mean64;
    r.out_std64 = a.out_std64; r.tab64 = a.tab64;
    return r;
}

// The re-score launches run their own workgroup shape: RS_NW waves sharing the tables below.
// Two waves per SIMD: a third (12 waves, <= 168 VGPRs) made each chunk 1.85x slower -- the
// SIMD's fp64 VALU is the shared resource, not latency (profiles/r04_v9_rescore_variants.txt).
#ifndef EWK_RS_NW
#define EWK_RS_NW 8
#endif
constexpr int RS_NW = EWK_RS_NW;
// LDS of the re-score launch.  The DCT table is whole, [m][k]: the half table (the DCT-II rows
// are (anti)symmetric) cost a mirrored index and a sign per band in the DCT's inner loop.
constexpr int RS_D = 0;                                     // double [NMEL][NMFCC]
constexpr int RS_MLO = RS_D + NMEL * NMFCC * 8;             // int [NMEL]
constexpr int RS_MOFF = RS_MLO + NMEL * 4;                  // int [NMEL + 1]
constexpr int RS_MW = RS_MOFF + (NMEL + 4) * 4;             // float [2 NBIN + 2 NMEL]
constexpr int RS_MW_N = 2 * NBIN + 2 * NMEL;
constexpr int RS_WAVES = (RS_MW + RS_MW_N * 4 + 15) & ~15;
// Two frames in flight per wave (rs_frames): each has its own FFT buffer.
constexpr int RS_NF = 2;
constexpr int RS_BUF = 0;                                   // per wave: RS_NF x (double2 [256] FFT / double P[257])
constexpr int RS_XA = RS_NF * 256 * 16;                     // double [NMEL][kRsFrames]: the chunk's log-mel
constexpr int RS_WAVE_BYTES = RS_XA + NMEL * kRsFrames * 8;
constexpr int RS_FLAGS = RS_WAVES + RS_NW * RS_WAVE_BYTES;  // int [3 + RS_NW]: score_tail's flags
constexpr int RS_PRE = (RS_FLAGS + 4 * (3 + RS_NW) + 15) & ~15;   // TickPre (empty-launch tick end)
constexpr int RS_LDS = RS_PRE + 32;
static_assert(RS_LDS <= 160 * 1024, "the re-score workgroup must fit a CU's LDS");
static_assert(NMFCC == 20 && kRsFrames == 8, "the DCT lane split assumes 20 coefficients and 8-frame chunks");

// Between a wave's LDS writes and its other lanes' reads: LDS operations of one wave execute in
// program order, so a compiler barrier suffices (a wavefront-scope fence would also wait for
// the next frame's sample loads, rs_chunk).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// A segment's samples for the fp64 path (linear batch or wrap-aware ring slice).
struct SegView {
    const float* p;       // linear: the batch base; ring: stream ring base (float32) ...
    const int16_t* p16;   // ... or int16 ring base (EWK_RING_I16)
    int64_t start;        // linear: segment offset; ring: physical index of sample 0
    int64_t ring;         // 0 = linear
    int32_t len;
};

template <int RING>
__device__ __forceinline__ SegView rs_view(const RsArgs& a, int seg) {
    SegView v;
    if (RING) {
        const ewk_event ev = a.events[seg];
        v.p = a.pcm ? a.pcm + (int64_t)ev.stream * a.ring_len : nullptr;
        v.p16 = a.pcm16 ? a.pcm16 + (int64_t)ev.stream * a.ring_len : nullptr;
        v.start = ev.ring_start;
        v.ring = a.ring_len;
        v.len = ev.length;
    } else {
        v.p = a.pcm;
        v.p16 = nullptr;
        v.start = a.offsets[seg];
        v.ring = 0;
        v.len = a.lengths[seg];
    }
    return v;
}

// Per-lane constants of the frame pipeline (from the fp64 tables in global memory, L2-hot).
struct RsLane {
    double win[8];    // w[2n], w[2n+1] for n = lane + 64 r
    double2 tw[9];    // Stockham twiddles W_{4 Ns}^{r (lane % Ns)}, Ns = 4, 16, 64, r = 1..3
    double2 tu[4];    // untangle (cos, sin)(2 pi k / 512), k = lane + 64 r
};

__device__ __forceinline__ void rs_lane_init(const Tables64* __restrict__ tb, int lane, RsLane& c) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int n = lane + 64 * r;
        c.win[2 * r] = tb->win[2 * n];
        c.win[2 * r + 1] = tb->win[2 * n + 1];
        c.tu[r] = make_double2(tb->cs[n], tb->sn[n]);
    }
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const int lg = 2 * it + 2, e = lane & ((1 << lg) - 1);   // Ns = 4 << (2 it)
#pragma unroll
        for (int r = 1; r < 4; ++r) {
            const int idx = ((128 >> lg) * r * e) & (NFFT - 1);  // W_{4 Ns}^{r e} = W_512^{(128 / Ns) r e}
            c.tw[3 * it + r - 1] = make_double2(tb->cs[idx], -tb->sn[idx]);
        }
    }
}

__device__ __forceinline__ double2 zmul(double2 a, double2 w) {
    return make_double2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}

// The WG-shared tables: the DCT as [m][k] (lanes of one band read 20 consecutive doubles)
// and the Slaney bands' packed support.
__device__ void rs_load_tables(const Tables64* __restrict__ tb, unsigned char* smem) {
    double* D = reinterpret_cast<double*>(smem + RS_D);
    int* mlo = reinterpret_cast<int*>(smem + RS_MLO);
    int* moff = reinterpret_cast<int*>(smem + RS_MOFF);
    float* mw = reinterpret_cast<float*>(smem + RS_MW);
    for (int i = threadIdx.x; i < NMEL * NMFCC; i += blockDim.x) {
        const int m = i / NMFCC, k = i % NMFCC;
        D[i] = tb->dct[k * NMEL + m];
    }
    for (int i = threadIdx.x; i < NMEL; i += blockDim.x) mlo[i] = tb->mel_lo[i];
    for (int i = threadIdx.x; i <= NMEL; i += blockDim.x) moff[i] = tb->mel_off[i];
    for (int i = threadIdx.x; i < 2 * NBIN + 2 * NMEL; i += blockDim.x) mw[i] = tb->mel_w[i];
}

// One frame t of the segment -> column f of the chunk's log-mel tile (split at theta_s),
// with the running max, the ambiguity flag (|x - theta_s| <= W) and the NaN flag.
// A segment's samples through a buffer descriptor (as the float32 pass, SegSrc): the range
// check returns 0 for an offset of -1, so a frame's eight loads are branch-free and all in
// flight at once (per-sample bounds branches put a vmcnt wait behind every load).
template <int RING>
struct RsSrc {
    __amdgpu_buffer_rsrc_t rsrc;   // linear: the segment; ring: the whole stream ring
    int32_t len, start, ring;
};
template <int RING>
__device__ __forceinline__ RsSrc<RING> rs_src(const SegView& v) {
    RsSrc<RING> r;
    const void* p = RING == 2 ? (const void*)v.p16 : (const void*)(RING ? v.p : v.p + v.start);
    const uint64_t bu = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)bu), hi = __builtin_amdgcn_readfirstlane((uint32_t)(bu >> 32));
    const int32_t n = __builtin_amdgcn_readfirstlane(RING ? (int32_t)v.ring : v.len);
    r.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                               n * (RING == 2 ? 2 : 4), 0x00020000);
    r.len = __builtin_amdgcn_readfirstlane(v.len);
    r.start = __builtin_amdgcn_readfirstlane((int32_t)v.start);
    r.ring = n;
    return r;
}
template <int RING>
__device__ __forceinline__ float rs_sample(const RsSrc<RING>& v, int q) {
    const bool in = (unsigned)q < (unsigned)v.len;   // stft(center=True, pad_mode='constant')
    int phys = q;
    if (RING) phys = q + v.start >= v.ring ? q + v.start - v.ring : q + v.start;
    const int off = in ? phys * (RING == 2 ? 2 : 4) : -1;
    if (RING == 2) return (float)(short)__builtin_amdgcn_raw_buffer_load_b16(v.rsrc, off, 0, 0) * (1.0f / 32768.0f);
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(v.rsrc, off, 0, 0));
}
// The eight samples lane j needs of frame t (x[2n], x[2n + 1] for n = j + 64 r), requested one
// frame ahead of their use (rs_chunk), so a frame's loads wait behind the previous frame's FFT.
template <int RING>
__device__ __forceinline__ void rs_load(const RsSrc<RING>& v, int t, int lane, float (&s)[8]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int q = t * HOP - NFFT / 2 + 2 * (lane + 64 * r);
        s[2 * r] = rs_sample(v, q);
        s[2 * r + 1] = rs_sample(v, q + 1);
    }
}

// The windowed frame z[n] = w[2n] x[2n] + i w[2n+1] x[2n+1], n = lane + 64 r.
__device__ __forceinline__ void rs_window(const float (&smp)[8], const RsLane& c, double2 (&x)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = make_double2(c.win[2 * r] * (double)smp[2 * r], c.win[2 * r + 1] * (double)smp[2 * r + 1]);
}

// FFT buffer slot of complex element i (16-B units): the low 4 bits XORed with 5 x (i >> 4).
// Every radix-4 Stockham store (slot ((j >> lg) << (lg + 2)) + j % 4^lg + r 4^lg) and every
// natural-order read then hits 16 distinct 16-B bank groups per 16 lanes (unswizzled, the Ns = 1
// and 4 stores were 4-way conflicts: 41 % of the launch's LDS cycles).  scripts/f64_chunk_model.py
// checks the permutation and the conflict counts.
__device__ __forceinline__ int rs_swz(int i) { return i ^ (((i >> 4) * 5) & 15); }

// NF frames f0 .. f0 + NF - 1 (samples already windowed) -> columns f0 .. of the chunk's
// log-mel tile, interleaved: the frames' FFT stages, untangles and bands are independent
// instruction streams, so one frame's LDS round trips and fp64 latencies overlap the other's
// (one frame at a time, a chunk waited 70 % of its cycles).  valid[j]: frame j counts towards
// mx / amb / nanf / clp (a chunk's odd last frame rides along as a dummy).
template <int NF>
__device__ __forceinline__ void rs_frames(const double2 (&xw)[NF][4], const bool (&valid)[NF], const RsLane& c,
                                          unsigned char* wbuf, const unsigned char* smem, int lane, int f0,
                                          double theta_s, double W, double& mx, bool& amb, bool& nanf,
                                          bool& clp EWK_RS_PARAM) {
    EWK_RS_TS(p0);
    double2 x[NF][4];
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[j][r] = xw[j][r];
    // radix-4 Stockham autosort: v[r] = d[j + 64 r], v[r] *= W_{4 Ns}^{r (j % Ns)}, DFT4,
    // V[r] -> d'[(j / Ns) 4 Ns + j % Ns + r Ns]; natural order after Ns = 64
#ifndef EWK_RS_SKIP_FFT
    for (int it = 0; it < 4; ++it) {
#else
    for (int it = 0; it < 4; it += 3) {
#endif
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            double2* buf = reinterpret_cast<double2*>(wbuf + RS_BUF) + 256 * j;
            if (it > 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) x[j][r] = buf[rs_swz(lane + 64 * r)];
#pragma unroll
                for (int r = 1; r < 4; ++r) x[j][r] = zmul(x[j][r], c.tw[3 * (it - 1) + r - 1]);
            }
            const double2 a0 = make_double2(x[j][0].x + x[j][2].x, x[j][0].y + x[j][2].y);
            const double2 a1 = make_double2(x[j][0].x - x[j][2].x, x[j][0].y - x[j][2].y);
            const double2 a2 = make_double2(x[j][1].x + x[j][3].x, x[j][1].y + x[j][3].y);
            const double2 a3 = make_double2(x[j][1].x - x[j][3].x, x[j][1].y - x[j][3].y);
            x[j][0] = make_double2(a0.x + a2.x, a0.y + a2.y);
            x[j][2] = make_double2(a0.x - a2.x, a0.y - a2.y);
            x[j][1] = make_double2(a1.x + a3.y, a1.y - a3.x);   // a1 - i a3
            x[j][3] = make_double2(a1.x - a3.y, a1.y + a3.x);   // a1 + i a3
        }
        const int lg = 2 * it;
        const int base = it < 3 ? ((lane >> lg) << (lg + 2)) + (lane & ((1 << lg) - 1)) : lane;
        wave_sync();   // every lane has read this iteration's inputs
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            double2* buf = reinterpret_cast<double2*>(wbuf + RS_BUF) + 256 * j;
#pragma unroll
            for (int r = 0; r < 4; ++r) buf[rs_swz(base + (r << lg))] = x[j][r];   // (it = 3: Z[lane + 64 r])
        }
        wave_sync();
    }
    EWK_RS_TS(p1);
    EWK_RS_PH(1, p0, p1);
    // untangle: X[k] = E + W512^k O,  E = (Z[k] + conj Z[256-k]) / 2,  O = (Z[k] - conj Z[256-k]) / 2i
    double p[NF][4], d256[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const double2* buf = reinterpret_cast<const double2*>(wbuf + RS_BUF) + 256 * j;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = lane + 64 * r;
            const double2 zk = x[j][r], zc = buf[rs_swz((256 - k) & 255)];
            const double er = 0.5 * (zk.x + zc.x), ei = 0.5 * (zk.y - zc.y);
            const double orr = 0.5 * (zk.y + zc.y), oi = -0.5 * (zk.x - zc.x);
            const double2 cs = c.tu[r];
            const double xr = er + (orr * cs.x + oi * cs.y);
            const double xi = ei + (oi * cs.x - orr * cs.y);
            p[j][r] = xr * xr + xi * xi;
        }
        d256[j] = x[j][0].x - x[j][0].y;   // k = 256 (lane 0): W512^256 = -1 exactly
    }
    wave_sync();
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        double* P = reinterpret_cast<double*>(wbuf + RS_BUF) + 512 * j;
#pragma unroll
        for (int r = 0; r < 4; ++r) P[lane + 64 * r] = p[j][r];
        if (lane == 0) P[256] = d256[j] * d256[j];
    }
    wave_sync();
    EWK_RS_TS(p2);
    EWK_RS_PH(2, p1, p2);
    // mel (every non-zero weight of the band, in bin order) + dB; lane: bands lane, 127 - lane
    const int* mlo = reinterpret_cast<const int*>(smem + RS_MLO);
    const int* moff = reinterpret_cast<const int*>(smem + RS_MOFF);
    const float* mw = reinterpret_cast<const float*>(smem + RS_MW);
    double* xa = reinterpret_cast<double*>(wbuf + RS_XA);
    // a fixed-width window per band, read unconditionally (one LDS round trip, no branch):
    // kRsMelWLo bins for the lane's low band (bands 0..63 span <= 3 bins), kRsMelW for its high
    // one; past the band's support the weight is selected to 0, and fma(0, p, acc) = acc, so the
    // sum is the band's, in bin order
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int m = h ? NMEL - 1 - lane : lane;
        const int kw = h ? kRsMelW : kRsMelWLo;   // (h unrolled: a constant)
        const int lo = mlo[m], o0 = moff[m], nw = moff[m + 1] - o0;
        // every weight read unconditionally (clamped index), then selected: a conditional read
        // made each weight its own exec-masked block (24 branches per frame pair)
        float ww[kRsMelW];
#pragma unroll
        for (int q = 0; q < kRsMelW; ++q) ww[q] = q < kw ? mw[min(o0 + q, RS_MW_N - 1)] : 0.0f;
#pragma unroll
        for (int q = 0; q < kRsMelW; ++q) ww[q] = q < nw ? ww[q] : 0.0f;
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            const double* P = reinterpret_cast<const double*>(wbuf + RS_BUF) + 512 * j;
            double pw[kRsMelW];
#pragma unroll
            for (int q = 0; q < kRsMelW; ++q) pw[q] = q < kw ? P[lo + q] : 0.0;   // lo + q < 2 * 256: inside the frame's buffer
            double acc = 0.0;
#ifndef EWK_RS_SKIP_MEL
            // past the band: weight 0 times a finite power of this frame (its FFT buffer; a NaN
            // there means NaN samples, and then every bin is NaN) adds +-0, and acc + -0 = acc
#pragma unroll
            for (int q = 0; q < kRsMelW; ++q)
                if (q < kw) acc = fma((double)ww[q], pw[q], acc);
#else   // (timing experiment: one bin per band)
            acc = pw[0] + (double)ww[0] + (double)nw;
#endif
#ifndef EWK_RS_SKIP_LOG
            // (ewk_db64.h: 10 log10 in ~30 float64 instructions; the library's log10 takes ~100)
            const double db = ewk_db64(acc < 1e-10 ? 1e-10 : acc);   // np.maximum: NaN propagates
#else
            const double db = acc;
#endif
            // the A operand, or -0.0 for a value the clamp replaces (NaN included): fma(d, -0, A) = A
            // as with +0, and db is never -0.0 (10 log10(acc), acc >= 1e-10), so -0.0 also marks
            // the B operand for rs_dct (no second tile)
            xa[m * kRsFrames + f0 + j] = db >= theta_s ? db : -0.0;
            // selects, not a branch: the four bands' log10 chains (~90 dependent fp64 ops
            // each) stay in one block, where the scheduler can interleave them
            const bool vj = valid[j];
            clp = clp | (vj & !(db >= theta_s));
            mx = vj ? fmax(mx, db) : mx;
            amb = amb | (vj & (fabs(db - theta_s) <= W));
            nanf = nanf | (vj & (db != db));
        }
    }
    wave_sync();
    EWK_RS_TS(p3);
    EWK_RS_PH(3, p2, p3);
    EWK_RS_PH(7, 0ull, 1ull);
}

// DCT of the chunk's n frames split at theta_s: lane k < 20 returns A_k, B_k of frames 0..7
// (A: the values x >= theta_s, B: the weights of the others -- NaN included -- which the
// clamp replaces by theta; rs_frame stored those as -0.0).  Lanes (k, h) = (l % 20, l / 20),
// l < 60, take bands [43 h, 43 h + 43), EWK_RS_DCT_U bands' reads in flight together; the
// thirds are added in a fixed order (h = 0, 1, 2).
#ifndef EWK_RS_DCT_U
#define EWK_RS_DCT_U 2
#endif
__device__ __forceinline__ void rs_dct(const unsigned char* smem, unsigned char* wbuf, int lane, bool need_b,
                                       double (&A)[8], double (&B)[8]) {
    const double* D = reinterpret_cast<const double*>(smem + RS_D);
    double* xa = reinterpret_cast<double*>(wbuf + RS_XA);
#pragma unroll
    for (int f = 0; f < 8; ++f) { A[f] = 0.0; B[f] = 0.0; }
    if (lane < 60) {
        const int k = lane % NMFCC, h = lane / NMFCC;
        const int m0 = 43 * h;
#ifndef EWK_RS_SKIP_DCT
        const int m1 = min(NMEL, m0 + 43);
#else
        const int m1 = m0 + 1;
#endif
        const double* dp = D + k;
        const double4* xp = reinterpret_cast<const double4*>(xa);
        // one band: A[f] += D[k][m] x[m][f]; B[f] += D[k][m] where x[m][f] was clamped (-0.0)
        auto band = [&](double d, const double4& n0, const double4& n1) {
            const double av[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
#pragma unroll
            for (int f = 0; f < 8; ++f) A[f] = fma(d, av[f], A[f]);
            if (need_b) {   // (wave-uniform: a chunk with no clamped value has B = 0 exactly)
#pragma unroll
                for (int f = 0; f < 8; ++f) {
                    const bool clamped = __double2hiint(av[f]) == (int)0x80000000;   // -0.0
                    B[f] = fma(d, clamped ? 1.0 : 0.0, B[f]);
                }
            }
        };
        // kRsDctU bands per step, their reads issued together (one LDS wait per step, bands in
        // order: the same sums as one band per step)
        constexpr int kRsDctU = EWK_RS_DCT_U;
        int m = m0;
        for (; m + kRsDctU <= m1; m += kRsDctU) {
            double d[kRsDctU];
            double4 n[kRsDctU][2];
#pragma unroll
            for (int u = 0; u < kRsDctU; ++u) {
                d[u] = dp[(m + u) * NMFCC];
                n[u][0] = xp[2 * (m + u)];
                n[u][1] = xp[2 * (m + u) + 1];
            }
#pragma unroll
            for (int u = 0; u < kRsDctU; ++u) band(d[u], n[u][0], n[u][1]);
        }
        for (; m < m1; ++m) band(dp[m * NMFCC], xp[2 * m], xp[2 * m + 1]);
    }
    wave_sync();
    if (lane >= NMFCC && lane < 60) {   // thirds 1, 2 park their sums in the (consumed) XA tile
        double* red = xa + (lane - NMFCC) * 16;
#pragma unroll
        for (int f = 0; f < 8; ++f) { red[f] = A[f]; red[8 + f] = B[f]; }
    }
    wave_sync();
    if (lane < NMFCC) {
        const double* r1 = xa + lane * 16;
        const double* r2 = xa + (NMFCC + lane) * 16;
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            A[f] = (A[f] + r1[f]) + r2[f];
            B[f] = (B[f] + r1[8 + f]) + r2[8 + f];
        }
    }
    wave_sync();
}

__device__ __forceinline__ double wave_max_d(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o, 64));
    return x;
}

// One chunk (frames 8c .. 8c + n - 1): lane k < 20 returns its 7 sums {rA, rB, sA, sB, sAA,
// sAB, sBB} (shift = the chunk's first frame); mx / n / flags are wave-uniform.
template <int RING>
__device__ void rs_chunk(const RsSrc<RING>& v, int T, int c, double theta_s, double W, const RsLane& cl,
                         const unsigned char* smem, unsigned char* wbuf, int lane, double (&pv)[7], double& mx,
                         int& n, int& flags) {
    const int t0 = c * kRsFrames;
    n = min(kRsFrames, T - t0);
    double m = -INFINITY;
    bool amb = false, nanf = false, clp = false;
#ifdef EWK_RS_TIMING
    unsigned long long rph[8] = {};
#endif
    float smp[RS_NF][8];
#pragma unroll
    for (int j = 0; j < RS_NF; ++j) rs_load(v, t0 + j, lane, smp[j]);   // (past T: range-checked zeros)
    for (int f = 0; f < n; f += RS_NF) {
        EWK_RS_TS(w0);
        double2 xw[RS_NF][4];
        bool valid[RS_NF];
#pragma unroll
        for (int j = 0; j < RS_NF; ++j) {
            rs_window(smp[j], cl, xw[j]);
            valid[j] = f + j < n;
        }
        // the next frames' loads go out only after these frames' samples are consumed (issued
        // before, the compiler's in-order vmcnt wait for these samples also covered the first
        // of them; time-neutral, profiles/r04_v9_rescore_pmc.txt)
#pragma unroll
        for (int j = 0; j < RS_NF; ++j)
            asm volatile("" ::"v"(xw[j][0].x), "v"(xw[j][0].y), "v"(xw[j][1].x), "v"(xw[j][1].y), "v"(xw[j][2].x),
                         "v"(xw[j][2].y), "v"(xw[j][3].x), "v"(xw[j][3].y)
                         : "memory");
        EWK_RS_TS(w1);
        EWK_RS_PH(0, w0, w1);
        if (f + RS_NF < n) {
#pragma unroll
            for (int j = 0; j < RS_NF; ++j) rs_load(v, t0 + f + RS_NF + j, lane, smp[j]);
        }
        rs_frames<RS_NF>(xw, valid, cl, wbuf, smem, lane, f, theta_s, W, m, amb, nanf, clp EWK_RS_ARG);
    }
    double A[8], B[8];
    EWK_RS_TS(d0);
    rs_dct(smem, wbuf, lane, __ballot(clp) != 0, A, B);
    EWK_RS_TS(d1);
    EWK_RS_PH(4, d0, d1);
    const double rA = A[0], rB = B[0];
    double sA = 0.0, sB = 0.0, sAA = 0.0, sAB = 0.0, sBB = 0.0;
#pragma unroll
    for (int f = 1; f < 8; ++f) {
        if (f < n) {
            const double dA = A[f] - rA, dB = B[f] - rB;
            sA += dA;
            sB += dB;
            sAA = fma(dA, dA, sAA);
            sAB = fma(dA, dB, sAB);
            sBB = fma(dB, dB, sBB);
        }
    }
    pv[0] = rA; pv[1] = rB; pv[2] = sA; pv[3] = sB; pv[4] = sAA; pv[5] = sAB; pv[6] = sBB;
    mx = wave_max_d(m);
    flags = (__ballot(amb) ? 1 : 0) | (__ballot(nanf) ? 2 : 0);
    EWK_RS_TS(d2);
    EWK_RS_PH(5, d1, d2);
    EWK_RS_PH(6, 0ull, 1ull);
#ifdef EWK_RS_TIMING
    if (lane == 0)
        for (int k = 0; k < 8; ++k) (void)atomicAdd(&g_rs_ph[k], rph[k]);
#endif
}

// A part record's fields cross waves (any XCD) inside one launch: they are stored and loaded as
// agent-scope relaxed atomics (global_store / global_load with sc1: performed at the agent's
// coherence point, no copy kept in a CU's vector L1 or an XCD's L2), so the hand-off does not
// depend on the pool's memory type or on which records share a 128-B line.  The writer's
// s_waitcnt vmcnt(0) (its stores acknowledged) precedes its done count; the finishing wave's
// agent acquire (buffer_inv sc1) follows the count that made it last.  DESIGN.md, "fp64
// re-score", hand-off.
// (global address space: global_* instructions, counted by vmcnt alone, not flat_*)
template <class T>
__device__ __forceinline__ void rs_st(T* p, T v) {
    __hip_atomic_store((__attribute__((address_space(1))) T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T rs_ld(const T* p) {
    return __hip_atomic_load((__attribute__((address_space(1))) T*)const_cast<T*>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

// Chunk sums merged in chunk order as polynomials in theta (the clamp is known only at the end):
// S1(theta) = P1a + theta P1b, S2(theta) = P2a + theta P2b + theta^2 P2c around the first
// chunk's first frame c_0(theta) = rA0 + theta rB0.
struct RsAcc {
    double rA0 = 0.0, rB0 = 0.0, P1a = 0.0, P1b = 0.0, P2a = 0.0, P2b = 0.0, P2c = 0.0;
    bool init = false;
};

__device__ __forceinline__ void rs_merge(RsAcc& s, const double (&pv)[7], int n) {
    const double rA = pv[0], rB = pv[1], sA = pv[2], sB = pv[3], sAA = pv[4], sAB = pv[5], sBB = pv[6];
    if (!s.init) {
        s.rA0 = rA; s.rB0 = rB;
        s.P1a = sA; s.P1b = sB;
        s.P2a = sAA; s.P2b = 2.0 * sAB; s.P2c = sBB;
        s.init = true;
        return;
    }
    const double dA = rA - s.rA0, dB = rB - s.rB0, nd = (double)n;
    s.P2a += sAA + 2.0 * dA * sA + nd * dA * dA;
    s.P2b += 2.0 * sAB + 2.0 * dA * sB + 2.0 * dB * sA + 2.0 * nd * dA * dB;
    s.P2c += sBB + 2.0 * dB * sB + nd * dB * dB;
    s.P1a += sA + nd * dA;
    s.P1b += sB + nd * dB;
}

// Finish one slot (one wave): the exact theta from the chunk maxima, the ambiguous chunks
// recomputed with it, the merge, mean / population std, the reference's float64 (or float32)
// score arithmetic and the outputs.  parts == nullptr: serial slot (every chunk computed here).
template <int RING>
__device__ void rs_finish(const RsArgs& a, RsSlot* sp, int seg, int T, float theta_s32, const RsPart* parts,
                          const RsLane& cl, const unsigned char* smem, unsigned char* wbuf, int lane) {
    const RsSrc<RING> v = rs_src<RING>(rs_view<RING>(a, seg));
    const int nch = (T + kRsFrames - 1) / kRsFrames;
    const double theta_s = (double)theta_s32;
    double mx = -INFINITY;
    int fl = 0;
    RsAcc acc;
    double pv[7];
    if (parts) {   // lane c reads chunk c's max and flags: one memory round trip per 64 chunks
        for (int c0 = 0; c0 < nch; c0 += 64) {
            double m = -INFINITY;
            int f = 0;
            if (c0 + lane < nch) { m = rs_ld(&parts[c0 + lane].mx); f = rs_ld(&parts[c0 + lane].flags); }
            mx = fmax(mx, wave_max_d(m));
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) f |= __shfl_xor(f, o, 64);
            fl |= f;
        }
    } else {   // serial: a first pass with theta_s, merged as it goes
        for (int c = 0; c < nch; ++c) {
            double m;
            int n, f;
            rs_chunk(v, T, c, theta_s, kRsWindow, cl, smem, wbuf, lane, pv, m, n, f);
            mx = fmax(mx, m);
            fl |= f;
            rs_merge(acc, pv, n);
        }
    }
    const double theta = mx - kRsTopDb;
    const bool nan_in = (fl & 2) != 0;
    const bool redo_all = !(fabs(theta - theta_s) <= kRsWindow);
    if (lane == 0 && parts) { EWK_RS_ADD(6, redo_all); EWK_RS_ADD(7, nch); }
    if (lane == 0 && !nan_in && theta == theta) EWK_RS_MAX(14, fmin(fabs(theta - theta_s), 1e9) * 1e9);   // (1e-9 dB units)
    if (!nan_in && (parts || redo_all || (fl & 1))) {
        if (!parts) acc = RsAcc();
        // the part records are read one chunk ahead of their merge (uncached memory: a round
        // trip each), in chunk order
        double nx[7];
        int nn = 0, nfl = 0;
        auto fetch = [&](int c) {
            if (parts && c < nch) {
                nn = rs_ld(&parts[c].n);
                nfl = rs_ld(&parts[c].flags);
                if (lane < NMFCC) {
#pragma unroll
                    for (int q = 0; q < 7; ++q) nx[q] = rs_ld(&parts[c].v[q * NMFCC + lane]);
                }
            }
        };
        fetch(0);
        for (int c = 0; c < nch; ++c) {
            int n = nn;
            const int cfl = nfl;
#pragma unroll
            for (int q = 0; q < 7; ++q) pv[q] = nx[q];
            fetch(c + 1);
            if (!parts || redo_all || (cfl & 1)) {   // classification at the exact theta
                double m;
                int f;
                if (lane == 0 && parts) EWK_RS_ADD(8, 1);
                rs_chunk(v, T, c, theta, -1.0, cl, smem, wbuf, lane, pv, m, n, f);
            }
            rs_merge(acc, pv, n);
        }
    }
    double mean = 0.0, sd = 0.0;
    if (lane < NMFCC) {
        const double Td = (double)T;
        const double S1 = fma(theta, acc.P1b, acc.P1a);
        const double S2 = acc.P2a + theta * acc.P2b + theta * theta * acc.P2c;
        mean = fma(theta, acc.rB0, acc.rA0) + S1 / Td;
        double var = (S2 - S1 * S1 / Td) / Td;
        sd = sqrt(var > 0.0 ? var : 0.0);
        if (nan_in) { mean = __builtin_nan(""); sd = __builtin_nan(""); }
        if (a.out_mean64) {
            a.out_mean64[(int64_t)seg * NMFCC + lane] = mean;
            a.out_std64[(int64_t)seg * NMFCC + lane] = sd;
        }
    }
    double* st = reinterpret_cast<double*>(wbuf + RS_BUF);
    if (lane < NMFCC) { st[lane] = mean; st[NMFCC + lane] = sd; }
    wave_sync();
    if (lane == 0) {
        if (a.has_template) {
            double score;
            if (a.cand_f32) {
                float c32[2 * NMFCC];
                for (int i = 0; i < 2 * NMFCC; ++i) c32[i] = (float)st[i];
                score = score_f32cand(a.tmpl, a.tmpl + NMFCC, c32, c32 + NMFCC);
            } else {
                score = score_f64cand(a.tmpl, a.tmpl + NMFCC, st, st + NMFCC);
            }
            const int match = score >= a.threshold;
            if (RING) {
                a.events[seg].score = score;
                a.events[seg].match = match;
                a.events[seg].flags |= EWK_EV_RESCORED;
            } else {
                if (a.out_score) a.out_score[seg] = score;
                if (a.out_match) a.out_match[seg] = (uint8_t)match;
            }
        }
    }
    wave_sync();
}

// List segment `seg` (lane 0 of its scoring wave, after its float32 score is written).  Plain
// stores: the list is read by the re-score launch that follows the scorer (stream order).
__device__ __forceinline__ void rs_list(const ScoreArgs& a, int seg, int len, float theta_s) {
    const int s = atomicAdd(&a.rs_ctl[0], 1);
    if (s >= a.rs_cap) return;   // list full: the float32 score stands
    const int T = 1 + len / HOP;
    const int nch = (T + kRsFrames - 1) / kRsFrames;
    int serial = a.list_all, base = 0;   // list_all (every segment): one wave each, no part records
    bool failed = false;
    if (!serial) {
        base = atomicAdd(&a.rs_ctl[1], nch);
        failed = base < 0 || base > a.rs_part_cap - nch;   // part pool full (or the cursor wrapped)
        if (failed) serial = 1;                             // this slot runs serially
    }
    RsSlot* p = a.rs_slots + s;
    p->seg = seg;
    p->T = T;
    p->base = base;
    p->nclaim = serial ? 1 : nch;
    p->done = 0;
    p->theta_s = theta_s;
    p->serial = serial;
    if (serial) {
        a.rs_serial[atomicAdd(&a.rs_ctl[2], 1)] = s;
        if (failed && base >= 0)   // the reserved records inside the pool: nobody's chunks
            for (int c = base; c < min(base + nch, a.rs_part_cap); ++c) a.rs_parts[c].slot = -1;
    } else {
        for (int c = 0; c < nch; ++c) a.rs_parts[base + c].slot = s;
    }
}

// Lane 0: claim the next unit -- a chunk (part record g of the reserved range, one atomic),
// then, once every chunk is taken, a whole serial slot.
struct RsClaim {
    int slot = -1, unit = 0, seg = 0, T = 0, base = 0, serial = 0, nclaim = 0;
    float theta_s = 0.0f;
};
// A wave's first claim of the launch is part record (its index in the grid) -- no atomic: one
// device-scope fetch-add address serves ~1 claim per 11 ns and the launch's 2,048 waves would
// all claim at once (~23 us for the last; scripts/probes/atomic_probe.hip) -- the rest come
// from the cursor, offset by the grid's waves.
__device__ __forceinline__ int rs_grid_waves() { return (int)gridDim.x * RS_NW; }
__device__ __forceinline__ RsClaim rs_claim(const RsArgs& a, int n_parts, int n_serial, int& first) {
    RsClaim r;
    int s = -1;
    for (;;) {
        int g;
        if (first >= 0) {
            g = first;
            first = -1;
        } else {
            g = rs_grid_waves() + __hip_atomic_fetch_add(&a.rs_ctl[4], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        EWK_RS_ADD(12, 1);
        if (g >= n_parts) break;
        s = a.rs_parts[g].slot;
        if (s >= 0) {
            const RsSlot* p = a.rs_slots + s;
            r.unit = g - p->base;
            break;
        }
    }
    if (s < 0) {   // every chunk is taken: the serial slots
        const int q = __hip_atomic_fetch_add(&a.rs_ctl[5], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (q >= n_serial) return r;
        s = a.rs_serial[q];
        r.unit = 0;
    }
    const RsSlot* p = a.rs_slots + s;
    r.slot = s; r.nclaim = p->nclaim;
    r.seg = p->seg; r.T = p->T; r.base = p->base; r.serial = p->serial; r.theta_s = p->theta_s;
    return r;
}

// The list sizes of this launch (fixed while it runs: the lister was the previous launch).
__device__ __forceinline__ int rs_n_parts(const RsArgs& a) {
    return min(__hip_atomic_load(&a.rs_ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), a.rs_part_cap);
}
__device__ __forceinline__ int rs_n_serial(const RsArgs& a) {
    return min(__hip_atomic_load(&a.rs_ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), a.rs_cap);
}

// One wave drains the list until nothing is claimable; true if it finished a slot.
// first_claim: the launch's main drain (a wave's own part record first); the last workgroup's
// second drain takes cursor claims only.
template <int RING>
__device__ __attribute__((noinline)) bool rs_drain(const RsArgs& a, unsigned char* smem, int wave, int lane,
                                                   bool first_claim) {
    unsigned char* wbuf = smem + RS_WAVES + wave * RS_WAVE_BYTES;
    if (lane == 0) EWK_RS_ADD(0, 1);   // waves that drain
#ifdef EWK_RS_TIMING
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#endif
    RsLane cl;
    bool have_lane = false, finished = false;
    const int n_parts = rs_n_parts(a), n_serial = rs_n_serial(a);
    int first = first_claim ? (int)blockIdx.x * RS_NW + wave : -1;   // (lane 0's)
    for (;;) {
        RsClaim c;
        if (lane == 0) c = rs_claim(a, n_parts, n_serial, first);
        const int slot = __shfl(c.slot, 0, 64);
        if (slot < 0) break;
        const int unit = __shfl(c.unit, 0, 64), seg = __shfl(c.seg, 0, 64), T = __shfl(c.T, 0, 64);
        const int base = __shfl(c.base, 0, 64), serial = __shfl(c.serial, 0, 64), nclaim = __shfl(c.nclaim, 0, 64);
        const float theta_s = __shfl(c.theta_s, 0, 64);
        if (!have_lane) { rs_lane_init(a.tab64, lane, cl); have_lane = true; }
        RsSlot* sp = a.rs_slots + slot;
        if (serial) {
            if (lane == 0) EWK_RS_ADD(5, 1);
            rs_finish<RING>(a, sp, seg, T, theta_s, nullptr, cl, smem, wbuf, lane);
            finished = true;
            continue;
        }
#ifdef EWK_RS_TIMING
        const unsigned long long c0 = __builtin_amdgcn_s_memrealtime();
#endif
        const RsSrc<RING> v = rs_src<RING>(rs_view<RING>(a, seg));
        double pv[7], mx;
        int n, flags;
        rs_chunk(v, T, unit, (double)theta_s, kRsWindow, cl, smem, wbuf, lane, pv, mx, n, flags);
        RsPart* pp = a.rs_parts + base + unit;
        if (lane < NMFCC) {
#pragma unroll
            for (int q = 0; q < 7; ++q) rs_st(&pp->v[q * NMFCC + lane], pv[q]);
        }
        if (lane == 0) { rs_st(&pp->mx, mx); rs_st(&pp->n, n); rs_st(&pp->flags, flags); }
#ifdef EWK_RS_TIMING
        if (lane == 0) { EWK_RS_ADD(1, 1); EWK_RS_ADD(2, __builtin_amdgcn_s_memrealtime() - c0); }
#endif
        // the part record's (agent-coherent) stores are acknowledged before the count: no L2
        // write-back (a release would add buffer_wbl2 sc1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int last = 0;
        if (lane == 0) last = __hip_atomic_fetch_add(&sp->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nclaim - 1;
        if (__shfl(last, 0, 64)) {
            // Acquire (agent scope, lowered to buffer_inv sc1): the other waves' part records are
            // read through this CU's vector L1, which may still hold lines of the same records
            // from an earlier tick; the invalidate drops them.  The writers' side needs no
            // release: records are uncached memory (stores complete at memory, s_waitcnt
            // vmcnt(0) above orders them before the count).
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#ifdef EWK_RS_TIMING
            const unsigned long long f0 = __builtin_amdgcn_s_memrealtime();
#endif
            rs_finish<RING>(a, sp, seg, T, theta_s, a.rs_parts + base, cl, smem, wbuf, lane);
#ifdef EWK_RS_TIMING
            if (lane == 0) { EWK_RS_ADD(3, 1); EWK_RS_ADD(4, __builtin_amdgcn_s_memrealtime() - f0); }
#endif
            finished = true;
        }
    }
#ifdef EWK_RS_TIMING
    if (lane == 0) {
        const unsigned long long d = __builtin_amdgcn_s_memrealtime() - r0;
        (void)atomicMax(&g_rs_dbg[10], d);
        EWK_RS_ADD(11, d);
    }
#endif
    return finished;
}

// Anything listed that no wave has taken yet (thread 0)?
// first_claim: this workgroup's waves have not drained yet (their own part records count).
__device__ __forceinline__ bool rs_pending(const RsArgs& a, bool first_claim) {
    const int n_parts = rs_n_parts(a);
    return (first_claim && (int)blockIdx.x * RS_NW < n_parts) ||
           rs_grid_waves() + __hip_atomic_load(&a.rs_ctl[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n_parts ||
           __hip_atomic_load(&a.rs_ctl[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < rs_n_serial(a);
}

// The end of a scoring pass (one workgroup, after the list is drained): re-arm the counters
// for the next launch, advance the event watermark (ring mode) and write the poll mirror.
// pre (empty launch, thread 0 of workgroup 0): the event count and the bank's counters, loaded
// at the launch's start together with the list count (three dependent round trips -> one); with
// no re-score write to publish, the counters need no fence (the launch's end releases them).
struct TickPre {
    int32_t n_events;
    uint4 c;
};
template <int RING>
__device__ void tick_end(const ScoreArgs& a, const TickPre* pre = nullptr) {
    if (threadIdx.x == 0) {
        if (RING) *a.adv_ev_base = pre ? pre->n_events : *a.n_events;
        *a.work = 0;
#pragma unroll
        for (int i = 0; i < kRsCtl; ++i) a.rs_ctl[i] = 0;
        // (no fence: every workgroup of this launch has counted out, so the readers of these
        // counters are later launches, and the launch's end releases them)
    }
    if (RING && a.mirror) {   // poll mirror: the bank's counters and first events -> pinned host memory
        __syncthreads();   // this workgroup's own re-score writes (its second drain) are done
        const volatile int32_t* vc = a.evc;
        const uint4 c = pre ? pre->c : make_uint4((uint32_t)vc[0], (uint32_t)vc[1], (uint32_t)vc[2], (uint32_t)vc[3]);
        const int32_t n = (int32_t)min(min((uint32_t)(c.x - (uint32_t)a.ev_base0), (uint32_t)a.n_seg),
                                       (uint32_t)a.mirror_chunk);
        if (threadIdx.x == 0) *reinterpret_cast<uint4*>(a.mirror) = c;
        const uint4* src = reinterpret_cast<const uint4*>(a.events);
        uint4* dst = reinterpret_cast<uint4*>(a.mirror + 16);
        const int nq = n * (int)(sizeof(ewk_event) / 16);
        // every workgroup that wrote a score released it before its arrival count, and the
        // fence after the last arrival acquired them for this workgroup (the scorer's own
        // scores come from the previous launch)
        for (int i = threadIdx.x; i < nq; i += blockDim.x) dst[i] = src[i];
    }
}

// Every workgroup of a re-score launch (k_rescore_linear / k_rescore_ring, right after the
// scorer): drain the list, count out; the last workgroup out drains what is left and ends the
// pass (tick_end).  A workgroup that finished a slot (wrote a score the poll mirror copies)
// publishes with a device-scope release before its arrival count.  With nothing listed (most
// streaming ticks) workgroup 0 ends the pass alone and the others leave at once.
template <int RING>
__device__ void score_tail(const ScoreArgs& a, unsigned char* smem) {
    // [0] last, [1 + wave] finished a slot, [1 + RS_NW] pending, [2 + RS_NW] slots listed (its own
    // slot: wave 0 rewrites [1 + RS_NW] before the other waves need have read this count)
    int* flag = reinterpret_cast<int*>(smem + RS_FLAGS);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const RsArgs ra = rs_args(a);
    TickPre* pre = reinterpret_cast<TickPre*>(smem + RS_PRE);
    if (threadIdx.x == 0) {
        // (workgroup 0 also requests what the tick end needs, in the same round trip)
        int32_t ne = 0;
        uint4 c = make_uint4(0, 0, 0, 0);
        if (RING && blockIdx.x == 0) {
            ne = *a.n_events;
            if (a.mirror) {
                const volatile int32_t* vc = a.evc;
                c = make_uint4((uint32_t)vc[0], (uint32_t)vc[1], (uint32_t)vc[2], (uint32_t)vc[3]);
            }
        }
        flag[2 + RS_NW] = a.rs_slots ? __hip_atomic_load(&a.rs_ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        pre->n_events = ne;
        pre->c = c;
    }
    __syncthreads();
    if (flag[2 + RS_NW] == 0) {   // nothing listed: the list stays empty for this launch
        if (blockIdx.x == 0) tick_end<RING>(a, RING ? pre : nullptr);
        return;
    }
    bool loaded = false, finished = false;
    if (threadIdx.x == 0) flag[1 + RS_NW] = rs_pending(ra, true);
    __syncthreads();
    if (flag[1 + RS_NW]) {
        if (threadIdx.x == 0) EWK_RS_ADD(9, 1);   // workgroups that drain
        rs_load_tables(a.tab64, smem);
        __syncthreads();
        loaded = true;
        finished = rs_drain<RING>(ra, smem, wave, lane, true);
    }
    if (lane == 0) flag[1 + wave] = finished;
    // Hand-off of the finished slots' scores (rs_finish: plain stores) to the last workgroup's
    // poll-mirror copy (tick_end), MI355X_MICROARCH.md "Valid forms": every storing wave's
    // stores are acknowledged before the barrier, thread 0 releases (L2 write-back) and WAITS
    // for the write-back before its count -- the compiler drops that wait after buffer_wbl2
    // when the scoreboard looks empty (round 5's ISA: `buffer_wbl2 sc1; buffer_inv sc1;
    // global_atomic_add`, so the count could overtake the write-back and the mirror copy read
    // a re-scored event's float32 score) -- and each wave of the last workgroup acquires.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int any = 0;
        for (int w = 0; w < RS_NW; ++w) any |= flag[1 + w];
        if (any) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        flag[0] = __hip_atomic_fetch_add(&a.rs_ctl[3], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                  (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!flag[0]) return;
#ifdef EWK_RS_TIMING
    const unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
#endif
    // acquire what every other workgroup released before its count (each wave: its own loads)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the last workgroup: every other has drained and counted out
    if (threadIdx.x == 0) flag[1 + RS_NW] = rs_pending(ra, false);
    __syncthreads();
    if (flag[1 + RS_NW]) {
        if (!loaded) {
            rs_load_tables(a.tab64, smem);
            __syncthreads();
        }
        rs_drain<RING>(ra, smem, wave, lane, false);
    }
    __syncthreads();
    tick_end<RING>(a);
#ifdef EWK_RS_TIMING
    if (threadIdx.x == 0) EWK_RS_ADD(13, __builtin_amdgcn_s_memrealtime() - t_last);
#endif
}

// Linear batches: the list of a k_score_f32<0> launch is drained by this launch right after
// it (stream-ordered: the list is complete), so the batch scorer itself makes no call and keeps
// its register allocation; every workgroup drains, the last one out resets the counters.
__global__ __launch_bounds__(64 * RS_NW, 1) void k_rescore_linear(ScoreArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    score_tail<0>(a, smem);
}

// Ring mode (a streaming tick): the same, right after the tick's scorer launch.  Every listed
// segment is known when it starts, so all its workgroups drain from the first cycle (inside the
// scorer, workgroups that ran out of float32 work before the last listings counted out, and the
// last one drained the rest alone: 0.07 -> 0.78 ms per 8,192-stream tick); its last workgroup
// ends the tick (counters, event watermark, poll mirror).
template <int RING>
__global__ __launch_bounds__(64 * RS_NW, 1) void k_rescore_ring(ScoreArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    score_tail<RING>(a, smem);
}
