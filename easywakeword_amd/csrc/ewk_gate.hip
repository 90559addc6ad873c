// ewk_gate.hip -- level-1 gate for many concurrent streams on gfx950.
//
// One wave per stream, streams independent (no cross-wave sync).  Per tick:
//   a1  ring ingest           SoundBuffer._add_sound_to_buffer  wakeword.py:454-470
//   a2  block RMS + pct25     SoundBuffer._adjust_silence_threshold  :472-486
//   a3  last-0.1 s RMS test   SoundBuffer.is_silent / return_last_n_seconds  :488-513
//   a4  timing FSM            WakeWord._detect_word  :1048-1098
//   a5  segment cut + queue   WakeWord._detect_word  :1100-1118
// All comparisons are float64 and bit-identical to the reference's numpy
// arithmetic: squares of float32 samples are exact in float64, sums follow
// numpy's pairwise order (chunks of 8192, 8-accumulator leaves of <= 128,
// split at n2 = n/2 - (n/2)%8; the tree is flattened once on the host and
// evaluated level by level across the wave), the percentile follows numpy
// 2.2's "linear" method (_compute_virtual_index / _lerp), and the clock is
// tick * tick_seconds.
//
// Incremental state per stream (the reference recomputes everything per tick):
//   * block_rms[b]: RMS of physical block b, refreshed only for the blocks the
//     tick's samples overlap (the other blocks hold the same samples, hence the
//     same value);
//   * sorted_rms: the same multiset kept sorted (one remove + one insert per
//     refreshed block, wave-parallel), so np.percentile(all_rms, 25) is a lookup
//     of the two order statistics it interpolates;
//   * the tick's samples are staged in LDS, so the refreshed block and the last
//     0.1 s window are summed without re-reading the ring; when the window is the
//     refreshed block (aligned ticks, n_last == block) its sum is reused.
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "ewk_gate.h"

// float64 parity with numpy requires un-fused multiply/add (e.g. the percentile lerp)
#pragma clang fp contract(off)

namespace ewk {

// ---- host: flatten numpy's pairwise recursion for one chunk --------------------
static int split_point(int n) {
    int n2 = n / 2;
    n2 -= n2 % 8;
    return n2;
}

void build_pw_tree(int n, PwTree* t) {
    memset(t, 0, sizeof(*t));
    t->n = n;
    if (n <= 0) return;
    struct Node { int a, b, h; };   // children as tagged ids: >= 0 leaf, < 0 internal (-1 - index)
    std::vector<Node> inner;
    int nleaf = 0;
    // returns tagged id and height
    struct R { int id, h; };
    auto rec = [&](auto&& self, int s, int m) -> R {
        if (m <= 128) {
            t->leaf_start[nleaf] = (int16_t)s;
            t->leaf_len[nleaf] = (int16_t)m;
            return R{nleaf++, 0};
        }
        const int n2 = split_point(m);
        const R a = self(self, s, n2);
        const R b = self(self, s + n2, m - n2);
        inner.push_back(Node{a.id, b.id, std::max(a.h, b.h) + 1});
        return R{-1 - (int)(inner.size() - 1), std::max(a.h, b.h) + 1};
    };
    rec(rec, 0, n);
    t->n_leaves = nleaf;
    // order internal nodes by height (children always lower), keep creation order within a level
    std::vector<int> order(inner.size());
    for (size_t i = 0; i < inner.size(); ++i) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return inner[x].h < inner[y].h; });
    std::vector<int> pos(inner.size());
    for (size_t k = 0; k < order.size(); ++k) pos[order[k]] = (int)k;
    auto node_id = [&](int tag) { return tag >= 0 ? tag : nleaf + pos[-1 - tag]; };
    int levels = 0;
    for (size_t k = 0; k < order.size(); ++k) {
        const Node& nd = inner[order[k]];
        t->left[k] = (int16_t)node_id(nd.a);
        t->right[k] = (int16_t)node_id(nd.b);
        t->level_end[nd.h - 1] = (int16_t)(k + 1);
        levels = nd.h;
    }
    t->n_levels = levels;
    // balanced: every level pairs the previous level's nodes in order (node 2k with 2k + 1),
    // there are 2^d <= 16 leaves and each has >= 8 elements (1,600: 16 leaves of 96 / 104)
    bool bal = nleaf >= 1 && nleaf <= 16 && (nleaf & (nleaf - 1)) == 0;
    for (int l = 0; bal && l < nleaf; ++l) bal = t->leaf_len[l] >= 8;
    int first = 0, cnt = nleaf, k = 0;   // level h's nodes: ids [first, first + cnt)
    for (int h = 0; bal && h < levels; ++h) {
        for (int q = 0; bal && q < cnt / 2; ++q, ++k)
            bal = t->left[k] == first + 2 * q && t->right[k] == first + 2 * q + 1 && k < t->level_end[h];
        bal = bal && k == t->level_end[h];
        first = h == 0 ? nleaf : first + cnt;
        cnt /= 2;
    }
    t->balanced = bal && cnt == 1;
}

// per-wave LDS bytes of k_gate_ticks: tree values / sort scratch, then the stage (16-B aligned)
__host__ __device__ inline size_t gate_wave_lds(int32_t val_len, int32_t stage, int stage_es) {
    return (((size_t)val_len * 8 + 15) & ~(size_t)15) + (((size_t)stage * stage_es + 15) & ~(size_t)15);
}

int gate_stage_len(int block, int64_t n_last) {
    const int64_t m = std::max<int64_t>(block, n_last);
    if (m > 4096) return 0;              // long callbacks: sum straight from the ring
    return (int)((m + 3) & ~3);
}

// ---- device ---------------------------------------------------------------------
// The lane index through an empty asm: values derived from it (per-lane offsets) are then
// computed where they are used instead of being hoisted out of the stream loop and kept live
// (or spilled) across everything in between.
__device__ __forceinline__ int lane_here(int lane) {
    asm volatile("" : "+v"(lane));
    return lane;
}
__device__ __forceinline__ void wave_sync() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// Ring samples are written once per tick and read back only for the few cut segments:
// non-temporal stores keep them from filling the L2 with dirty lines that every launch
// end must write back before the scorer can start.
typedef float f32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nt_store4(float* p, float4 v) {
    f32x4_nt x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4_nt*>(p));
}

struct LdsSrc {
    const float* p;
    __device__ __forceinline__ float operator()(int i) const { return p[i]; }
};

// the int16 stage of the vector int16 path (DMA 3): the PCM16 value / 32768, exactly the float
// the float stage held (half the LDS: five workgroups of four waves fit a CU)
struct LdsSrc16 {
    const int16_t* p;
    __device__ __forceinline__ float operator()(int i) const { return (float)p[i] * (1.0f / 32768.0f); }
};

struct RingSrc {
    const float* ring;
    const int16_t* ring16;   // int16 ring (EWK_RING_I16) when set: value = x / 32768, exact
    int32_t first;   // physical index of element 0
    int32_t R;
    __device__ __forceinline__ float operator()(int i) const {
        int k = first + i;
        if (k >= R) k -= R;
        return ring16 ? (float)ring16[k] * (1.0f / 32768.0f) : ring[k];
    }
};

// Sum of squares of one leaf (n <= 128) exactly as numpy's inner loop.
template <typename Src>
__device__ __forceinline__ double leaf_sumsq(const Src& src, int s, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) { const double x = src(s + i); r += x * x; }
        return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { const double x = src(s + j); r[j] = x * x; }
    int i = 8;
    const int lim = n - (n % 8);
    for (; i < lim; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const double x = src(s + i + j); r[j] += x * x; }
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) { const double x = src(s + i); res += x * x; }
    return res;
}

// DPP / permlane helpers for doubles (wave-uniform control)
template <int CTRL, int BANKS>
__device__ __forceinline__ double dpp_mov_d(double x) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xf, BANKS, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xf, BANKS, false);
    return __hiloint2double(hi, lo);
}
// the value of lane ^ 16 (rows 0 <-> 1, 2 <-> 3) / lane ^ 32 (rows 0, 1 <-> 2, 3)
template <int W>
__device__ __forceinline__ double swap_rows_d(double x, int lane) {
    const uint32_t lo = (uint32_t)__double2loint(x), hi = (uint32_t)__double2hiint(x);
    const auto rl = W == 16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                            : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = W == 16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                            : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    // (vdst, vsrc) = (x, x): the upper half of each pair finds the partner in vdst, the lower in vsrc
    const bool upper = (lane & W) != 0;
    return __hiloint2double((int)(upper ? rh[0] : rh[1]), (int)(upper ? rl[0] : rl[1]));
}

// A balanced chunk (build_pw_tree: 2^d <= 16 leaves of >= 8 elements, paired in order) without LDS:
// lane = leaf % 8 * 8 + j runs accumulator j of leaf (leaf % 8) + 8 s for s = 0, 1 (numpy's
// r[j] += x[i + j]^2, i = 8, 16, ...); the eight accumulators combine as
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) by DPP exchanges (lane ^ 1, ^ 2, 7 - lane
// within eight: every lane of the eight then holds the same bits, a + b == b + a), the tail
// elements are added in order, and the leaves pair in order across lane groups (row_ror:8,
// rows ^ 1, rows ^ 2, then set 0 + set 1) -- numpy's additions, operand for operand.
template <typename Src>
__device__ double tree_sumsq_bal(const Src& src, const PwTree* t, int lane) {
    const int L = t->n_leaves;
    const int j = lane & 7, li = lane >> 3;
    double tot[2] = {0.0, 0.0};
#pragma unroll
    for (int set = 0; set < 2; ++set) {
        if (8 * set >= L) break;   // (wave-uniform)
        const int l = li + 8 * set < L ? li + 8 * set : 0;   // (lanes past the last leaf: a copy of leaf 0, unused)
        const int s0 = t->leaf_start[l], m = t->leaf_len[l], m8 = m - m % 8;
        double r;
        { const double x = src(s0 + j); r = x * x; }
        for (int i = 8; i < m8; i += 8) { const double x = src(s0 + i + j); r += x * x; }
        r = r + dpp_mov_d<0xB1, 0xf>(r);   // quad_perm [1,0,3,2]: lane ^ 1
        r = r + dpp_mov_d<0x4E, 0xf>(r);   // quad_perm [2,3,0,1]: lane ^ 2
        r = r + dpp_mov_d<0x141, 0xf>(r);  // row_half_mirror: 7 - lane within eight
        for (int i = m8; i < m; ++i) { const double x = src(s0 + i); r += x * x; }
        // leaves of this set: pairs (row_ror:8), then rows ^ 1, rows ^ 2
        if (L > 1) r = r + dpp_mov_d<0x128, 0xf>(r);   // row_ror:8
        if (L > 2) r = r + swap_rows_d<16>(r, lane);
        if (L > 4) r = r + swap_rows_d<32>(r, lane);
        tot[set] = r;
    }
    // lane 0 holds its set's sum (for fewer than 8 leaves the rows past them hold copies of leaf
    // 0); for 16 leaves the root adds the two halves in order.  Broadcast: a uniform result.
    const double res = L > 8 ? tot[0] + tot[1] : tot[0];
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(res)),
                            __builtin_amdgcn_readfirstlane(__double2loint(res)));
}

// One chunk (n = t->n elements of src) in numpy's pairwise order, wave-parallel.
// val: per-wave LDS scratch of 10 * n_leaves doubles (node values, then the leaves'
// 8 accumulators).  Each accumulator chain of a leaf runs on its own lane (numpy's
// r[j] += x[i + j]^2, i = 8, 16, ...), a second step combines the eight in numpy's
// order and adds the < 8 tail elements -- the same additions as leaf_sumsq.
// Uniform result.
template <typename Src>
__device__ double tree_sumsq(const Src& src, const PwTree* t, int lane, double* val) {
    if (t->balanced) return tree_sumsq_bal(src, t, lane);   // (the default 1,600-sample block: 16 leaves)
    const int L = t->n_leaves;
    double* acc8 = val + 2 * L;
    for (int q = lane; q < 8 * L; q += 64) {
        const int l = q >> 3, j = q & 7;
        const int s0 = t->leaf_start[l], n = t->leaf_len[l];
        if (n >= 8) {
            double r;
            { const double x = src(s0 + j); r = x * x; }
            const int lim = n - (n % 8);
            for (int i = 8; i < lim; i += 8) { const double x = src(s0 + i + j); r += x * x; }
            acc8[q] = r;
        }
    }
    wave_sync();
    for (int l = lane; l < L; l += 64) {
        const int s0 = t->leaf_start[l], n = t->leaf_len[l];
        double res;
        if (n < 8) {
            res = 0.0;
            for (int i = 0; i < n; ++i) { const double x = src(s0 + i); res += x * x; }
        } else {
            const double* r = acc8 + 8 * l;
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            for (int i = n - (n % 8); i < n; ++i) { const double x = src(s0 + i); res += x * x; }
        }
        val[l] = res;
    }
    wave_sync();
    int b = 0;
    for (int h = 0; h < t->n_levels; ++h) {
        const int e = t->level_end[h];
        for (int k = b + lane; k < e; k += 64) val[L + k] = val[t->left[k]] + val[t->right[k]];
        b = e;
        wave_sync();
    }
    const double r = (L == 1) ? val[0] : val[L + b - 1];   // the root is the last internal node
    wave_sync();
    return r;
}

// np.add.reduce(x**2) over n samples: chunks of 8192 accumulated from 0.0.
template <typename MakeSrc>
__device__ double pw_sumsq(const MakeSrc& make, int n, const PwTree* full, const PwTree* rem, int lane,
                           double* val) {
    double acc = 0.0;
    for (int c0 = 0; c0 < n; c0 += kPwChunk) {
        const int cn = min(kPwChunk, n - c0);
        acc += tree_sumsq(make(c0), cn == kPwChunk ? full : rem, lane, val);   // (full->n == kPwChunk)
    }
    return acc;
}

// First fill: rank-sort v (global, nb values) into dst (global).
__device__ void rank_sort(const double* v, double* dst, int nb, int lane) {
    for (int i = lane; i < nb; i += 64) {
        const double x = v[i];
        int r = 0;
        for (int k = 0; k < nb; ++k) {
            const double y = v[k];
            r += (y < x) || (y == x && k < i);
        }
        dst[r] = x;
    }
}

// src (sorted) with one occurrence of vo replaced by vn -> dst (sorted).
// Returns false when vo is absent (cache inconsistent: caller re-sorts).
__device__ bool sorted_replace(const double* src, double* dst, int nb, double vo, double vn, int lane) {
    int pos = nb;
    for (int i = lane; i < nb; i += 64)
        if (src[i] == vo) { pos = i; break; }
    for (int m = 1; m < 64; m <<= 1) pos = min(pos, __shfl_xor(pos, m, 64));
    if (pos >= nb) return false;
    int cnt = 0;
    for (int i = lane; i < nb; i += 64) cnt += (i != pos && src[i] < vn) ? 1 : 0;
    for (int m = 1; m < 64; m <<= 1) cnt += __shfl_xor(cnt, m, 64);
    for (int i = lane; i < nb; i += 64) {
        if (i == pos) continue;
        const int i1 = i < pos ? i : i - 1;
        dst[i1 < cnt ? i1 : i1 + 1] = src[i];
    }
    if (lane == 0) dst[cnt] = vn;
    return true;
}

// numpy.percentile(v, 25) ("linear") from the sorted copy.
__device__ __forceinline__ double percentile25_sorted(const double* sorted, int nb) {
    // virtual index = n*q + (alpha + q*(1-alpha-beta)) - 1, alpha = beta = 1, q = 0.25
    const double q = 0.25;
    const double vi = (double)nb * q + (1.0 + q * (1.0 - 1.0 - 1.0)) - 1.0;
    const double prevd = floor(vi);
    int prev = (int)prevd, next = prev + 1;
    if (vi >= (double)(nb - 1)) { prev = nb - 1; next = nb - 1; }
    if (vi < 0.0) { prev = 0; next = 0; }
    const double gamma = vi - prevd;
    const double a = sorted[prev], b = sorted[next];
    // numpy _lerp: a + (b-a)*t, replaced by b - (b-a)*(1-t) where t >= 0.5
    const double d = b - a;
    double r = a + d * gamma;
    if (gamma >= 0.5) r = b - d * (1.0 - gamma);
    return r;
}

// the register allocator must allow 4 waves per SIMD (121 VGPRs; 5 spill and run 37 % slower)
#ifndef EWK_GATE_WPE
#define EWK_GATE_WPE 4
#endif
constexpr int kGateWavesPerEU = EWK_GATE_WPE;
// workgroups of 4 waves, one stream per wave up to 524,288 streams, more loop inside the waves.
// (Round 1 capped the grid at one resident wave per slot, 1,024 workgroups, so each wave ran
// its streams in sequence behind the previous stream's final stores; letting the hardware
// refill freed slots with new waves instead took the tick from 11.6 to 9.2 ms at 2 M streams,
// 0.75 to 0.65 ms at 131,072 and 77 to 72 us at 8,192.)
#ifndef EWK_GATE_GRID_MAX
#define EWK_GATE_GRID_MAX 131072
#endif
constexpr int kGateGridMax = EWK_GATE_GRID_MAX;
constexpr int kDma4Chunks = 8;
constexpr int kPcm16Pieces = 4;    // int16 path: ticks of up to 4 * 512 samples in 16-B pieces
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));     // 16-B DMA path: ticks of up to 8 * 256 samples copied to the ring in one batch
constexpr int kIngestLoads = 4;    // tick samples per lane loaded ahead of the ring stores (16: 166 VGPRs, 3 waves/SIMD, 10 % slower)

// ---- register-resident block RMS multiset (n_blocks <= 64 * RB) ------------------
// Element i of a per-stream array lives in lane i % 64, slot i / 64.
template <int RB>
__device__ __forceinline__ double reg_get(const double (&v)[RB], int i) {
    double r = 0.0;
#pragma unroll
    for (int j = 0; j < RB; ++j)
        if ((i >> 6) == j) r = __shfl(v[j], i & 63, 64);
    return r;
}

template <int RB>
__device__ __forceinline__ void reg_set(double (&v)[RB], int i, double x, int lane, uint32_t& dirty) {
#pragma unroll
    for (int j = 0; j < RB; ++j)
        if ((i >> 6) == j && lane == (i & 63)) { v[j] = x; dirty |= 1u << j; }
}

// so (sorted, nb values) with one occurrence of vo replaced by vn, kept sorted: the
// new element d comes from old element d - 1, d or d + 1 (or is vn), so the update is
// two neighbour shuffles.  Returns false when vo is absent (caller re-sorts).
template <int RB>
__device__ bool reg_replace(double (&so)[RB], int nb, double vo, double vn, int lane, uint32_t& dirty) {
    int pos = nb;
#pragma unroll
    for (int j = RB - 1; j >= 0; --j) {
        const unsigned long long m = __ballot(lane + 64 * j < nb && so[j] == vo);
        if (m) pos = 64 * j + __ffsll((long long)m) - 1;
    }
    if (pos >= nb) return false;
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const int i = lane + 64 * j;
        cnt += __popcll(__ballot(i < nb && i != pos && so[j] < vn));
    }
    double prev[RB], next[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const double up = __shfl(so[j], (lane + 63) & 63, 64);    // element d - 1 (lane 0: slot j-1's lane 63)
        const double dn = __shfl(so[j], (lane + 1) & 63, 64);     // element d + 1 (lane 63: slot j+1's lane 0)
        prev[j] = up;
        next[j] = dn;
    }
    // the cross-slot neighbours for lane 0 / lane 63 (wave-uniform shuffles)
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const double tail = j > 0 ? __shfl(so[j - 1], 63, 64) : 0.0;
        const double head = j + 1 < RB ? __shfl(so[j + 1], 0, 64) : 0.0;
        if (lane == 0) prev[j] = tail;
        if (lane == 63) next[j] = head;
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const int d = lane + 64 * j;
        const int i1 = d < cnt ? d : d - 1;
        const int i = i1 < pos ? i1 : i1 + 1;
        const double x = i == d ? so[j] : (i < d ? prev[j] : next[j]);
        so[j] = d == cnt ? vn : x;
        if (d >= min(pos, cnt) && d <= max(pos, cnt)) dirty |= 1u << (RB + j);   // elements that moved
    }
    return true;
}

// First fill / repair: so = sorted copy of gr (stable rank sort through LDS scratch tmp[nb]).
template <int RB>
__device__ void reg_rank_sort(const double (&gr)[RB], double (&so)[RB], int nb, double* tmp, int lane, uint32_t& dirty) {
    dirty |= ((1u << RB) - 1) << RB;
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const int i = lane + 64 * j;
        const double x = gr[j];
        int r = 0;
#pragma unroll
        for (int jj = 0; jj < RB; ++jj)
            for (int kk = 0; kk < 64; ++kk) {
                const int k = 64 * jj + kk;
                const double y = __shfl(gr[jj], kk, 64);
                r += k < nb && ((y < x) || (y == x && k < i));
            }
        if (i < nb) tmp[r] = x;
    }
    wave_sync();
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const int i = lane + 64 * j;
        so[j] = i < nb ? tmp[i] : 0.0;
    }
    wave_sync();
}

// numpy.percentile(v, 25) ("linear") from the register-resident sorted copy.
template <int RB>
__device__ __forceinline__ double reg_percentile25(const double (&so)[RB], int nb) {
    const double q = 0.25;
    const double vi = (double)nb * q + (1.0 + q * (1.0 - 1.0 - 1.0)) - 1.0;
    const double prevd = floor(vi);
    int prev = (int)prevd, next = prev + 1;
    if (vi >= (double)(nb - 1)) { prev = nb - 1; next = nb - 1; }
    if (vi < 0.0) { prev = 0; next = 0; }
    const double gamma = vi - prevd;
    const double a = reg_get(so, prev), b = reg_get(so, next);
    const double d = b - a;
    double r = a + d * gamma;
    if (gamma >= 0.5) r = b - d * (1.0 - gamma);
    return r;
}

// RB > 0: the stream's block RMS array and its sorted copy live in registers for the
// whole launch (RB slots per lane, n_blocks <= 64 * RB): loaded once, updated with
// wave shuffles, stored once -- no dependent global round trips per tick.  RB = 0:
// both stay in global memory (any n_blocks).
template <int RB, int DMA>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kGateWavesPerEU, 8))) void k_gate_ticks(GateArgs g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const PwTree* __restrict__ trees = g.trees;   // read-only, cache-resident
    // persistent over streams: wave w takes streams w, w + waves-in-grid, ...; the next
    // stream's first tick is requested (LDS-DMA) as soon as this stream's last tick has
    // issued its stage reads, so its HBM latency overlaps this stream's FSM and stores
    // (readfirstlane: the compiler then knows the stream, hence its state, is wave-uniform --
    // scalar loads into SGPRs instead of a copy of GateStream in every lane's VGPRs)
    int s = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + wave);
    const int wstride = (int)gridDim.x * 4;
    constexpr int kStageEs = DMA == 3 ? 2 : 4;   // int16 stage for the vector int16 path
    const size_t per_wave = gate_wave_lds(g.val_len, g.stage, kStageEs);
    // The trees of the block and last-window sums (lengths < one 8192 chunk) in LDS: every tree
    // level reads its node indices, and from L1/L2 those dependent loads set the block sum's
    // time (~4 us of a ~14 us stream-tick).  (The full-chunk trees, for callbacks > 8192
    // samples, stay in global memory.)
    PwTree* ltree = reinterpret_cast<PwTree*>(smem + 4 * per_wave);
    {
        static_assert(sizeof(PwTree) % 16 == 0, "trees are copied in 16-B pieces");
        constexpr int kPieces = (int)(sizeof(PwTree) / 16);
        const uint4* src0 = reinterpret_cast<const uint4*>(trees + kTreeBlockRem);
        const uint4* src1 = reinterpret_cast<const uint4*>(trees + kTreeLastRem);
        uint4* dst = reinterpret_cast<uint4*>(ltree);
        for (int i = threadIdx.x; i < 2 * kPieces; i += blockDim.x) dst[i] = i < kPieces ? src0[i] : src1[i - kPieces];
        __syncthreads();
    }
    if (s >= g.n_streams) return;
    unsigned char* w = smem + wave * per_wave;
    double* val = reinterpret_cast<double*>(w);
    float* stage = reinterpret_cast<float*>(w + (((size_t)g.val_len * 8 + 15) & ~(size_t)15));
    int16_t* stage16 = reinterpret_cast<int16_t*>(stage);   // (DMA 3)
    // the staged samples [c0, ...) as a summation source
    auto stage_src = [&](int c0) {
        if constexpr (DMA == 3) return LdsSrc16{stage16 + c0};
        else return LdsSrc{stage + c0};
    };

    const int R = (int)g.ring_len;        // the reference ring: block grid, pointer, fill level
    const int Rs = (int)g.sring_len;      // samples stored per stream (== R unless compact)
    const int fs = g.block;
    const int nb = g.n_blocks;
    const int nl = (int)min<int64_t>(g.n_last, g.ring_len);
    // the first tick's samples are requested before the state: no load waits on another
    float xin[kIngestLoads];
    auto load_chunk = [&](int t, int c0) {
        const int64_t so = (int64_t)s * g.stride + (int64_t)t * g.tick_stride;
#pragma unroll
        for (int m = 0; m < kIngestLoads; ++m) {
            const int i = c0 + lane + 64 * m;
            xin[m] = i < fs ? (g.pcm16 ? (float)__builtin_nontemporal_load(g.pcm16 + so + i) * (1.0f / 32768.0f)
                                       : __builtin_nontemporal_load(g.pcm + so + i)) : 0.0f;
        }
    };
    // DMA == 3 (int16 input, block % 8 == 0, 16-B aligned rows): the tick's samples in 16-B
    // pieces (8 per lane), all in flight at once, widened in registers -- one global round
    // trip per tick like the float32 LDS-DMA path (the 4-sample chunks above take seven)
    u32x4 raw[kPcm16Pieces];
    auto load_vec = [&](int ss, int t) {
        const int16_t* src = g.pcm16 + (int64_t)ss * g.stride + (int64_t)t * g.tick_stride;
        const int ln = lane_here(lane);
#pragma unroll
        for (int c = 0; c < kPcm16Pieces; ++c) {
            const int i0 = 8 * (ln + 64 * c);
            raw[c] = i0 < fs ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + i0)) : u32x4{0, 0, 0, 0};
        }
    };
    // float32 input with the tick staged in LDS: the tick's samples go global -> LDS by
    // LDS-DMA (global_load_lds), all in flight at once with no VGPRs -- one global round
    // trip per tick instead of one per register chunk
    const bool staged = g.stage >= fs && g.stage >= nl;
    constexpr bool dma = DMA == 1 || DMA == 2;   // launch_gate: float32 input, tick and window fit the stage
    auto dma_tick = [&](int ss, int t) {
        const float* src = g.pcm + (int64_t)ss * g.stride + (int64_t)t * g.tick_stride;
        if (DMA == 2) {   // 16-B pieces (1 KiB per wave-instruction): tick rows 16-B aligned, block % 4 == 0
            for (int c0 = 0; c0 < fs; c0 += 256) {
                if (c0 + 4 * lane < fs)
                    __builtin_amdgcn_global_load_lds(src + c0 + 4 * lane,
                                                     (__attribute__((address_space(3))) void*)(stage + c0), 16, 0, 0);
            }
            return;
        }
        for (int c0 = 0; c0 < fs; c0 += 64) {
            if (c0 + lane < fs)
                __builtin_amdgcn_global_load_lds(src + c0 + lane, (__attribute__((address_space(3))) void*)(stage + c0),
                                                 4, 0, 0);
        }
    };
    if (dma) dma_tick(s, 0);
    else if (DMA == 3) load_vec(s, 0);
    else load_chunk(0, 0);
    for (;;) {
    float* ring = g.ring ? g.ring + (int64_t)s * Rs : nullptr;
    int16_t* ring16 = g.ring16 ? g.ring16 + (int64_t)s * Rs : nullptr;   // PCM16 pushes only (host-checked)
    GateStream st = g.st[s];
    double* grms = g.block_rms + (int64_t)s * nb;
    double* sorted2 = g.sorted_rms + (int64_t)s * 2 * nb;
    const PwTree* tbf = trees + kTreeBlockFull;
    const PwTree* tbr = ltree;
    const PwTree* tlf = trees + kTreeLastFull;
    const PwTree* tlr = ltree + 1;
    constexpr int RBn = RB > 0 ? RB : 1;
    double gr[RBn], srt[RBn];
    uint32_t dirty = 0;   // register path: bit j = gr[j] changed, bit RB + j = srt[j] changed (stored back only then)
    if (RB > 0) {   // (this path never double-buffers: sorted_sel stays 0)
#pragma unroll
        for (int j = 0; j < RBn; ++j) {
            const int i = lane + 64 * j;
            gr[j] = i < nb ? grms[i] : 0.0;
            srt[j] = i < nb ? sorted2[i] : 0.0;
        }
    }

    for (int t = 0; t < g.n_ticks; ++t) {
        const int64_t tick = g.tick0 + t + 1;                    // tick being delivered
        const double t_prev = (double)(tick - 1) * g.tick_seconds;
        // start()-mode re-entry (TimeoutError -> _detect_word again), before the sleep
        if (st.started && g.reentry_timeout > 0.0 && t_prev - st.start_time > g.reentry_timeout) {
            st.state = kWaiting;
            st.start_time = t_prev;
            if (st.last_silent) { st.state = kInSilence; st.silence_start = t_prev; }
            st.reentries += 1;
        }
        // ---- a1: ingest `fs` samples at the write pointer (and stage them in LDS)
        const int p0 = st.pointer;
        const int sp0 = st.spos;    // == p0 for the full ring
        // chunks of kIngestLoads loads per lane in flight before any store (the ring may
        // alias the input as far as the compiler knows: a load-store loop serialises them);
        // chunk 0 of this tick was requested before the previous tick's compute
        if (DMA == 2) {   // 16-B ring stores from the stage (ring rows and p0 4-float aligned: no group wraps)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            wave_sync();
#pragma unroll
            for (int h = 0; h < kDma4Chunks; h += 4) {   // batches of 4 (16 VGPRs)
                float4 xv[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 256 * (h + c) + 4 * lane;
                    xv[c] = i < fs ? *reinterpret_cast<const float4*>(stage + i) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = 256 * (h + c) + 4 * lane;
                    if (i < fs) {
                        int k = sp0 + i;
                        if (k >= Rs) k -= Rs;
                        nt_store4(ring + k, xv[c]);
                    }
                }
                if (256 * (h + 4) >= fs) break;
            }
        } else if (dma) {   // this tick's samples landed in the stage: ring stores from LDS
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            wave_sync();
            for (int c0 = 0; c0 < fs; c0 += 64 * kIngestLoads) {
#pragma unroll
                for (int m = 0; m < kIngestLoads; ++m) {
                    const int i = c0 + lane + 64 * m;
                    xin[m] = i < fs ? stage[i] : 0.0f;
                }
#pragma unroll
                for (int m = 0; m < kIngestLoads; ++m) {
                    const int i = c0 + lane + 64 * m;
                    if (i < fs) {   // (float32 input: never an int16 ring)
                        int k = sp0 + i;
                        if (k >= Rs) k -= Rs;
                        ring[k] = xin[m];
                    }
                }
            }
        }
        if (DMA == 3) {   // int16 pieces: ring (int16 as delivered, or widened) and stage stores
            const int ln = lane_here(lane);
#pragma unroll
            for (int c = 0; c < kPcm16Pieces; ++c) {
                const int i0 = 8 * (ln + 64 * c);
                if (i0 < fs) {
                    int k = sp0 + i0;   // 8-sample groups never straddle the wrap (Rs % 8 == 0)
                    if (k >= Rs) k -= Rs;
                    const u32x4 w = raw[c];
                    float v[8];
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        v[2 * h] = (float)(short)(w[h] & 0xffffu) * (1.0f / 32768.0f);
                        v[2 * h + 1] = (float)((int)w[h] >> 16) * (1.0f / 32768.0f);
                    }
                    if (ring16) {
                        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(ring16 + k));
                    } else {
                        nt_store4(ring + k, make_float4(v[0], v[1], v[2], v[3]));
                        nt_store4(ring + k + 4, make_float4(v[4], v[5], v[6], v[7]));
                    }
                    if (staged) *reinterpret_cast<u32x4*>(stage16 + i0) = w;   // the int16 samples as delivered
                }
            }
            if (t + 1 < g.n_ticks) load_vec(s, t + 1);   // next tick's samples, in flight during this tick
        }
        for (int c0 = 0; c0 < ((dma || DMA == 3) ? 0 : fs); c0 += 64 * kIngestLoads) {
            if (c0 > 0) load_chunk(t, c0);
#pragma unroll
            for (int m = 0; m < kIngestLoads; ++m) {
                const int i = c0 + lane + 64 * m;
                if (i < fs) {
                    int k = sp0 + i;
                    if (k >= Rs) k -= Rs;
                    if (ring16) ring16[k] = (int16_t)(xin[m] * 32768.0f);   // the PCM16 value, exactly
                    else ring[k] = xin[m];
                    if (staged) stage[i] = xin[m];
                }
            }
        }
        if (t + 1 < g.n_ticks && !dma && DMA != 3) load_chunk(t + 1, 0);   // next tick's samples, in flight during this tick
        __threadfence_block();
        wave_sync();
        const bool wrapped = p0 + fs > R;
        st.pointer = (int32_t)((p0 + fs) % R);
        st.spos = (int32_t)((sp0 + fs) % Rs);
        st.collected = min(st.collected + (int64_t)fs, (int64_t)R);
        const bool full = st.collected >= R;
        // block sum of the window when it coincides with a refreshed block
        double reuse_sum = 0.0;
        bool have_reuse = false;
        // ---- a2: threshold over the physical blocks (only once the ring is full)
        if (full) {
            auto block_sum = [&](int b) -> double {
                const int a0 = b * fs;
                if (staged && a0 == p0)   // the block is exactly this tick's samples
                    return pw_sumsq(stage_src, fs, tbf, tbr, lane, val);
                // reference-ring position a0 + c0 lives at sample-ring position sp0 + (a0 + c0 - p0)
                // (the identity for the full ring; compact rings only reach this path for
                // blocks written within the last Rs samples)
                return pw_sumsq([&](int c0) {
                    int k = (sp0 + (a0 + c0 - p0)) % Rs;
                    if (k < 0) k += Rs;
                    return RingSrc{ring, ring16, k, Rs};
                }, fs, tbf, tbr, lane, val);
            };
            if (!st.filled && g.compact) {
                // compact ring: every block RMS was kept as its samples arrived (the blocks
                // are whole ticks); the last one is this tick's, then the first sort
                const int b = p0 / fs;
                const double v = sqrt(block_sum(b) / (double)fs);
                if (RB > 0) reg_set(gr, b, v, lane, dirty);
                else if (lane == 0) grms[b] = v;
                __threadfence_block();
                wave_sync();
                if (RB > 0) reg_rank_sort(gr, srt, nb, val, lane, dirty);
                else rank_sort(grms, sorted2, nb, lane);
                st.sorted_sel = 0;
                st.filled = 1;
            } else if (!st.filled) {
                for (int b = 0; b < nb; ++b) {
                    const double sum = block_sum(b);
                    if (RB > 0) reg_set(gr, b, sqrt(sum / (double)fs), lane, dirty);
                    else if (lane == 0) grms[b] = sqrt(sum / (double)fs);
                }
                __threadfence_block();
                wave_sync();
                if (RB > 0) reg_rank_sort(gr, srt, nb, val, lane, dirty);
                else rank_sort(grms, sorted2, nb, lane);
                st.sorted_sel = 0;
                st.filled = 1;
            } else {
                // refresh the physical blocks overlapping the written range [p0, p0+fs) (mod R)
                auto refresh = [&](int a0, int a1) {   // [a0, a1) inside [0, R)
                    const int b0 = a0 / fs;
                    const int b1 = (a1 - 1) / fs;
                    for (int b = b0; b <= b1 && b < nb; ++b) {
                        const double sum = block_sum(b);
                        const double v = sqrt(sum / (double)fs);
                        if (nl == fs && b * fs + fs == (int)st.pointer + (st.pointer == 0 ? R : 0)) {
                            reuse_sum = sum;
                            have_reuse = true;
                        }
                        if (RB > 0) {
                            const double vo = reg_get(gr, b);
                            reg_set(gr, b, v, lane, dirty);
                            if (!reg_replace(srt, nb, vo, v, lane, dirty)) reg_rank_sort(gr, srt, nb, val, lane, dirty);
                            continue;
                        }
                        const double vo = grms[b];
                        if (lane == 0) grms[b] = v;
                        const double* cur = sorted2 + (int64_t)st.sorted_sel * nb;
                        double* nxt = sorted2 + (int64_t)(st.sorted_sel ^ 1) * nb;
                        __threadfence_block();
                        wave_sync();
                        if (!sorted_replace(cur, nxt, nb, vo, v, lane)) {
                            __threadfence_block();
                            wave_sync();
                            rank_sort(grms, nxt, nb, lane);
                        }
                        st.sorted_sel ^= 1;
                        __threadfence_block();
                        wave_sync();
                    }
                };
                if (!wrapped) refresh(p0, p0 + fs);
                else { refresh(p0, R); refresh(0, p0 + fs - R); }
            }
            double p25;
            if (RB > 0) {
                p25 = reg_percentile25(srt, nb);
            } else {
                __threadfence_block();
                wave_sync();
                p25 = percentile25_sorted(sorted2 + (int64_t)st.sorted_sel * nb, nb);
            }
            const double thr = p25 * 1.5;
            // Python max(new, MIN): MIN only if MIN > new
            st.threshold = (g.min_threshold > thr) ? g.min_threshold : thr;
        } else if (g.compact) {
            // filling a compact ring: keep this block's RMS now (its samples will not all
            // be in the sample ring when the reference ring first fills)
            const int b = p0 / fs;
            const double v = sqrt(pw_sumsq(stage_src, fs, tbf, tbr, lane, val) /
                                  (double)fs);
            if (RB > 0) reg_set(gr, b, v, lane, dirty);
            else if (lane == 0) grms[b] = v;
        }
        // ---- a3: is_silent(): RMS of the last n_last samples < threshold
        bool silent = true;
        if (nl > 0) {
            double sum;
            if (have_reuse) {
                sum = reuse_sum;
            } else if (staged && nl <= fs) {   // the window lies in this tick's samples
                sum = pw_sumsq([&](int c0) { return stage_src(fs - nl + c0); }, nl, tlf, tlr, lane, val);
            } else {
                int first = st.spos - nl;
                if (first < 0) first += Rs;
                sum = pw_sumsq([&](int c0) {
                    int f = first + c0;
                    if (f >= Rs) f -= Rs;
                    return RingSrc{ring, ring16, f, Rs};
                }, nl, tlf, tlr, lane, val);
            }
            const double rms = sqrt(sum / (double)nl);
            st.last_rms = rms;
            silent = rms < st.threshold;
        }
        if (dma && t + 1 < g.n_ticks) {   // the stage's last reader (a3) has issued its reads
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            dma_tick(s, t + 1);
        } else if (dma && s + wstride < g.n_streams) {   // last tick: the next stream's first
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            dma_tick(s + wstride, 0);
        }
        st.last_silent = silent;
        st.tick = tick;
        const double now = (double)tick * g.tick_seconds;
        // ---- a4/a5: detector
        if (!st.started) {
            if (full) {   // _wait_for_buffer returned: _detect_word entry check
                st.started = 1;
                st.state = kWaiting;
                st.start_time = now;
                if (silent) { st.state = kInSilence; st.silence_start = now; }
            }
            continue;
        }
        {   // wave-uniform FSM (every lane holds the same state): no divergent branch, no broadcast
            switch (st.state) {
            case kWaiting:
                if (silent) { st.state = kInSilence; st.silence_start = now; }
                break;
            case kInSilence:
                if (!silent) {
                    if (now - st.silence_start >= g.pre_speech_silence) { st.state = kInSound; st.sound_start = now; }
                    else st.state = kWaiting;
                }
                break;
            case kInSound: {
                const double d = now - st.sound_start;
                if (!silent) {
                    if (d > g.speech_duration_max) st.state = kWaiting;
                } else {
                    if (g.speech_duration_min <= d && d <= g.speech_duration_max) {
                        st.state = kAfterSound;
                        st.sound_end = now;
                    } else st.state = kWaiting;
                }
                break;
            }
            case kAfterSound:
                if (silent) {
                    if (now - st.sound_end >= g.post_speech_silence) {
                        const double xs = st.sound_start - now - g.padding;
                        const double xe = st.sound_end - now + g.padding;
                        int64_t nreq = (int64_t)(fabs(xs) * (double)g.sample_rate);
                        if (nreq > R) nreq = R;
                        const int64_t e = (int64_t)(fabs(xe) * (double)g.sample_rate);
                        int64_t stop = nreq - e;   // python a[:len-e]
                        if (stop < 0) { stop += nreq; if (stop < 0) stop = 0; }
                        if (stop > nreq) stop = nreq;
                        // (the host sizes a compact ring for the longest possible request)
                        int64_t start = (int64_t)st.spos - nreq;
                        if (start < 0) start += Rs;
                        ewk_event ev;
                        ev.stream = s;
                        ev.length = (int32_t)stop;
                        ev.tick = tick;
                        ev.ring_start = start;
                        ev.time = now;
                        ev.score = __builtin_nan("");
                        ev.match = 0;
                        ev.flags = ((double)stop / (double)g.sample_rate > g.max_segment_seconds) ? EWK_EV_SKIPPED : 0;
                        if (lane == 0) {
                            const uint32_t slot = (uint32_t)atomicAdd(g.ev_count, 1) - (uint32_t)g.ev_base0;
                            if (slot < (uint32_t)g.ev_cap) g.events[slot] = ev;
                            else atomicAdd(g.ev_dropped, 1);
                        }
                        st.state = kWaiting;
                    }
                } else st.state = kWaiting;
                break;
            }
        }
    }
    if (RB > 0 && (st.filled || g.compact)) {   // only the elements this launch changed (one block RMS per tick)
#pragma unroll
        for (int j = 0; j < RBn; ++j) {
            const int i = lane + 64 * j;
            if (i < nb && (dirty & (1u << j))) grms[i] = gr[j];
            if (i < nb && (dirty & (1u << (RB + j)))) sorted2[i] = srt[j];
        }
    }
    if (lane == 0) g.st[s] = st;
    s += wstride;
    if (s >= g.n_streams) break;
    if (DMA == 3) load_vec(s, 0);
    else if (!dma) load_chunk(0, 0);
    }
}

// _detect_word entry (wakeword.py:1048-1057) for streams whose detection runs: state from
// the current is_silent(), start_time = now.  Streams still filling their ring are left
// alone (their entry happens in k_gate_ticks when the ring first fills).
__global__ void k_reenter(GateStream* st, int32_t first, int32_t n, double tick_seconds) {
    const int i = first + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= first + n) return;
    GateStream s = st[i];
    if (!s.started) return;
    const double now = (double)s.tick * tick_seconds;
    s.state = s.last_silent ? kInSilence : kWaiting;
    if (s.last_silent) s.silence_start = now;
    s.start_time = now;
    st[i] = s;
}

// Ring initialisation (ewk_reset_streams).  Round 6's recording build caught the ring scorer
// reading four 128-B lines of ZEROS -- the ring's initial fill -- where the gate had written
// samples twice since ("The ring-path miss recurred"); the fill used
// hipMemsetAsync.  Here every line is written by an agent-scope store (global_store sc1:
// performed at memory, not kept in the XCD's L2), 8 B per lane.
__global__ void k_ring_zero(uint64_t* p, size_t n8) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x)
        __hip_atomic_store(p + i, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
hipError_t launch_ring_zero(void* p, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    if (bytes % 8 || ((uintptr_t)p & 7)) return hipErrorInvalidValue;
    const size_t n8 = bytes / 8;
    const unsigned grid = (unsigned)std::min<size_t>(4096, (n8 + 255) / 256);
    hipLaunchKernelGGL(k_ring_zero, dim3(grid), dim3(256), 0, s, static_cast<uint64_t*>(p), n8);
    return hipGetLastError();
}

hipError_t launch_reenter(GateStream* st, int32_t first, int32_t n, double tick_seconds, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_reenter, dim3((n + 255) / 256), dim3(256), 0, s, st, first, n, tick_seconds);
    return hipGetLastError();
}

int gate_val_len(const PwTree* trees_host, int n_blocks) {
    int m = 0;
    for (int k = 0; k < kNumTrees; ++k) m = std::max(m, 10 * trees_host[k].n_leaves);
    if (n_blocks <= 64 * kGateRegMax) m = std::max(m, n_blocks);   // register path's rank-sort scratch
    return std::max(2, (m + 1) & ~1);
}

hipError_t launch_gate(const GateArgs& g, hipStream_t s) {
    if (g.n_streams <= 0 || g.n_ticks <= 0) return hipSuccess;
    // one wave per stream (the hardware refills freed slots), up to kGateGridMax workgroups
    const int grid = std::min((g.n_streams + 3) / 4, kGateGridMax);
    // (the int16 vector path stages int16; every other path float)
    const int64_t nl = std::min<int64_t>(g.n_last, g.ring_len);
    const bool dma = g.pcm16 == nullptr && g.stage >= g.block && g.stage >= nl;
    // 16-B pieces: every tick row 16-B aligned, whole 4-sample groups that never straddle the ring wrap
    const bool dma4 = dma && g.block % 4 == 0 && g.block <= 256 * kDma4Chunks &&
                      g.stride % 4 == 0 && g.tick_stride % 4 == 0 && g.ring_len % 4 == 0 && g.sring_len % 4 == 0 &&
                      ((uintptr_t)g.pcm & 15) == 0;
    // int16 input in 16-B pieces: rows 16-B aligned, whole 8-sample groups
    const bool vec16 = g.pcm16 != nullptr && g.block % 8 == 0 && g.block <= 512 * kPcm16Pieces &&
                       g.stride % 8 == 0 && g.tick_stride % 8 == 0 && g.sring_len % 8 == 0 &&
                       ((uintptr_t)g.pcm16 & 15) == 0;
    // the DMA 3 instantiations (and only they) stage int16
    const bool i16stage = vec16 && !dma4 && g.n_blocks <= 64 * kGateRegMax;
    const size_t lds = 4 * gate_wave_lds(g.val_len, g.stage, i16stage ? 2 : 4) +
                       2 * sizeof(PwTree);   // + the two sub-chunk trees (k_gate_ticks)
    if (g.n_blocks <= 128) {
        if (dma4) hipLaunchKernelGGL((k_gate_ticks<2, 2>), dim3(grid), dim3(256), lds, s, g);
        else if (vec16) hipLaunchKernelGGL((k_gate_ticks<2, 3>), dim3(grid), dim3(256), lds, s, g);
        else if (dma) hipLaunchKernelGGL((k_gate_ticks<2, 1>), dim3(grid), dim3(256), lds, s, g);
        else hipLaunchKernelGGL((k_gate_ticks<2, 0>), dim3(grid), dim3(256), lds, s, g);
    } else if (g.n_blocks <= 64 * kGateRegMax) {
        if (dma4) hipLaunchKernelGGL((k_gate_ticks<kGateRegMax, 2>), dim3(grid), dim3(256), lds, s, g);
        else if (vec16) hipLaunchKernelGGL((k_gate_ticks<kGateRegMax, 3>), dim3(grid), dim3(256), lds, s, g);
        else if (dma) hipLaunchKernelGGL((k_gate_ticks<kGateRegMax, 1>), dim3(grid), dim3(256), lds, s, g);
        else hipLaunchKernelGGL((k_gate_ticks<kGateRegMax, 0>), dim3(grid), dim3(256), lds, s, g);
    } else {
        hipLaunchKernelGGL((k_gate_ticks<0, 0>), dim3(grid), dim3(256), lds, s, g);
    }
    return hipGetLastError();
}

}  // namespace ewk

