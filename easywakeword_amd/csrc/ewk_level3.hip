// ewk_level3.hip -- the data formats either side of the hot path:
//
//   * k_normalize: the level-3 confirm stage's pre-processing of gated segments,
//     WakeWord._transcribe_audio (reference wakeword.py:1019-1025):
//         y = x - np.mean(x); m = np.max(np.abs(y)); if m > 0: y = y / m
//         y = y * 1.5; y = np.clip(y, -1.0, 1.0)
//     in float64, bit-identical to numpy: the mean follows np.add.reduce's
//     pairwise order (chunks of 8192, 8-accumulator leaves of <= 128, split at
//     n2 = n/2 - (n/2)%8), every other step is elementwise IEEE arithmetic.
//     One wave per segment, read straight from the stream ring (gathered events)
//     or from a linear float32 batch; each 8192-sample chunk is staged in LDS and its
//     pairwise tree evaluated lane-parallel (split top-down, combined bottom-up).
//   * k_decode_pcm16: librosa.load / soundfile / PortAudio int16 -> float32
//     (x / 32768, exact), the WAV/PCM16 ingest of SURVEY.md 8f.2.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "ewk_internal.h"

#pragma clang fp contract(off)

namespace ewk {

template <typename Src>
__device__ __forceinline__ double l3_leaf_sum(const Src& x, int s, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r += x(s + i);
        return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = x(s + j);
    int i = 8;
    const int lim = n - (n % 8);
    for (; i < lim; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += x(s + i + j);
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += x(s + i);
    return res;
}

struct L3Src {
    const float* base;   // linear: segment start; ring: stream ring (float32) ...
    const int16_t* base16;   // ... or int16 ring (EWK_RING_I16): x / 32768, exact
    int32_t start;       // ring: physical index of sample 0
    int32_t ring;        // 0 = linear
    __device__ __forceinline__ double operator()(int i) const {
        if (!ring) return (double)base[i];
        int k = start + i;
        if (k >= ring) k -= ring;
        return base16 ? (double)base16[k] * (1.0 / 32768.0) : (double)base[k];
    }
};

struct L3Lds {   // a staged chunk (LDS)
    const float* p;
    __device__ __forceinline__ double operator()(int i) const { return (double)p[i]; }
};

// numpy's pairwise recursion over one chunk, lane-parallel: the tree is split top-down
// one depth at a time (a node of m > 128 elements splits at n2 = m/2 - (m/2)%8), each
// leaf is summed by one lane from the staged chunk, and the internal nodes are combined
// bottom-up as left + right -- the same additions as the recursion, so bit-identical.
constexpr int kL3Depth = 9;     // 8192 -> <= 128 within 7 splits; uneven splits may take one more
constexpr int kL3Nodes = 128;   // nodes per depth (a chunk has <= 128 leaves)

__device__ __forceinline__ void l3_sync() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(64) void k_normalize(L3Args a) {
    __shared__ float s_x[8192];                               // the staged chunk
    __shared__ int16_t s_ns[kL3Depth][kL3Nodes], s_nl[kL3Depth][kL3Nodes], s_nc[kL3Depth][kL3Nodes];
    __shared__ double s_nv[kL3Depth][kL3Nodes];
    __shared__ int16_t s_leaf_d[kL3Nodes], s_leaf_k[kL3Nodes];
    __shared__ int s_cnt[kL3Depth + 1];
    const int lane = threadIdx.x;
    const int i = blockIdx.x;
    if (i >= a.n) return;
    L3Src x;
    int n;
    if (a.ring_len) {
        const ewk_event ev = a.events[i];
        x.base = a.pcm ? a.pcm + (int64_t)ev.stream * a.ring_len : nullptr;
        x.base16 = a.pcm16 ? a.pcm16 + (int64_t)ev.stream * a.ring_len : nullptr;
        x.start = (int32_t)ev.ring_start;
        x.ring = (int32_t)a.ring_len;
        n = ev.length;
    } else {
        x.base = a.pcm + a.offsets[i];
        x.base16 = nullptr;
        x.start = 0;
        x.ring = 0;
        n = a.lengths[i];
    }
    if (n <= 0) return;
    double* out = a.out + a.out_offsets[i];
    // ---- np.mean: pairwise sum per 8192-element chunk, chunks accumulated from 0.0
    double acc = 0.0;
    for (int c0 = 0; c0 < n; c0 += 8192) {
        const int cn = min(8192, n - c0);
        const L3Src xc{x.base, x.base16, x.ring ? (x.start + c0) % x.ring : 0, x.ring};
        const L3Src xl = x.ring ? xc : L3Src{x.base + c0, nullptr, 0, 0};
        for (int k0 = 0; k0 < cn; k0 += 64 * 8) {   // coalesced staging, 8 loads per lane in flight
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + 64 * u + lane;
                v[u] = k < cn ? (float)xl(k) : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + 64 * u + lane;
                if (k < cn) s_x[k] = v[u];
            }
        }
        // top-down split
        if (lane == 0) {
            s_ns[0][0] = 0;
            s_nl[0][0] = (int16_t)cn;
            s_cnt[0] = 1;
            s_cnt[kL3Depth] = 0;   // leaves
        }
        l3_sync();
        int depth = 0;
        for (int d = 0; d < kL3Depth; ++d) {
            const int cnt = s_cnt[d];
            int made = 0, leaves = s_cnt[kL3Depth];
            for (int k0 = 0; k0 < cnt; k0 += 64) {
                const int k = k0 + lane;
                int st = 0, m = 0;
                if (k < cnt) {
                    st = s_ns[d][k];
                    m = s_nl[d][k];
                }
                const bool split = k < cnt && m > 128;
                const bool leaf = k < cnt && m <= 128;
                const uint64_t ms = __ballot(split), ml = __ballot(leaf);
                const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
                if (split) {
                    int n2 = m / 2;
                    n2 -= n2 % 8;
                    const int c = 2 * (made + __popcll(ms & below));
                    s_ns[d + 1][c] = (int16_t)st;
                    s_nl[d + 1][c] = (int16_t)n2;
                    s_ns[d + 1][c + 1] = (int16_t)(st + n2);
                    s_nl[d + 1][c + 1] = (int16_t)(m - n2);
                    s_nc[d][k] = (int16_t)c;
                } else if (leaf) {
                    const int q = leaves + __popcll(ml & below);
                    s_leaf_d[q] = (int16_t)d;
                    s_leaf_k[q] = (int16_t)k;
                    s_nc[d][k] = -1;
                }
                made += __popcll(ms);
                leaves += __popcll(ml);
            }
            l3_sync();
            if (lane == 0) {   // (a chunk of <= 8192 splits at most 7 times: d + 1 < kL3Depth)
                if (d + 1 < kL3Depth) s_cnt[d + 1] = 2 * made;
                s_cnt[kL3Depth] = leaves;
            }
            l3_sync();
            depth = d;
            if (made == 0) break;
        }
        // leaf sums, one lane per leaf
        const L3Lds xs{s_x};
        const int nleaf = s_cnt[kL3Depth];
        for (int q = lane; q < nleaf; q += 64) {
            const int d = s_leaf_d[q], k = s_leaf_k[q];
            s_nv[d][k] = l3_leaf_sum(xs, s_ns[d][k], s_nl[d][k]);
        }
        l3_sync();
        // bottom-up: internal node = left + right
        for (int d = depth - 1; d >= 0; --d) {
            const int cnt = s_cnt[d];
            for (int k = lane; k < cnt; k += 64) {
                const int c = s_nc[d][k];
                if (c >= 0) s_nv[d][k] = s_nv[d + 1][c] + s_nv[d + 1][c + 1];
            }
            l3_sync();
        }
        acc += s_nv[0][0];
        l3_sync();
    }
    const double mean = acc / (double)n;
    // ---- np.max(np.abs(y)) (order-free)
    double m = 0.0;
    bool nan = false;
    for (int k = lane; k < n; k += 64) {
        const double y = fabs(x(k) - mean);
        nan |= y != y;
        m = fmax(m, y);
    }
    for (int s = 1; s < 64; s <<= 1) {
        m = fmax(m, __shfl_xor(m, s, 64));
        nan |= __shfl_xor((int)nan, s, 64) != 0;
    }
    if (nan) m = __builtin_nan("");   // np.max propagates NaN
    const bool scale = m > 0.0;       // NaN > 0 is False, like the reference's `if max_val > 0`
    for (int k = lane; k < n; k += 64) {
        double y = x(k) - mean;
        if (scale) y = y / m;
        y = y * 1.5;
        out[k] = y < -1.0 ? -1.0 : (y > 1.0 ? 1.0 : y);   // np.clip keeps NaN
    }
}

hipError_t launch_normalize(const L3Args& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_normalize, dim3(a.n), dim3(64), 0, s, a);   // one wave per segment
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_decode_pcm16(const int16_t* __restrict__ in, float* __restrict__ out,
                                                      int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = (float)in[i] * (1.0f / 32768.0f);
}

hipError_t launch_decode_pcm16(const int16_t* in, float* out, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8 * 256 * 8);
    hipLaunchKernelGGL(k_decode_pcm16, dim3((unsigned)blocks), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

}  // namespace ewk
