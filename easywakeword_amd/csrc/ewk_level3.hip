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
//     or from a linear float32 batch.
//   * k_decode_pcm16: librosa.load / soundfile / PortAudio int16 -> float32
//     (x / 32768, exact), the WAV/PCM16 ingest of SURVEY.md 8f.2.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "ewk_internal.h"

#pragma clang fp contract(off)

namespace ewk {

constexpr int kL3MaxLeaves = 128;   // a chunk of <= 8192 elements has <= 128 leaves

// Leaves of numpy's pairwise recursion over [0, n), depth-first, left to right.
__device__ int l3_build_leaves(int n, int16_t* lstart, int16_t* llen) {
    int st_s[16], st_n[16];
    int sp = 0, cnt = 0;
    st_s[sp] = 0;
    st_n[sp] = n;
    ++sp;
    while (sp > 0) {
        --sp;
        const int s = st_s[sp], m = st_n[sp];
        if (m <= 128) {
            lstart[cnt] = (int16_t)s;
            llen[cnt] = (int16_t)m;
            ++cnt;
        } else {
            int n2 = m / 2;
            n2 -= n2 % 8;
            st_s[sp] = s + n2; st_n[sp] = m - n2; ++sp;   // right pushed first: left visited first
            st_s[sp] = s;      st_n[sp] = n2;     ++sp;
        }
    }
    return cnt;
}

// Post-order recombination of the leaf sums: f(m) = m <= 128 ? leaf : f(n2) + f(m - n2).
__device__ double l3_combine(int n, const double* leaf) {
    int st_n[16], st_state[16];
    double st_val[16];
    int sp = 1, li = 0;
    st_n[0] = n;
    st_state[0] = 0;
    double ret = 0.0;
    while (sp > 0) {
        const int top = sp - 1;
        const int m = st_n[top];
        if (m <= 128) {
            ret = leaf[li++];
            --sp;
            while (sp > 0) {   // deliver ret to the parent
                const int p = sp - 1;
                if (st_state[p] == 1) {   // left done: keep it, descend right
                    st_val[p] = ret;
                    st_state[p] = 2;
                    int n2 = st_n[p] / 2;
                    n2 -= n2 % 8;
                    st_n[sp] = st_n[p] - n2;
                    st_state[sp] = 0;
                    ++sp;
                    break;
                }
                ret = st_val[p] + ret;    // right done: combine
                --sp;
            }
        } else {
            st_state[top] = 1;
            int n2 = m / 2;
            n2 -= n2 % 8;
            st_n[sp] = n2;
            st_state[sp] = 0;
            ++sp;
        }
    }
    return ret;
}

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
    const float* base;   // linear: segment start; ring: stream ring
    int32_t start;       // ring: physical index of sample 0
    int32_t ring;        // 0 = linear
    __device__ __forceinline__ double operator()(int i) const {
        if (!ring) return (double)base[i];
        int k = start + i;
        if (k >= ring) k -= ring;
        return (double)base[k];
    }
};

struct L3Lds {   // a staged chunk (LDS)
    const float* p;
    __device__ __forceinline__ double operator()(int i) const { return (double)p[i]; }
};

__global__ __launch_bounds__(256) void k_normalize(L3Args a) {
    __shared__ int16_t s_lstart[4][kL3MaxLeaves], s_llen[4][kL3MaxLeaves];
    __shared__ double s_leaf[4][kL3MaxLeaves];
    __shared__ int s_cnt[4];
    // each 8192-sample chunk is staged with coalesced loads before the leaf sums (a
    // lane's leaf read straight from global memory costs a scattered round trip per
    // 8 samples)
    __shared__ float s_x[4][8192];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= a.n) return;
    L3Src x;
    int n;
    if (a.ring_len) {
        const ewk_event ev = a.events[i];
        x.base = a.pcm + (int64_t)ev.stream * a.ring_len;
        x.start = (int32_t)ev.ring_start;
        x.ring = (int32_t)a.ring_len;
        n = ev.length;
    } else {
        x.base = a.pcm + a.offsets[i];
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
        if (lane == 0) s_cnt[wave] = l3_build_leaves(cn, s_lstart[wave], s_llen[wave]);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        const int nl = s_cnt[wave];
        const L3Src xc{x.base, x.ring ? (x.start + c0) % x.ring : 0, x.ring};
        const L3Src xl = x.ring ? xc : L3Src{x.base + c0, 0, 0};
        float* sx = s_x[wave];
        for (int k0 = 0; k0 < cn; k0 += 64 * 8) {   // 8 loads per lane in flight
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + 64 * u + lane;
                v[u] = k < cn ? (float)xl(k) : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + 64 * u + lane;
                if (k < cn) sx[k] = v[u];
            }
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        const L3Lds xs{sx};
        for (int l = lane; l < nl; l += 64) s_leaf[wave][l] = l3_leaf_sum(xs, s_lstart[wave][l], s_llen[wave][l]);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        double part = 0.0;
        if (lane == 0) part = l3_combine(cn, s_leaf[wave]);
        acc += __shfl(part, 0, 64);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
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
    hipLaunchKernelGGL(k_normalize, dim3((a.n + 3) / 4), dim3(256), 0, s, a);
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
