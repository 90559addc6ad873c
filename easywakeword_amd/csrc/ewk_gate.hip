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
// split at n2 = n/2 - (n/2)%8), the percentile follows numpy 2.2's "linear"
// method (_compute_virtual_index / _lerp), and the clock is tick * tick_seconds.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ewk_gate.h"

// float64 parity with numpy requires un-fused multiply/add (e.g. the percentile lerp)
#pragma clang fp contract(off)

namespace ewk {

constexpr int kMaxLeaves = 256;   // n <= 8192 per chunk -> <= 128 leaves

// ---- numpy pairwise sum of squares, exact order --------------------------------
// Leaves of chunk [0, n): depth-first, left to right.  Built by every lane
// identically (uniform control flow, registers only).
struct LeafList {
    int32_t start[kMaxLeaves];
    int32_t len[kMaxLeaves];
    int32_t count;
};

__device__ __forceinline__ int split_point(int n) {
    int n2 = n / 2;
    n2 -= n2 % 8;
    return n2;
}

// Enumerate leaves of pw(n) into LDS (lane 0) -- iterative DFS.
__device__ void build_leaves(int n, int32_t* lstart, int32_t* llen, int32_t* lcount) {
    int st_s[32], st_n[32];
    int sp = 0, cnt = 0;
    st_s[sp] = 0;
    st_n[sp] = n;
    ++sp;
    while (sp > 0) {
        --sp;
        const int s = st_s[sp], m = st_n[sp];
        if (m <= 128) {
            lstart[cnt] = s;
            llen[cnt] = m;
            ++cnt;
        } else {
            const int n2 = split_point(m);
            // push right first so the left subtree is visited first
            st_s[sp] = s + n2; st_n[sp] = m - n2; ++sp;
            st_s[sp] = s;      st_n[sp] = n2;     ++sp;
        }
    }
    *lcount = cnt;
}

// Recombine leaf sums in the recursion's post-order: pw(n) = pw(left) + pw(right).
__device__ double combine_leaves(int n, const double* leaf, int& li) {
    // explicit stack emulating: f(m) = m<=128 ? leaf[li++] : f(n2) + f(m-n2)
    int st_n[32];
    int st_state[32];
    double st_val[32];
    int sp = 0;
    st_n[0] = n;
    st_state[0] = 0;
    sp = 1;
    double ret = 0.0;
    while (sp > 0) {
        const int top = sp - 1;
        const int m = st_n[top];
        if (m <= 128) {
            ret = leaf[li++];
            --sp;
            // deliver ret to parent
            while (sp > 0) {
                const int p = sp - 1;
                if (st_state[p] == 1) {         // left finished -> store, go right
                    st_val[p] = ret;
                    st_state[p] = 2;
                    st_n[sp] = st_n[p] - split_point(st_n[p]);
                    st_state[sp] = 0;
                    ++sp;
                    break;
                } else {                        // right finished -> combine
                    ret = st_val[p] + ret;
                    --sp;
                }
            }
        } else {
            st_state[top] = 1;
            st_n[sp] = split_point(m);
            st_state[sp] = 0;
            ++sp;
        }
    }
    return ret;
}

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

// numpy np.add.reduce(x**2) over n float32 samples read through src(i), wave-cooperative.
// scratch: >= 2*kMaxLeaves ints + kMaxLeaves doubles of per-wave LDS.
template <typename Src>
__device__ double wave_pairwise_sumsq(const Src& src, int n, int lane, int32_t* lstart, int32_t* llen,
                                      int32_t* lcount, double* lsum) {
    double acc = 0.0;
    for (int c0 = 0; c0 < n; c0 += 8192) {
        const int cn = min(8192, n - c0);
        if (lane == 0) build_leaves(cn, lstart, llen, lcount);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        const int nl = *lcount;
        for (int l = lane; l < nl; l += 64) lsum[l] = leaf_sumsq(src, c0 + lstart[l], llen[l]);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        double part = 0.0;
        if (lane == 0) {
            int li = 0;
            part = combine_leaves(cn, lsum, li);
        }
        part = __shfl(part, 0, 64);
        acc += part;
        asm volatile("" ::: "memory");
    }
    return acc;
}

struct RingSrc {
    const float* ring;
    int64_t first;   // physical index of element 0
    int64_t R;
    __device__ __forceinline__ float operator()(int i) const {
        int64_t k = first + i;
        if (k >= R) k -= R;
        return ring[k];
    }
};

// numpy percentile(v, 25) ("linear"), v of length nb held in LDS.
__device__ double wave_percentile25(const double* v, int nb, int lane, double* sel) {
    // virtual index = n*q + (alpha + q*(1-alpha-beta)) - 1, alpha = beta = 1, q = 0.25
    const double q = 0.25;
    const double vi = (double)nb * q + (1.0 + q * (1.0 - 1.0 - 1.0)) - 1.0;
    double prevd = floor(vi);
    int prev = (int)prevd, next = prev + 1;
    if (vi >= (double)(nb - 1)) { prev = nb - 1; next = nb - 1; }
    if (vi < 0.0) { prev = 0; next = 0; }
    const double gamma = vi - prevd;
    // rank selection with index tie-break
    for (int i = lane; i < nb; i += 64) {
        const double x = v[i];
        int r = 0;
        for (int k = 0; k < nb; ++k) {
            const double y = v[k];
            r += (y < x) || (y == x && k < i);
        }
        if (r == prev) sel[0] = x;
        if (r == next) sel[1] = x;
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const double a = sel[0], b = sel[1];
    // numpy _lerp: a + (b-a)*t, replaced by b - (b-a)*(1-t) where t >= 0.5
    const double d = b - a;
    double r = a + d * gamma;
    if (gamma >= 0.5) r = b - d * (1.0 - gamma);
    return r;
}

__global__ __launch_bounds__(256) void k_gate_ticks(GateArgs g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = blockIdx.x * 4 + wave;
    if (s >= g.n_streams) return;
    unsigned char* w = smem + wave * g.lds_per_wave;
    int32_t* lstart = reinterpret_cast<int32_t*>(w);
    int32_t* llen = lstart + kMaxLeaves;
    int32_t* lcount = llen + kMaxLeaves;                           // + 4 ints pad
    double* lsum = reinterpret_cast<double*>(lcount + 4);
    double* sel = lsum + kMaxLeaves;                               // 2 doubles
    double* brms = sel + 2;                                        // nb doubles

    const int64_t R = g.ring_len;
    const int fs = g.block;
    const int nb = g.n_blocks;
    float* ring = g.ring + (int64_t)s * R;
    GateStream st = g.st[s];
    // per-stream block RMS cache lives in global memory; stage in LDS when full
    double* grms = g.block_rms + (int64_t)s * nb;

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
        // ---- a1: ingest `fs` samples at the write pointer
        const float* src = g.pcm + (int64_t)s * g.stride + (int64_t)t * g.tick_stride;
        const int64_t p0 = st.pointer;
        for (int i = lane; i < fs; i += 64) {
            int64_t k = p0 + i;
            if (k >= R) k -= R;
            ring[k] = src[i];
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        st.pointer = (int32_t)((p0 + fs) % R);
        st.collected = min(st.collected + (int64_t)fs, R);
        const bool full = st.collected >= R;
        // ---- a2: threshold over the physical blocks (only once the ring is full)
        if (full) {
            // refresh the physical blocks overlapping the written range [p0, p0+fs)
            // (mod R); all blocks on the first fill (nothing was cached before)
            auto refresh = [&](int64_t a0, int64_t a1) {   // [a0, a1) inside [0, R)
                const int b0 = (int)(a0 / fs);
                const int b1 = (int)((a1 - 1) / fs);
                for (int b = b0; b <= b1 && b < nb; ++b) {
                    RingSrc rs{ring, (int64_t)b * fs, R};
                    const double sum = wave_pairwise_sumsq(rs, fs, lane, lstart, llen, lcount, lsum);
                    if (lane == 0) grms[b] = sqrt(sum / (double)fs);
                }
            };
            if (!st.filled) refresh(0, (int64_t)nb * fs);
            else if (p0 + fs <= R) refresh(p0, p0 + fs);
            else { refresh(p0, R); refresh(0, p0 + fs - R); }
            st.filled = 1;
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            for (int i = lane; i < nb; i += 64) brms[i] = grms[i];
            asm volatile("" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            const double p25 = wave_percentile25(brms, nb, lane, sel);
            const double thr = p25 * 1.5;
            // Python max(new, MIN): MIN only if MIN > new
            st.threshold = (g.min_threshold > thr) ? g.min_threshold : thr;
        }
        // ---- a3: is_silent(): RMS of the last n_last samples < threshold
        bool silent = true;
        {
            int64_t nl = g.n_last;
            if (nl > R) nl = R;
            if (nl > 0) {
                int64_t first = (int64_t)st.pointer - nl;
                if (first < 0) first += R;
                RingSrc rs{ring, first, R};
                const double sum = wave_pairwise_sumsq(rs, (int)nl, lane, lstart, llen, lcount, lsum);
                const double rms = sqrt(sum / (double)nl);
                st.last_rms = rms;
                silent = rms < st.threshold;
            }
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
        if (lane == 0) {
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
                        int64_t start = (int64_t)st.pointer - nreq;
                        if (start < 0) start += R;
                        ewk_event ev;
                        ev.stream = s;
                        ev.length = (int32_t)stop;
                        ev.tick = tick;
                        ev.ring_start = start;
                        ev.time = now;
                        ev.score = __builtin_nan("");
                        ev.match = 0;
                        ev.flags = ((double)stop / (double)g.sample_rate > g.max_segment_seconds) ? EWK_EV_SKIPPED : 0;
                        const int slot = atomicAdd(g.ev_count, 1);
                        if (slot < g.ev_cap) g.events[slot] = ev;
                        else atomicAdd(g.ev_dropped, 1);
                        st.state = kWaiting;
                    }
                } else st.state = kWaiting;
                break;
            }
        }
        // lane 0 owns the FSM fields; keep the wave's copy coherent
        st.state = __shfl(st.state, 0, 64);
        st.silence_start = __shfl(st.silence_start, 0, 64);
        st.sound_start = __shfl(st.sound_start, 0, 64);
        st.sound_end = __shfl(st.sound_end, 0, 64);
    }
    if (lane == 0) g.st[s] = st;
}

hipError_t launch_gate(const GateArgs& g, hipStream_t s) {
    if (g.n_streams <= 0 || g.n_ticks <= 0) return hipSuccess;
    const int grid = (g.n_streams + 3) / 4;
    hipLaunchKernelGGL(k_gate_ticks, dim3(grid), dim3(256), 4 * g.lds_per_wave, s, g);
    return hipGetLastError();
}

int gate_lds_per_wave(int n_blocks) {
    const int bytes = kMaxLeaves * 4 * 2 + 16 + kMaxLeaves * 8 + 16 + n_blocks * 8;
    return (bytes + 15) & ~15;
}

}  // namespace ewk
