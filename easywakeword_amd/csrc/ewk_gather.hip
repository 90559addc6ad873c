// ewk_gather.hip -- device-side compaction of positive detections for the level-3
// confirm gather (SURVEY.md 8b `ewk_gather_detections`, 8e).
//
// The reference runs its optional confirm once per detection (wakeword.py:1120-1130); on
// N GPUs only the positives cross xGMI, so the per-segment score/match arrays a batch
// step leaves in HBM are compacted on the device into (id, score, step) records plus a
// device count -- what a C/C++ host hands to its own RCCL collective.  Stable (segment
// order), three short launches, no host sync:
//   k_compact_count   one 256-thread block per 4096 segments: its match count;
//   k_compact_scan    one block: exclusive scan of the block counts after the base
//                     (*d_count when appending, else 0), and the new *d_count;
//   k_compact_scatter each block writes its matches at its offset (wave ballot scans).
#include <hip/hip_runtime.h>

#include "ewk_internal.h"

namespace ewk {

constexpr int kCompactThreads = 256;
constexpr int kCompactPer = 16;                                    // segments per thread
constexpr int kCompactChunk = kCompactThreads * kCompactPer;       // segments per block

int compact_blocks(int32_t n) { return (n + kCompactChunk - 1) / kCompactChunk; }

__global__ __launch_bounds__(kCompactThreads) void k_compact_count(const uint8_t* __restrict__ match, int32_t n,
                                                                  int32_t* __restrict__ block_count) {
    __shared__ int red[kCompactThreads / 64];
    const int64_t b0 = (int64_t)blockIdx.x * kCompactChunk;
    int c = 0;
#pragma unroll 4
    for (int k = 0; k < kCompactPer; ++k) {
        const int64_t i = b0 + (int64_t)k * kCompactThreads + threadIdx.x;
        c += (i < n && match[i]) ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kCompactThreads / 64; ++w) t += red[w];
        block_count[blockIdx.x] = t;
    }
}

// One block: block_off[b] = base + sum of block_count[0..b); *d_count = base + total.
__global__ __launch_bounds__(1024) void k_compact_scan(const int32_t* __restrict__ block_count, int32_t nb,
                                                       int32_t* __restrict__ block_off, int32_t* __restrict__ d_count,
                                                       int append) {
    __shared__ int wsum[16];
    __shared__ int carry;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) carry = append ? *d_count : 0;
    __syncthreads();
    for (int b0 = 0; b0 < nb; b0 += 1024) {
        const int b = b0 + (int)threadIdx.x;
        const int v = b < nb ? block_count[b] : 0;
        int incl = v;   // inclusive wave scan
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d, 64);
            if (lane >= d) incl += t;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        int before = carry;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        if (b < nb) block_off[b] = before + incl - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = before + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) *d_count = carry;
}

__global__ __launch_bounds__(kCompactThreads) void k_compact_scatter(const double* __restrict__ score,
                                                                    const uint8_t* __restrict__ match, int32_t n,
                                                                    int64_t first_id, int64_t step,
                                                                    const int32_t* __restrict__ block_off,
                                                                    ewk_positive* __restrict__ out) {
    __shared__ int wcount[kCompactThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t b0 = (int64_t)blockIdx.x * kCompactChunk;
    int off = block_off[blockIdx.x];
    for (int k = 0; k < kCompactPer; ++k) {   // segment order: slab k, then wave, then lane
        const int64_t i = b0 + (int64_t)k * kCompactThreads + threadIdx.x;
        const bool m = i < n && match[i];
        const uint64_t bal = __ballot(m);
        if (lane == 0) wcount[wave] = __popcll(bal);
        __syncthreads();
        int before = off;
        for (int w = 0; w < wave; ++w) before += wcount[w];
        if (m) {
            const int slot = before + __popcll(bal & ((1ull << lane) - 1ull));
            ewk_positive r;
            r.id = first_id + i;
            r.score = score[i];
            r.step = step;
            out[slot] = r;
        }
        int tot = 0;
        for (int w = 0; w < kCompactThreads / 64; ++w) tot += wcount[w];
        off += tot;
        __syncthreads();
    }
}

hipError_t launch_compact_positives(const double* score, const uint8_t* match, int32_t n, int64_t first_id,
                                    int64_t step, ewk_positive* out, int32_t* d_count, int32_t* scratch, int append,
                                    hipStream_t s) {
    const int nb = compact_blocks(n);
    int32_t* bcount = scratch;
    int32_t* boff = scratch + nb;
    if (nb > 0) hipLaunchKernelGGL(k_compact_count, dim3(nb), dim3(kCompactThreads), 0, s, match, n, bcount);
    hipLaunchKernelGGL(k_compact_scan, dim3(1), dim3(1024), 0, s, bcount, nb, boff, d_count, append);
    if (nb > 0)
        hipLaunchKernelGGL(k_compact_scatter, dim3(nb), dim3(kCompactThreads), 0, s, score, match, n, first_id, step,
                           boff, out);
    return hipGetLastError();
}

}  // namespace ewk
