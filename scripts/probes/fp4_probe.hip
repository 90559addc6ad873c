// fp4_probe.hip -- the four-lanes-per-frame pass (scripts/experiments/fp4/ewk_fp4.h) alone: log-mel values of
// every frame of a batch of equal-length segments (check mode), or timed passes (time mode).
//
//   fp4_probe check <pcm.f32> <n_seg> <len> <out.f32>       -> out[seg][t][128] (dB, no top_db)
//   fp4_probe time  <n_seg> <len> <reps> [dct]               -> frames/s of pass (+ DCT)
//
// scripts/fp4_probe.py builds it, writes the input and compares check-mode output with the
// oracle (oracle/mfcc_ref.py) before top_db.  One 8-wave workgroup per CU, persistent waves
// taking segments from an atomic counter, like the product scorer's linear mode.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../experiments/fp4/ewk_fp4.h"

using namespace ewk;

#ifndef FP4_NW
#define FP4_NW 8
#endif
constexpr int NW = FP4_NW;   // waves per workgroup (one workgroup per CU: 8 = two waves per SIMD)
#ifdef FP4_TIMING
__device__ unsigned long long g_tdbg[8];
#define TARG , tdbg
#else
#define TARG
#endif
// (padded past half the CU's LDS: one workgroup per CU whatever NW is)
constexpr int PROBE_LDS_MIN = fp4::TABLE_BYTES + NW * fp4::STAGE_BYTES;
constexpr int PROBE_LDS = PROBE_LDS_MIN > 82 * 1024 ? PROBE_LDS_MIN : 82 * 1024;

template <int MODE>   // 0 check (write log-mel), 1 time (checksum), 2 time with DCT, 3 check MFCC (pass + DCT)
__global__ __launch_bounds__(64 * NW, 1) void k_probe(const Fp4Tables* __restrict__ tab, const float* __restrict__ pcm,
                                                      int n_seg, int len, int* work, float* out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    fp4::fill_tables(tab, smem, 1.0f, threadIdx.x, blockDim.x);
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* stage = reinterpret_cast<float*>(smem + fp4::TABLE_BYTES +
                                            __builtin_amdgcn_readfirstlane(wave * fp4::STAGE_BYTES));
    const int T = 1 + len / HOP, npass = (T + 15) / 16;
    float sink = 0.0f;
#ifdef FP4_TIMING
    uint64_t tdbg[8] = {};
#endif
    for (;;) {
        int idx = 0;
        if (lane == 0) idx = atomicAdd(work, 1);
        idx = __shfl(idx, 0, 64);
        if (idx >= n_seg) break;
        const uint64_t sb = (uint64_t)(pcm + (int64_t)idx * len);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)sb), hi = __builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                                                            __builtin_amdgcn_readfirstlane(len * 4), 0x00020000);
        fp4::stage_dma_linear(rs, -NFFT / 2, stage, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int ps = 0; ps < npass; ++ps) {
            const int t0 = 16 * ps;
            float lm[32], vmax = -INFINITY, vmin = INFINITY, nanp = 0.0f;
            const bool valid = t0 + (lane & 15) < T;
            fp4::pass(smem, stage, lane, valid, lm, vmax, vmin, nanp, [&]() {
                if (ps + 1 < npass) fp4::stage_dma_linear(rs, (t0 + 16) * HOP - NFFT / 2, stage, lane);
            } TARG);
#ifdef FP4_TIMING
            const uint64_t tw0 = __builtin_amdgcn_s_memtime();
#endif
            if (MODE == 0) {
                const int t = t0 + (lane & 15), r = lane >> 4;
                if (t < T)
#pragma unroll
                    for (int G = 0; G < 4; ++G)
#pragma unroll
                        for (int i = 0; i < 8; ++i)
                            out[((int64_t)idx * T + t) * NMEL + 32 * G + 8 * r + i] = lm[8 * G + i];
            } else if (MODE == 3) {
                float c[8];
                fp4::dct(lm, -INFINITY, smem, lane, c);
                const int t = t0 + (lane & 15), h = lane >> 4;
                if (t < T) {
                    float* lo2 = out + (int64_t)n_seg * T * NMFCC;   // the log-mel too, after the MFCCs
#pragma unroll
                    for (int G = 0; G < 4; ++G)
#pragma unroll
                        for (int i = 0; i < 8; ++i) lo2[((int64_t)idx * T + t) * NMEL + 32 * G + 8 * h + i] = lm[8 * G + i];
#pragma unroll
                    for (int i = 0; i < 4; ++i) out[((int64_t)idx * T + t) * NMFCC + 4 * h + i] = c[i];
                    if (h == 0)
#pragma unroll
                        for (int i = 0; i < 4; ++i) out[((int64_t)idx * T + t) * NMFCC + 16 + i] = c[4 + i];
                }
            } else if (MODE == 2) {
                float c[8];
                fp4::dct(lm, vmax - 80.0f, smem, lane, c);
#pragma unroll
                for (int i = 0; i < 8; ++i) sink += c[i];
            } else {
#pragma unroll
                for (int i = 0; i < 32; ++i) sink += lm[i];
            }
            sink += vmax + vmin + nanp;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next pass's samples have landed
#ifdef FP4_TIMING
            tdbg[7] += __builtin_amdgcn_s_memtime() - tw0;   // consumer + the wait for the next stage
#endif
        }
    }
    if (MODE != 0 && sink == 12345.678f) out[0] = sink;   // keep the work alive
#ifdef FP4_TIMING
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&g_tdbg[k], (unsigned long long)tdbg[k]);
#endif
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 2;                                                               \
        }                                                                           \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) return 1;
    const bool mfcc = !strcmp(argv[1], "mfcc");
    const bool check = !strcmp(argv[1], "check") || mfcc;
    Fp4Tables* ht = (Fp4Tables*)calloc(1, sizeof(Fp4Tables));
    build_tables_fp4(ht);
    if (!ht->ok4) {
        fprintf(stderr, "tables not ok\n");
        return 3;
    }
    Fp4Tables* dt;
    CK(hipMalloc(&dt, sizeof(Fp4Tables)));
    CK(hipMemcpy(dt, ht, sizeof(Fp4Tables), hipMemcpyHostToDevice));
    int n_seg, len;
    std::vector<float> pcm;
    if (check) {
        n_seg = atoi(argv[3]);
        len = atoi(argv[4]);
        pcm.resize((size_t)n_seg * len);
        FILE* f = fopen(argv[2], "rb");
        if (!f || fread(pcm.data(), 4, pcm.size(), f) != pcm.size()) return 4;
        fclose(f);
    } else {
        n_seg = atoi(argv[2]);
        len = atoi(argv[3]);
        pcm.resize((size_t)n_seg * len);
        uint32_t s = 12345;
        for (auto& x : pcm) {
            s = s * 1664525u + 1013904223u;
            x = ((int)(s >> 8) - (1 << 23)) * (1.0f / (1 << 23)) * 0.3f;
        }
    }
    const int T = 1 + len / HOP;
    float *dp, *dout;
    int* dw;
    CK(hipMalloc(&dp, pcm.size() * 4));
    CK(hipMemcpy(dp, pcm.data(), pcm.size() * 4, hipMemcpyHostToDevice));
    const size_t nout = check ? (size_t)n_seg * T * (mfcc ? NMFCC + NMEL : NMEL) : 1;
    CK(hipMalloc(&dout, nout * 4));
    CK(hipMalloc(&dw, 4));
    int dev_cu = 256;
    hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, 0);
    if (check) {
        CK(hipMemset(dw, 0, 4));
        if (mfcc) hipLaunchKernelGGL(k_probe<3>, dim3(dev_cu), dim3(64 * NW), PROBE_LDS, 0, dt, dp, n_seg, len, dw, dout);
        else hipLaunchKernelGGL(k_probe<0>, dim3(dev_cu), dim3(64 * NW), PROBE_LDS, 0, dt, dp, n_seg, len, dw, dout);
        CK(hipDeviceSynchronize());
        std::vector<float> o(nout);
        CK(hipMemcpy(o.data(), dout, nout * 4, hipMemcpyDeviceToHost));
        FILE* f = fopen(argv[5], "wb");
        fwrite(o.data(), 4, nout, f);
        fclose(f);
        printf("fp4_probe check: %d segments x %d frames written\n", n_seg, T);
        return 0;
    }
    const int reps = atoi(argv[4]);
    const bool with_dct = argc > 5 && !strcmp(argv[5], "dct");
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f, tot = 0.0f;
    for (int it = 0; it < reps + 3; ++it) {
        CK(hipMemset(dw, 0, 4));
        CK(hipEventRecord(e0));
        if (with_dct) hipLaunchKernelGGL(k_probe<2>, dim3(dev_cu), dim3(64 * NW), PROBE_LDS, 0, dt, dp, n_seg, len, dw, dout);
        else hipLaunchKernelGGL(k_probe<1>, dim3(dev_cu), dim3(64 * NW), PROBE_LDS, 0, dt, dp, n_seg, len, dw, dout);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 3) {
            best = ms < best ? ms : best;
            tot += ms;
        }
    }
    const double frames = (double)n_seg * T, computed = (double)n_seg * ((T + 15) / 16) * 16;
    printf("fp4_probe time%s: %d segments x %d frames: best %.3f ms, mean %.3f ms -> %.3f G frames/s (%.3f G computed/s)\n",
           with_dct ? "+dct" : "", n_seg, T, best, tot / reps, frames / best * 1e-6, computed / best * 1e-6);
#ifdef FP4_TIMING
    unsigned long long d[8];
    CK(hipMemcpyFromSymbol(d, HIP_SYMBOL(g_tdbg), sizeof(d)));
    const char* nm[8] = {"load+DFT16", "twiddled DFT4", "transpose", "post-T", "untangle", "mel+log", "", "after+wait"};
    double tsum = 0;
    for (int k = 0; k < 8; ++k) if (k != 6) tsum += (double)d[k] / d[6];
    printf("cycles per pass (s_memtime, %llu passes):", d[6]);
    for (int k = 0; k < 8; ++k) if (k != 6) printf(" %s %.0f", nm[k], (double)d[k] / d[6]);
    printf(" | sum %.0f\n", tsum);
#endif
    return 0;
}
