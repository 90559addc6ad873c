// ewk_db64.h -- 10 log10(x) in float64 for the fp64 re-score's log-mel (ewk_rescore.h,
// rs_frames): the reference's power_to_db (librosa 0.11.0, 10.0 * np.log10(max(amin, S)),
// wakeword.py:561-563) on values x >= 1e-10 (the amin clamp comes first), NaN and +inf passed
// through.  Host and device: tests/test_db64.py builds this header with g++ and checks it
// against long double over the whole range the re-score sees.
//
// The device library's log10 carries extra-precision steps (~100 dependent float64
// instructions, four per frame pair and lane -- half the float64 work of a frame); this is
// the classic argument reduction x = 2^k m, m in [sqrt(1/2), sqrt(2)), f = m - 1,
// s = f / (2 + f), log(1 + f) = f - (hfsq - s (hfsq + R(s^2))) with the degree-7 minimax
// R of the freely distributable fdlibm e_log.c (< 1 ulp for log), ~30 instructions, then
// 10 log10(x) = k (10 log10 2) + log(m) (10 / ln 10): within a few ulps of 10 * log10(x),
// far below the re-score's 1e-9 parity bar (its inputs already differ from numpy's by the
// FFT's rounding).
#pragma once
#include <cmath>

#ifndef __HIPCC__
#define EWK_DB64_HD inline
#else
#define EWK_DB64_HD __host__ __device__ __forceinline__
#endif

EWK_DB64_HD double ewk_db64(double x) {
    constexpr double kLg1 = 6.666666666666735130e-01, kLg2 = 3.999999999940941908e-01,
                     kLg3 = 2.857142874366239149e-01, kLg4 = 2.222219843214978396e-01,
                     kLg5 = 1.818357216161805012e-01, kLg6 = 1.531383769920937332e-01,
                     kLg7 = 1.479819860511658591e-01;
    constexpr double kSqrtHalf = 0.70710678118654752440;
    constexpr double k10Log10_2 = 3.0102999566398119521;     // 10 log10(2)
    constexpr double k10InvLn10 = 4.3429448190325182765;     // 10 / ln(10)
    int k;
    double m = frexp(x, &k);   // [0.5, 1) (NaN / inf: returned as is)
    if (m < kSqrtHalf) { m += m; k -= 1; }
    const double f = m - 1.0;   // exact (m within a factor of 2 of 1)
    const double d = 2.0 + f;
    // s = f / d: a reciprocal seed, two Newton steps and a residual correction
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(d);
#else
    double r = (double)(1.0f / (float)d);
#endif
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    double s = f * r;
    s = fma(fma(-d, s, f), r, s);
    const double z = s * s, w = z * z;
    const double t1 = w * (kLg2 + w * (kLg4 + w * kLg6));
    const double t2 = z * (kLg1 + w * (kLg3 + w * (kLg5 + w * kLg7)));
    const double R = t2 + t1;
    const double hfsq = 0.5 * f * f;
    const double lnm = f - (hfsq - s * (hfsq + R));
    const double y = fma((double)k, k10Log10_2, lnm * k10InvLn10);
    return x == INFINITY ? x : y;
}
