// fp4_tables.h -- host tables of the shelved four-lanes-per-frame pass (ewk_fp4.h; round 5,
// measured slower than the product pass and kept out of libewk.so: DESIGN.md section 4,
// "Round 5").  Only scripts/probes/fp4_probe.hip includes this; it links the product's
// ewk_tables.cpp for the window, the librosa mel basis and the DCT rows.
#pragma once

#include <math.h>
#include <string.h>

#include <vector>

#include "../../../easywakeword_amd/csrc/ewk_internal.h"
#include "ewk_fp4_mel.h"

namespace ewk {

// Maps of the pass (scripts/fp4_model.py): the DFT64 output k'' that slot q of row g holds
// after the row transposition, and the factoring of the W64^(j k2) twiddles (form A:
// m (1 - i f), m = cos, f = tan; form B: m (f - i), m = sin, f = cot).
__host__ __device__ constexpr int f4_sigma0(int q) { return q < 8 ? q : (q < 15 ? q + 1 : 8); }
__host__ __device__ constexpr int f4_item(int g, int q) {
    return g == 0 ? 4 * f4_sigma0(q)
                  : (g == 2 ? 4 * q + 2 : (g == 1 ? 4 * q + (q < 8 ? 1 : 3) : 4 * q + (q < 8 ? 3 : 1)));
}
__host__ __device__ constexpr bool f4_formA(int jk) { return (jk % 32) <= 8 || (jk % 32) >= 24; }
// bin whose (cos, tan)(2 pi k / 512) untangle pair j = 4 q + k' of row g uses (row 0, q = 0:
// bins 64/192, 32/224, 96/160 and 128)
__host__ __device__ constexpr int f4_untangle_bin(int g, int j) {
    return (g == 0 && j < 4) ? (j == 0 ? 64 : (j == 1 ? 32 : (j == 2 ? 96 : 128))) : f4_item(g, j >> 2) + 64 * (j & 3);
}

struct Fp4Tables {
    float2 win4[4][64];      // [r][16 n1 + 4 a + c] = (w[2r + 8n'], w[2r + 8n' + 1]), n' = n1 + 4 (a + 4 c)
    float tw64[16][12];      // [k2][4 (j - 1)] = (m, -m, f, -f) of W64^(j k2), j = 1..3 (f4_formA)
    float4 tw4[4][16][3];    // [g][q][s - 1] = (-s, s, c, c) of W256^(s f4_item(g, q)) = c + i s
    float2 utc[4][32];       // [g][j] = (-cos, cos)(2 pi f4_untangle_bin(g, j) / 512)
    float2 utt[4][32];       // [g][j] = (t, t), t = tan(2 pi f4_untangle_bin(g, j) / 512)
    float melw4[4][F4_NINC]; // [g][e]: 0.25 x librosa weight of incidence e's band on row g's bin
    float dct[NMFCC * NMEL]; // DCT-II ortho rows 0..19
    int32_t ok4;             // the incidence list covers every non-zero weight of the basis
};

inline void build_tables_fp4(Fp4Tables* t) {
    const double kPi = 3.14159265358979323846;
    memset(t, 0, sizeof(*t));
    double w[NFFT];
    table_window(w);
    std::vector<float> mel(NMEL * NBIN);
    table_mel(mel.data());
    double d[NMFCC * NMEL];
    table_dct(d);
    for (int i = 0; i < NMFCC * NMEL; ++i) t->dct[i] = (float)d[i];
    for (int r = 0; r < 4; ++r)   // [r][n1][a][c]: column a of DFT16 block n1 reads 32 contiguous bytes
        for (int n1 = 0; n1 < 4; ++n1)
            for (int a = 0; a < 4; ++a)
                for (int c = 0; c < 4; ++c) {
                    const int np = n1 + 4 * (a + 4 * c);
                    t->win4[r][16 * n1 + 4 * a + c] = make_float2((float)w[2 * r + 8 * np], (float)w[2 * r + 8 * np + 1]);
                }
    for (int k2 = 1; k2 < 16; ++k2)
        for (int j = 1; j <= 3; ++j) {   // W64^(j k2) = m (1 - i f) (form A) or -i m (1 + i f) (form B)
            const int jk = j * k2;
            const double ph = 2.0 * kPi * jk / 64.0;
            const bool a = f4_formA(jk);
            const float m = (float)(a ? cos(ph) : sin(ph)), f = (float)(a ? tan(ph) : cos(ph) / sin(ph));
            float* e = &t->tw64[k2][4 * (j - 1)];
            e[0] = m; e[1] = -m; e[2] = f; e[3] = -f;
        }
    for (int g = 0; g < 4; ++g)
        for (int q = 0; q < 16; ++q)
            for (int s = 1; s <= 3; ++s) {
                const double ph = 2.0 * kPi * s * f4_item(g, q) / 256.0;
                const float c = (float)cos(ph), sn = (float)-sin(ph);
                t->tw4[g][q][s - 1] = make_float4(-sn, sn, c, c);
            }
    for (int g = 0; g < 4; ++g)
        for (int j = 0; j < 32; ++j) {
            const double ph = 2.0 * kPi * f4_untangle_bin(g, j) / 512.0;   // cos is never 0 in float (k = 128: 6.1e-17)
            const float c = (float)cos(ph);
            t->utc[g][j] = make_float2(-c, c);
            t->utt[g][j] = make_float2((float)(sin(ph) / cos(ph)), (float)(sin(ph) / cos(ph)));
        }
    // per-row weights of the incidence list; every non-zero weight must be covered
    std::vector<char> covered(NMEL * NBIN, 0);
    for (int G = 0; G < 4; ++G)
        for (int e = F4_INC_START[G]; e < F4_INC_START[G + 1]; ++e) {
            const bool real = e < F4_INC_START[G] + F4_INC_COUNT[G];
            const int m = 32 * G + F4_INC_BAND[e], slot = F4_INC_SLOT[e];
            for (int g = 0; g < 4; ++g) {
                const int b = f4_item(g, slot >> 2) + 64 * (slot & 3);
                const float wv = real ? mel[m * NBIN + b] : 0.0f;
                t->melw4[g][e] = 0.25f * wv;
                if (real && wv != 0.0f) covered[m * NBIN + b] = 1;
            }
        }
    t->ok4 = 1;
    for (int m = 0; m < NMEL; ++m)
        for (int b = 0; b < NBIN; ++b)
            if (mel[m * NBIN + b] != 0.0f && !covered[m * NBIN + b]) t->ok4 = 0;
}

}  // namespace ewk
