// ewk_tables.cpp -- host construction of the constant tables of the scorer.
//
// Window : scipy.signal.get_window('hann', 512, fftbins=True)  (scipy 1.15.3)
//          = general_cosine(513, [0.5, 0.5]) truncated to 512 points,
//          fac = linspace(-pi, pi, 513), w = 0.5 + 0.5*cos(fac).
// Mel    : librosa 0.11.0 filters.mel(sr=16000, n_fft=512, n_mels=128, fmin=0,
//          fmax=8000, htk=False, norm="slaney", dtype=float32), including its
//          double rounding (triangle -> float32, then *= enorm in float64 -> float32).
// DCT    : scipy.fft.dct(type=2, norm="ortho") rows 0..19 over 128 mels.
#include <math.h>
#include <string.h>

#include <vector>

#include "ewk_internal.h"

namespace ewk {

static const double kPi = 3.14159265358979323846;

// numpy.linspace(start, stop, num) with endpoint=True (step form used by numpy 2.x)
static std::vector<double> linspace(double start, double stop, int num) {
    std::vector<double> y(num);
    const double div = num - 1;
    const double step = (stop - start) / div;
    for (int i = 0; i < num; ++i) y[i] = i * step + start;
    if (num > 1) y[num - 1] = stop;
    return y;
}

static void hann_periodic(double* w) {
    std::vector<double> fac = linspace(-kPi, kPi, NFFT + 1);
    for (int n = 0; n < NFFT; ++n) w[n] = 0.5 + 0.5 * cos(fac[n]);
}

// librosa hz_to_mel / mel_to_hz, Slaney scale.
static const double kFsp = 200.0 / 3;
static double hz_to_mel(double f) {
    const double min_log_hz = 1000.0;
    const double min_log_mel = min_log_hz / kFsp;
    const double logstep = log(6.4) / 27.0;
    if (f >= min_log_hz) return min_log_mel + log(f / min_log_hz) / logstep;
    return f / kFsp;
}
static double mel_to_hz(double m) {
    const double min_log_hz = 1000.0;
    const double min_log_mel = min_log_hz / kFsp;
    const double logstep = log(6.4) / 27.0;
    if (m >= min_log_mel) return min_log_hz * exp(logstep * (m - min_log_mel));
    return kFsp * m;
}

static void mel_dense(float* w /* [128][257] */) {
    const int sr = 16000;
    const double fmax = sr / 2.0;
    double fft[NBIN];
    const double val = 1.0 / (NFFT * (1.0 / sr));
    for (int k = 0; k < NBIN; ++k) fft[k] = k * val;
    std::vector<double> mels = linspace(hz_to_mel(0.0), hz_to_mel(fmax), NMEL + 2);
    std::vector<double> mel_f(NMEL + 2);
    for (int i = 0; i < NMEL + 2; ++i) mel_f[i] = mel_to_hz(mels[i]);
    for (int i = 0; i < NMEL; ++i) {
        const double fd0 = mel_f[i + 1] - mel_f[i];
        const double fd1 = mel_f[i + 2] - mel_f[i + 1];
        const double enorm = 2.0 / (mel_f[i + 2] - mel_f[i]);
        for (int k = 0; k < NBIN; ++k) {
            const double lower = -(mel_f[i] - fft[k]) / fd0;
            const double upper = (mel_f[i + 2] - fft[k]) / fd1;
            double tri = lower < upper ? lower : upper;
            if (!(tri > 0.0)) tri = 0.0;
            const float t32 = (float)tri;
            w[i * NBIN + k] = (float)((double)t32 * enorm);
        }
    }
}

static void dct_rows(double* d /* [20][128] */) {
    for (int k = 0; k < NMFCC; ++k) {
        const double s = k == 0 ? sqrt(1.0 / NMEL) : sqrt(2.0 / NMEL);
        for (int m = 0; m < NMEL; ++m) d[k * NMEL + m] = s * cos(kPi * k * (2.0 * m + 1.0) / (2.0 * NMEL));
    }
}

// Per-band read shifts of the mel stage.  Lane (f, j) of a scorer wave reads bins
// band_lo[j + 16 i] + q (q < group width) of frame 4 g + f for band group i, one ds_read_b32
// per (g, i, q); the 32 lanes of a half-wave (two frames, 16 bands) collide whenever two
// addresses share a bank.  A band narrower than its group width may start its read window
// up to (width - band width) bins early (the extra leading weights are zero: acc + 0 * p =
// acc, so the sums are bit-identical); the shifts are chosen band by band to minimise the
// worst bank multiplicity, then the sum of squared multiplicities (simulated LDS cycles of the
// stage: 296 -> 176 per wave pass, 160 conflict free).
static int melread_cost(const int* lo_s, int i, int width, long* sq) {
    int worst_total = 0;
    for (int g = 0; g < kNF; ++g)
        for (int q = 0; q < width; ++q)
            for (int h = 0; h < 2; ++h) {   // half-wave: frames 4 g + 2 h, 4 g + 2 h + 1
                int addr[32], worst = 0;
                for (int l = 0; l < 32; ++l) {
                    const int f = 2 * h + (l >> 4), j = l & 15;
                    addr[l] = scr_frame_off(4 * g + f) + lo_s[j + 16 * i] + q;
                }
                for (int b = 0; b < 64; ++b) {
                    int distinct[32], nd = 0;
                    for (int l = 0; l < 32; ++l) {
                        if (((addr[l] % 64) + 64) % 64 != b) continue;
                        bool seen = false;
                        for (int d = 0; d < nd; ++d) seen = seen || distinct[d] == addr[l];
                        if (!seen) distinct[nd++] = addr[l];
                    }
                    worst = nd > worst ? nd : worst;
                    *sq += (long)nd * nd;
                }
                worst_total += worst;
            }
    return worst_total;
}

static void mel_read_shifts(const int* lo, const int* n, const int* gw, int* shift) {
    int lo_s[NMEL];
    for (int m = 0; m < NMEL; ++m) { shift[m] = 0; lo_s[m] = lo[m]; }
    for (int m = 0; m < NMEL; ++m) {
        const int i = m / 16, slack = gw[i] - n[m];
        int best_s = 0, best_w = 1 << 30;
        long best_q = 0;
        for (int s = 0; s <= slack && lo[m] - s >= 0; ++s) {
            lo_s[m] = lo[m] - s;
            long sq = 0;
            const int w = melread_cost(lo_s, i, gw[i], &sq);
            if (w < best_w || (w == best_w && sq < best_q)) { best_w = w; best_q = sq; best_s = s; }
        }
        shift[m] = best_s;
        lo_s[m] = lo[m] - best_s;
    }
}

void build_tables(Tables* t) {
    memset(t, 0, sizeof(*t));
    double w[NFFT];
    hann_periodic(w);
    for (int n = 0; n < 256; ++n) t->win2[n] = make_float2((float)w[2 * n], (float)w[2 * n + 1]);
    for (int k1 = 0; k1 < 16; ++k1)
        for (int j = 0; j < 16; ++j) {
            const double a = 2.0 * kPi * (double)(j * k1) / 256.0;
            t->tw1[k1 * 16 + j] = make_float2((float)cos(a), (float)-sin(a));
        }
    for (int k = 0; k < 256; ++k) {
        const double a = 2.0 * kPi * (double)k / 512.0;
        t->tw2[k] = make_float2((float)cos(a), (float)sin(a));
    }
    std::vector<float> mel(NMEL * NBIN);
    mel_dense(mel.data());
    static const int kGroupW[8] = {2, 2, 2, 3, 4, 6, 9, 12};   // == kMelW in ewk_mfcc.hip
    int it0[8];
    int acc = 0;
    for (int i = 0; i < 8; ++i) { it0[i] = acc; acc += kGroupW[i]; }
    t->ok = acc == MEL_ITERS;
    int blo[NMEL], bn[NMEL], shift[NMEL];
    for (int m = 0; m < NMEL; ++m) {
        int lo = -1, hi = -1;
        for (int k = 0; k < NBIN; ++k)
            if (mel[m * NBIN + k] != 0.0f) {
                if (lo < 0) lo = k;
                hi = k;
            }
        if (lo < 0) { lo = 0; hi = -1; }
        blo[m] = lo;
        bn[m] = hi - lo + 1;
        if (bn[m] > kGroupW[m / 16] || lo + kGroupW[m / 16] > SCR_FRAME) t->ok = 0;
    }
    mel_read_shifts(blo, bn, kGroupW, shift);
    for (int m = 0; m < NMEL; ++m) {
        const int i = m / 16, j = m % 16, s = shift[m];
        t->band_lo[m] = blo[m] - s;   // the lane's read window starts s bins early
        for (int q = 0; q < kGroupW[i]; ++q)
            t->wpad[(it0[i] + q) * 16 + j] = q >= s && q - s < bn[m] ? 0.25f * mel[m * NBIN + blo[m] + q - s] : 0.0f;
    }
    double d[NMFCC * NMEL];
    dct_rows(d);
    for (int i = 0; i < NMFCC * NMEL; ++i) t->dct[i] = (float)d[i];
}

void build_tables64(Tables64* t) {
    memset(t, 0, sizeof(*t));
    hann_periodic(t->win);
    for (int n = 0; n < NFFT; ++n) {
        const double a = 2.0 * kPi * (double)n / NFFT;
        t->cs[n] = cos(a);
        t->sn[n] = sin(a);
    }
    mel_dense(t->melw_dense);
    dct_rows(t->dct);
    // exactly (anti)symmetric rows, D[k][127 - m] = (-1)^k D[k][m]: the re-score keeps bands
    // 0..63 of the table in LDS (ewk_rescore.h) -- the mirrored entries move by an ulp at most
    for (int k = 0; k < NMFCC; ++k)
        for (int m = NMEL / 2; m < NMEL; ++m)
            t->dct[k * NMEL + m] = (k & 1) ? -t->dct[k * NMEL + NMEL - 1 - m] : t->dct[k * NMEL + NMEL - 1 - m];
    int off = 0;
    for (int m = 0; m < NMEL; ++m) {
        int lo = -1, hi = -1;
        for (int k = 0; k < NBIN; ++k)
            if (t->melw_dense[m * NBIN + k] != 0.0f) {
                if (lo < 0) lo = k;
                hi = k;
            }
        if (lo < 0) { lo = 0; hi = -1; }
        t->mel_lo[m] = lo;
        t->mel_off[m] = off;
        for (int k = lo; k <= hi && off < (int)(sizeof(t->mel_w) / sizeof(float)); ++k) t->mel_w[off++] = t->melw_dense[m * NBIN + k];
    }
    t->mel_off[NMEL] = off;
}

void table_window(double* w) { hann_periodic(w); }
void table_mel(float* w) { mel_dense(w); }
void table_dct(double* d) { dct_rows(d); }

}  // namespace ewk
