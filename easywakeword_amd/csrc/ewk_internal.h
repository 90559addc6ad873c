// ewk_internal.h -- shared constants, table layout and launch prototypes.
// Internal to libewk.so; the public C ABI is include/ewk.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ewk.h"

namespace ewk {

// librosa.feature.mfcc(y, sr=16000, n_mfcc=20, n_fft=512, hop_length=160)
// as called by WordMatcher.extract_mfcc (wakeword.py:561-563).
constexpr int NFFT = 512;
constexpr int HOP = 160;
constexpr int NBIN = NFFT / 2 + 1;   // 257
constexpr int NMEL = 128;
constexpr int NMFCC = EWK_N_MFCC;    // 20
constexpr int MEL_ITERS = 40;        // unrolled mel FMAs per lane: sum of per-group band widths
constexpr int SCR_FRAME = 272;       // per-frame FFT scratch floats (16 rows x 17)
// fp32 scorer shape: two frames per 16-lane group per pass (kNF, two independent FFT
// instruction streams per lane; the untangle pairs conjugate bins inside a lane), eight
// waves per workgroup, one workgroup per CU (2 waves per SIMD at 256 VGPRs).
constexpr int kNF = 2;
#ifndef EWK_WAVES
#define EWK_WAVES 8
#endif
constexpr int WAVES = EWK_WAVES;   // waves per scorer workgroup (one workgroup per CU)
// start (floats) of frame fr's FFT scratch / power spectrum in a scorer wave's LDS scratch:
// the two frames a 16-lane group untangles side by side (fr, fr + 4) land 8 banks apart
__host__ __device__ constexpr int scr_frame_off(int fr) { return fr * SCR_FRAME + 8 * (fr >> 2); }

// Host-built constant tables (ewk_tables.cpp); copied to LDS by every workgroup.
struct Tables {
    float2 win2[256];        // (w[2n], w[2n+1]) periodic Hann, n = 0..255
    float2 tw1[256];         // [k1*16 + j] = exp(-2*pi*i*j*k1/256)
    float2 tw2[256];         // [k]  = (cos, sin)(2*pi*k/512) for the real-FFT untangle
    int32_t band_lo[NMEL];   // first non-zero bin of mel band m
    // 0.25 * librosa float32 weights (0.25 folds the untangle's 1/2 squared), laid
    // out [iteration][lane j] for band m = j + 16*i, zero-padded to the group width
    float wpad[MEL_ITERS * 16];
    float dct[NMFCC * NMEL]; // DCT-II ortho rows 0..19
    int32_t ok;              // every band fits its compile-time group width
};

// fp64 path tables (rescoring / reference precision).
struct Tables64 {
    double win[NFFT];        // periodic Hann (scipy.signal.get_window('hann', 512, fftbins=True))
    double cs[NFFT];         // cos(2*pi*n/512)
    double sn[NFFT];         // sin(2*pi*n/512)
    float melw_dense[NMEL * NBIN];  // librosa float32 mel basis [128][257]
    double dct[NMFCC * NMEL];
    // the basis's band support, packed: band m = weights mel_w[mel_off[m] .. mel_off[m+1])
    // on bins mel_lo[m], mel_lo[m] + 1, ... (every non-zero weight, in bin order)
    int32_t mel_lo[NMEL];
    int32_t mel_off[NMEL + 1];
    float mel_w[2 * NBIN + 2 * NMEL];
};

void build_tables(Tables* t);
// the builders build_tables uses (also linked by scripts/probes/fp4_probe.hip)
void table_window(double* w /* [512] */);
void table_mel(float* w /* [128][257] */);
void table_dct(double* d /* [20][128] */);
void build_tables64(Tables64* t);

// fp64 re-score (csrc/ewk_rescore.h).  A segment the float32 pass cannot decide alone is
// listed in a slot and its 8-frame chunks get consecutive part records; a launch after the
// scorer (k_rescore_linear / k_rescore_ring) claims the chunks with one atomic each (part
// record g -> its slot), each chunk's sums land in its part record, and the wave finishing a
// slot's last chunk combines them in chunk order.  A slot that finds the part pool full (or
// every slot of ewk_score_segments_f64) is serial: one wave runs its chunks in order.
constexpr int kRsFrames = 8;   // frames per re-score chunk
constexpr int kRsCtl = 8;      // ints of ScoreArgs::rs_ctl
constexpr int kRsMelW = 12;    // widest Slaney band of the basis in bins (fp64 mel window; checked at engine creation)
constexpr int kRsMelWLo = 3;   // widest of bands 0..63 (the fp64 path's window for a lane's low band; checked too)
struct RsSlot {
    int32_t seg;       // segment (linear) or event (ring) index
    int32_t T;         // frames
    int32_t nclaim;    // chunks (1 for a serial slot)
    int32_t base;      // first part record of the slot (pooled slots)
    int32_t pad;
    int32_t done;      // chunks finished (atomic; zeroed by the lister)
    float theta_s;     // speculative top_db clamp: the float32 pass's log-mel max - 80 dB
    int32_t serial;    // 1: one wave runs every chunk in order (no part records)
};
struct RsPart {                 // one chunk: per coefficient k, rA rB sA sB sAA sAB sBB ([7][20])
    double v[7 * 20];
    double mx;                  // log-mel max of the chunk's frames
    int32_t n;                  // frames
    int32_t flags;              // 1: a value within the ambiguity window of theta_s, 2: NaN
    int32_t slot;               // the slot this record belongs to (-1: a failed reservation)
    int32_t pad[3];
};
// Whole 128-B lines per record (1,152 B): the records of one slot are written at the same time
// by different waves into uncached memory, and records sharing a line lost bytes (round 4, a
// 1,184-B layout: a few wrong fp64 scores).
static_assert(sizeof(RsPart) % 128 == 0, "part records own their cache lines");

// Segment sources for the scorer.
//   linear: segment i = pcm[offsets[i] : offsets[i] + lengths[i]]
//   ring  : event i -> ring + stream*ring_len, first sample ring_start, wrap at ring_len
struct ScoreArgs {
    const float* pcm;
    const int16_t* pcm16;     // ring mode with an int16 ring (EWK_RING_I16): samples x 32768
    const int64_t* offsets;
    const int32_t* lengths;
    ewk_event* events;        // ring mode: read stream/ring_start/length, write score/match/flags
    const int32_t* n_events;  // ring mode: device-side event count
    const int32_t* ev_base;   // ring mode: first unscored event (watermark, count space)
    int32_t ev_base0;         // ring mode: the bank's epoch base (event slot = count - ev_base0, wrapping)
    int32_t* work;            // per-launch work counter (zeroed before the launch)
    int64_t ring_len;
    int32_t n_seg;            // linear mode count, ring mode capacity
    int32_t has_template;
    int32_t cand_f32;         // candidate dtype of the reference path: 1 float32, 0 float64
    const float* tmpl;        // [40] template mean[20], std[20]
    float uu_m32, uu_s32;     // template self-dots as numpy computes them (float32 sdot)
    float* out_mean;
    float* out_std;
    double* out_score;
    uint8_t* out_match;
    double threshold;
    double rescore_margin;
    int32_t* order;           // linear mode: work order scratch [n_seg] (longest first), nullptr = index order
    // fp64 re-score (nullptr rs_slots: none).  rs_ctl (kRsCtl ints): [0] slots listed,
    // [1] part records reserved, [2] serial slots listed, [3] workgroups out, [4] chunk claim
    // cursor, [5] serial claim cursor; the last workgroup out of the re-score launch zeroes
    // them (and *work) and, in ring mode, sets *adv_ev_base = *n_events.  The part records
    // live in uncached memory (hipDeviceMallocUncached): written by one wave and read by
    // another, on any XCD, with no L2 write-back or invalidate in between.
    int32_t* rs_ctl;
    RsSlot* rs_slots;
    int32_t* rs_serial;       // [rs_cap] serial slots, in listing order
    int32_t rs_cap;
    int32_t rs_part_cap;
    RsPart* rs_parts;
    int32_t list_all;         // every segment goes to the fp64 path (ewk_score_segments_f64)
    double* out_mean64;       // list_all: fp64 statistics [n][20]
    double* out_std64;
    int32_t* adv_ev_base;
    const struct Tables64* tab64;   // fp64 tables
    // ring mode poll mirror (nullptr: none): the last workgroup copies the bank's counters
    // (evc) and its first min(queued, mirror_chunk) events into pinned host memory
    unsigned char* mirror;
    const int32_t* evc;
    int32_t mirror_chunk;
};

// ring_mode: 0 linear batch, 1 ring events one segment per workgroup, 2 ring events one
// segment per wave (many events per tick)
hipError_t launch_score_f32(const Tables* d_tab, const ScoreArgs& a, int ring_mode, hipStream_t s);
// fp64 re-score of what a linear launch listed (ring launches drain their list themselves)
hipError_t launch_rescore_linear(const ScoreArgs& a, hipStream_t s);
hipError_t launch_rescore_ring(const ScoreArgs& a, hipStream_t s);
// streams from which a tick's events are scored one segment per wave (ring_mode 2)
constexpr int kRingWaveStreams = 65536;
// ScoreArgs::order holds n_seg indices followed by kLptScratch ints of bucket counters
constexpr int kLptScratch = 128;
hipError_t launch_snapshot(const int32_t* src, int32_t* dst, hipStream_t s);   // *dst = *src, stream-ordered
// counters + first min(queued, chunk) events of an event bank -> pinned host memory (poll mirror)
hipError_t launch_bank_mirror(const int32_t* evc, const ewk_event* ev, uint32_t base0, int32_t cap, int32_t chunk,
                              unsigned char* host, hipStream_t s);

constexpr int kScoreGridMax = 256;   // one resident workgroup wave of the grid
constexpr int kScoreGridRing = 256;                     // ring-mode grid (device-side event count)
int score_grid(int n_seg, int ring_mode);

// Level-3 pre-processing (ewk_level3.hip): segment i is pcm[offsets[i] ...][:lengths[i]]
// (linear) or the ring slice of events[i] (ring_len > 0); output at out[out_offsets[i]].
struct L3Args {
    const float* pcm;
    const int16_t* pcm16;        // ring mode with an int16 ring: samples x 32768
    const int64_t* offsets;
    const int32_t* lengths;
    const ewk_event* events;
    int64_t ring_len;            // 0 = linear
    const int64_t* out_offsets;
    double* out;
    int32_t n;
};
hipError_t launch_normalize(const L3Args& a, hipStream_t s);
hipError_t launch_decode_pcm16(const int16_t* in, float* out, int64_t n, hipStream_t s);

// ewk_gather.hip: positives compaction (scratch: 2 * compact_blocks(n) int32)
int compact_blocks(int32_t n);
hipError_t launch_compact_positives(const double* score, const uint8_t* match, int32_t n, int64_t first_id,
                                    int64_t step, ewk_positive* out, int32_t* d_count, int32_t* scratch, int append,
                                    hipStream_t s);

}  // namespace ewk
