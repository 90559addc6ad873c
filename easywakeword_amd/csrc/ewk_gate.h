// ewk_gate.h -- level-1 gate state and launch interface (internal).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ewk.h"

namespace ewk {

enum { kWaiting = 0, kInSilence = 1, kInSound = 2, kAfterSound = 3 };

// Per-stream state: SoundBuffer fields (wakeword.py:426-433) + _detect_word
// locals (wakeword.py:1048-1052), all float64 times on the virtual clock.
struct GateStream {
    int64_t collected;       // samples_collected (saturates at ring length)
    int64_t tick;            // last tick delivered
    double threshold;        // silence_threshold
    double last_rms;         // RMS of the last 0.1 s at the last tick
    double silence_start;
    double sound_start;
    double sound_end;
    double start_time;       // _detect_word start_time (re-entry timeout)
    int32_t pointer;
    int32_t state;
    int32_t started;
    int32_t last_silent;
    int32_t filled;          // block RMS cache + sorted copy valid
    int32_t reentries;
    int32_t sorted_sel;      // which of the two sorted_rms halves is current
    int32_t spos;            // write position in the sample ring (== pointer when it is the full ring)
};

// numpy's pairwise summation order (np.add.reduce on a contiguous float64 array,
// numpy/_core/src/umath/loops_utils.h.src pairwise_sum) for ONE chunk of n <= 8192
// elements, flattened on the host: leaves of <= 128 elements (8-accumulator loop),
// and the internal nodes grouped by height so a wave evaluates each level in parallel.
// Node ids: leaves 0..n_leaves-1, internal node k has id n_leaves + k.
constexpr int kPwChunk = 8192;
constexpr int kPwMaxLeaves = 256;
constexpr int kPwMaxLevels = 16;
struct PwTree {
    int32_t n;
    int32_t n_leaves;
    int32_t n_levels;
    int32_t balanced;   // 1: 2^d <= 16 leaves of one length >= 8, combined pairwise in leaf order (tree_sumsq's register path)
    int16_t leaf_start[kPwMaxLeaves];
    int16_t leaf_len[kPwMaxLeaves];
    int16_t left[kPwMaxLeaves];     // internal node k = val[left[k]] + val[right[k]]
    int16_t right[kPwMaxLeaves];
    int16_t level_end[kPwMaxLevels];   // internal nodes of height h+1: [level_end[h-1], level_end[h])
};
// The gate's summation lengths: the callback block (frame_size) and the last 0.1 s,
// each as a full-chunk tree (n = 8192, used when the length exceeds one chunk) and
// the tree of the final (or only) chunk.
enum { kTreeBlockFull = 0, kTreeBlockRem = 1, kTreeLastFull = 2, kTreeLastRem = 3, kNumTrees = 4 };
void build_pw_tree(int n, PwTree* t);

struct GateArgs {
    const float* pcm;        // stream s, tick t: pcm[s*stride + t*tick_stride + i]
    const int16_t* pcm16;    // or int16 PCM (same indexing), decoded as x / 32768 (exact)
    int64_t stride;
    int64_t tick_stride;
    int32_t n_ticks;
    int32_t n_streams;
    int64_t tick0;           // ticks already delivered
    float* ring;             // [n_streams][sring_len] sample rings (float32) ...
    int16_t* ring16;         // ... or int16 (EWK_RING_I16: PCM16 pushes stored as delivered)
    int64_t ring_len;        // the reference ring (buffer_seconds * sample_rate): blocks, pointer, fill
    int64_t sring_len;       // samples stored per stream (== ring_len, or a compact ring: see ewk_config.ring_samples)
    int32_t compact;         // sring_len < ring_len (block-aligned; block RMSs kept from the first write)
    int32_t pad0;
    double* block_rms;       // [n_streams][n_blocks] RMS of each physical block
    double* sorted_rms;      // [n_streams][2][n_blocks] the same values, ascending (double-buffered)
    GateStream* st;
    const PwTree* trees;     // kNumTrees
    int32_t block;           // callback frame_size
    int32_t n_blocks;        // ring_len // block
    int64_t n_last;          // int(0.1 * sample_rate)
    int32_t sample_rate;
    int32_t stage;           // per-wave LDS sample staging (floats); 0 = read the ring directly
    int32_t val_len;         // per-wave LDS doubles: tree node values (and the register path's sort scratch)
    double tick_seconds;
    double pre_speech_silence, speech_duration_min, speech_duration_max, post_speech_silence;
    double padding, max_segment_seconds, reentry_timeout, min_threshold;
    ewk_event* events;
    int32_t* ev_count;
    int32_t* ev_dropped;
    int32_t ev_cap;
    int32_t ev_base0;         // the bank's epoch base: event slot = count - ev_base0 (wrapping)
};

hipError_t launch_gate(const GateArgs& g, hipStream_t s);
hipError_t launch_reenter(GateStream* st, int32_t first, int32_t n, double tick_seconds, hipStream_t s);
// Zero a ring with agent-scope (sc1) stores: the lines go to memory and are dropped from the
// writing XCD's L2, so no cached copy of the initial zeros outlives the gate's first writes.
hipError_t launch_ring_zero(void* p, size_t bytes, hipStream_t s);
// register-resident block RMS arrays up to 64 * kGateRegMax blocks (10 s ring: block >= 313 samples)
constexpr int kGateRegMax = 8;
int gate_val_len(const PwTree* trees_host, int n_blocks);
// per-wave sample staging length for a config (0 when the lengths exceed the LDS budget)
int gate_stage_len(int block, int64_t n_last);

}  // namespace ewk
