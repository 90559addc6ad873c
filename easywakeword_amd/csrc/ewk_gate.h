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
    int32_t filled;          // block RMS cache valid
    int32_t reentries;
};

struct GateArgs {
    const float* pcm;        // stream s, tick t: pcm[s*stride + t*tick_stride + i]
    int64_t stride;
    int64_t tick_stride;
    int32_t n_ticks;
    int32_t n_streams;
    int64_t tick0;           // ticks already delivered
    float* ring;             // [n_streams][ring_len]
    int64_t ring_len;
    double* block_rms;       // [n_streams][n_blocks]
    GateStream* st;
    int32_t block;           // callback frame_size
    int32_t n_blocks;        // ring_len // block
    int64_t n_last;          // int(0.1 * sample_rate)
    int32_t sample_rate;
    int32_t lds_per_wave;
    double tick_seconds;
    double pre_speech_silence, speech_duration_min, speech_duration_max, post_speech_silence;
    double padding, max_segment_seconds, reentry_timeout, min_threshold;
    ewk_event* events;
    int32_t* ev_count;
    int32_t* ev_dropped;
    int32_t ev_cap;
};

hipError_t launch_gate(const GateArgs& g, hipStream_t s);
int gate_lds_per_wave(int n_blocks);

}  // namespace ewk
