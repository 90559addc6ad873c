/*
 * ewk.h -- C ABI of the MI355X-native EasyWakeWord hot path (levels 1 + 2).
 *
 * The reference has no FFI; its seams are Python duck types:
 *   - the WordMatcher protocol  (easywakeword/wakeword.py:520-639)
 *   - the SoundBuffer protocol  (easywakeword/wakeword.py:405-517)
 *   - the WakeWord._detect_word tick loop (easywakeword/wakeword.py:1036-1159)
 * Each entry point below names the reference interface it replaces.  The
 * Python facade (easywakeword_amd/wakeword.py) binds these with ctypes; the
 * binding a maintainer would add to the reference is shown in INTEGRATION.md.
 *
 * Conventions
 *   - every int-returning call returns EWK_OK (0) or a negative EWK_E* code;
 *     the message is in the thread-local ewk_last_error().  The facade maps
 *     EWK_EINVAL / EWK_ENOTEMPLATE to ValueError and the rest to RuntimeError.
 *   - the caller owns host arrays; the engine owns its device buffers and its
 *     HIP stream.  One engine per host thread; calls are not re-entrant per
 *     engine.
 *   - *_device entry points take device pointers (e.g. torch tensors'
 *     data_ptr()) and an optional hipStream_t (NULL = the engine's stream).
 */
#ifndef EWK_H
#define EWK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EWK_N_MFCC 20
#define EWK_ABI_VERSION 4

#define EWK_OK 0
#define EWK_EINVAL (-1)       /* bad parameter            -> ValueError            */
#define EWK_ENOTEMPLATE (-2)  /* no reference word set    -> ValueError (wakeword.py:608-609) */
#define EWK_EHIP (-3)         /* HIP runtime failure      -> RuntimeError          */
#define EWK_ENOMEM (-4)       /* allocation failure       -> MemoryError           */
#define EWK_ENODEV (-5)       /* no gfx950 device / bad device index -> RuntimeError */
#define EWK_EOVERWRITTEN (-6) /* ewk_normalize_events: an event's samples were overwritten in its
                                 ring since its tick -> RingOverwrittenError (a ValueError) */

/* event flags */
#define EWK_EV_SKIPPED 1      /* segment longer than max_segment_seconds: no level-2 call (wakeword.py:1113-1118) */
#define EWK_EV_RESCORED 2     /* score and decision from the fp64 path: the fp32 score fell inside
                                 rescore_margin, or the segment is very short (<= 16 frames), nearly
                                 stationary (|std| < 20) or has a vanishing MFCC mean (|mean| < 32,
                                 unless its similarity is negative beyond the fp32 error: NaN either way) */

/* ewk_score_segments* flags */
#define EWK_SCORE_REQUIRE_TEMPLATE 1   /* EWK_ENOTEMPLATE when no template (calculate_similarity) */
#define EWK_SCORE_F32_CANDIDATES 2     /* score with the reference's float32-candidate arithmetic
                                          (WordMatcher fed float32 audio); default: float64
                                          candidates, as SoundBuffer slices are (wakeword.py:428) */

/* ewk_config.ring_format */
#define EWK_RING_F32 0        /* float32 samples (any push)                                  */
#define EWK_RING_I16 1        /* int16 samples: PCM16 pushes only (ewk_push_pcm16 /
                                 ewk_push_many_pcm16), stored as delivered -- exact, half the
                                 HBM per stream; float32 pushes fail with EWK_EINVAL */

/* ewk_push flags */
#define EWK_PUSH_DEVICE 1     /* pcm is a device pointer */
#define EWK_PCM_DEVICE 1      /* input sample pointers are device memory (same bit as EWK_PUSH_DEVICE) */
#define EWK_OUT_DEVICE 4      /* output pointer is device memory (asynchronous where noted) */

typedef struct ewk_engine ewk_engine;

/* Defaults mirror the reference constants (wakeword.py:31-48, 405-431, 1100-1118). */
typedef struct ewk_config {
    int32_t sample_rate;          /* 16000  SoundBuffer.FREQUENCY                  */
    int32_t buffer_seconds;       /* 10     DEFAULT_BUFFER_SECONDS                 */
    int32_t block;                /* 1600   samples per callback == per tick       */
    int32_t ring_samples;         /* 0 = buffer_seconds * sample_rate (the reference ring).
                                     Otherwise samples kept per stream for segment reads: a
                                     compact ring with the same decisions and scores (block
                                     RMSs are kept per block as they arrive), for configs whose
                                     block divides the reference ring; must hold the longest
                                     possible segment request (max speech + post silence + one
                                     tick + padding) plus one tick, else EWK_EINVAL.  Saves HBM
                                     per stream (10 s -> 3 s: 640 KB -> 192 KB); ewk_read_last
                                     fails (EWK_EINVAL) for more than ring_samples. */
    double tick_seconds;          /* 0.1    time.sleep(0.1) in _detect_word        */
    double pre_speech_silence;    /* 0.8    DEFAULT_PRE_SPEECH_SILENCE             */
    double speech_duration_min;   /* 0.3    DEFAULT_SPEECH_DURATION_MIN            */
    double speech_duration_max;   /* 2.0    DEFAULT_SPEECH_DURATION_MAX            */
    double post_speech_silence;   /* 0.4    DEFAULT_POST_SPEECH_SILENCE            */
    double padding;               /* 0.05   wakeword.py:1101                       */
    double max_segment_seconds;   /* 3.0    wakeword.py:1115                       */
    double similarity_threshold;  /* 75.0   WakeWord(similarity_threshold=)        */
    double reentry_timeout;       /* <= 0: continuous; > 0: start()-mode re-entry every timeout s */
    double min_threshold;         /* 0.005  SoundBuffer.MIN_THRESHOLD              */
    double initial_threshold;     /* 0.01   SoundBuffer.silence_threshold init     */
    double rescore_margin;        /* 1e-3   |score - threshold| re-scored in fp64  */
    int32_t ring_format;          /* EWK_RING_F32 (default) or EWK_RING_I16                    */
    int32_t reserved1;
} ewk_config;

/* One level-1 pass (wakeword.py:1097-1124), with its level-2 result. */
typedef struct ewk_event {
    int32_t stream;
    int32_t length;               /* len(word_audio)                               */
    int64_t tick;                 /* virtual tick (time = tick * tick_seconds)     */
    int64_t ring_start;           /* first sample of the segment inside the stream ring */
    double time;
    double score;                 /* scaled similarity (NaN allowed)               */
    int32_t match;                /* score >= similarity_threshold                 */
    int32_t flags;                /* EWK_EV_*                                      */
} ewk_event;

/* Per-stream gate state snapshot (SoundBuffer + _detect_word locals). */
typedef struct ewk_stream_state {
    int64_t samples_collected;
    int64_t tick;
    double silence_threshold;
    double last_rms;
    double silence_start_time;
    double sound_start_time;
    double sound_end_time;
    double start_time;
    int32_t pointer;
    int32_t state;                /* 0 waiting, 1 in_silence, 2 in_sound, 3 after_sound */
    int32_t started;              /* detection running (ring filled once)          */
    int32_t last_silent;
} ewk_stream_state;

void ewk_default_config(ewk_config* cfg);
const char* ewk_last_error(void);
int ewk_abi_version(void);
/* number of visible HIP devices (0 when none); never fails */
int ewk_device_count(void);
/* Which HIP runtime this library's calls bind to: the file that defines the
 * hipLaunchKernel it resolved (dladdr) and hipRuntimeGetVersion (-1 if unavailable).
 * libewk.so links the system ROCm runtime (libamdhip64.so.7); a process that loaded
 * another copy first with RTLD_GLOBAL (PyTorch-ROCm wheels bundle one) binds that
 * copy instead -- then both libraries share ONE runtime and device pointers and
 * hipStream_t values pass between them.  Two runtimes that each own the device are
 * never in use at once. */
int ewk_runtime_info(char* path, int32_t cap, int32_t* hip_version);

/* Engine: device index, number of concurrent streams (0 = scorer only). */
int ewk_create(ewk_engine** out, int device, int32_t n_streams, const ewk_config* cfg);
void ewk_destroy(ewk_engine* e);
int ewk_sync(ewk_engine* e);
/* the engine's hipStream_t (as void*) */
void* ewk_stream_handle(ewk_engine* e);

/* ---- level 2: the matcher (WordMatcher, wakeword.py:520-639) ---------------- */

/* WordMatcher.set_reference(audio) (wakeword.py:569-578): template = MFCC
 * mean/std of `pcm` computed by the same HIP pipeline as every candidate. */
int ewk_template_from_pcm(ewk_engine* e, const float* pcm, int64_t n);
/* Direct template load (40 floats). */
int ewk_set_template(ewk_engine* e, const float* mean20, const float* std20);
/* Returns EWK_ENOTEMPLATE when none is set. */
int ewk_get_template(ewk_engine* e, float* mean20, float* std20);
/* WordMatcher.matches(audio, threshold) / WakeWord(similarity_threshold=) (wakeword.py:627-639, 676). */
int ewk_set_similarity_threshold(ewk_engine* e, double threshold);

/* WordMatcher.extract_mfcc + calculate_similarity + matches over a ragged
 * batch (wakeword.py:544-639).  Segment i is pcm[offsets[i] : offsets[i] +
 * lengths[i]].  Host buffers; any out_* may be NULL.  Without a template only
 * mean/std are produced (EWK_ENOTEMPLATE if flags has EWK_SCORE_REQUIRE_TEMPLATE). */
int ewk_score_segments(ewk_engine* e, const float* pcm, int64_t n_pcm,
                       const int64_t* offsets, const int32_t* lengths, int32_t n_seg,
                       float* out_mean, float* out_std, double* out_score, uint8_t* out_match,
                       int32_t flags);

/* Device-resident variant: every pointer is device memory; `stream` is a
 * hipStream_t (NULL = the engine stream).  Asynchronous; no host sync. */
int ewk_score_segments_device(ewk_engine* e, const float* d_pcm,
                              const int64_t* d_offsets, const int32_t* d_lengths, int32_t n_seg,
                              float* d_mean, float* d_std, double* d_score, uint8_t* d_match,
                              int32_t flags, void* stream);

/* fp64 reference-precision scorer (the rescoring path) on host buffers. */
int ewk_score_segments_f64(ewk_engine* e, const float* pcm, int64_t n_pcm,
                           const int64_t* offsets, const int32_t* lengths, int32_t n_seg,
                           double* out_mean, double* out_std, double* out_score, int32_t flags);

/* ---- level 1 + 2: the streaming gate (SoundBuffer + _detect_word) ------------ */

/* One tick for every stream: SoundBuffer._add_sound_to_buffer with a `block`
 * sample callback per stream (wakeword.py:454-486), then is_silent()
 * (wakeword.py:488-513) and one _detect_word FSM step (wakeword.py:1059-1118).
 * Stream s's samples are pcm[s*stride : s*stride + block].  Segments that pass
 * level 1 are scored on the device (level 2) and queued as events. */
int ewk_push(ewk_engine* e, const float* pcm, int64_t stride, int32_t flags);
/* Same for n_ticks consecutive ticks: tick t of stream s is
 * pcm[s*stride + t*tick_stride ...]. One launch sequence, no host sync. */
int ewk_push_many(ewk_engine* e, const float* pcm, int64_t stride, int64_t tick_stride,
                  int32_t n_ticks, int32_t flags);
/* int16 PCM variants (PortAudio / WAV PCM16 as delivered; decoded on the device as
 * x / 32768 -- exactly soundfile's / librosa.load's float32 -- halving ingest bytes). */
int ewk_push_pcm16(ewk_engine* e, const int16_t* pcm, int64_t stride, int32_t flags);
int ewk_push_many_pcm16(ewk_engine* e, const int16_t* pcm, int64_t stride, int64_t tick_stride,
                        int32_t n_ticks, int32_t flags);
/* Drain every queued event (waits for every push so far), sorted by (tick, stream).
 * If more than `cap` are queued nothing is consumed and EWK_EINVAL is returned (poll
 * again with a larger buffer).  If a bank overflowed (more than max(4096, 4 * n_streams)
 * events between polls) its events are dropped, the queue is re-armed so later pushes
 * keep working, and EWK_ENOMEM reports the loss. */
int ewk_poll(ewk_engine* e, ewk_event* out, int32_t cap, int32_t* n_out);
/* Pipelined drain: returns the events of the pushes made before the previous
 * ewk_poll_lagged call, without waiting for the pushes made since -- the GPU
 * keeps working on tick t while the host consumes tick t-1 (one call of latency). */
int ewk_poll_lagged(ewk_engine* e, ewk_event* out, int32_t cap, int32_t* n_out);
int ewk_get_stream_state(ewk_engine* e, int32_t stream, ewk_stream_state* out);
/* A new WakeWord._detect_word call (wakeword.py:1048-1057) on `stream` (-1 = all): for
 * streams whose detection runs, the FSM restarts from the current is_silent() with
 * start_time = now; `reentry_timeout` (<= 0: continuous, > 0: start()-mode re-entry
 * every reentry_timeout s) applies to every later push.  Stream-ordered, asynchronous. */
int ewk_reenter(ewk_engine* e, int32_t stream, double reentry_timeout);
/* SoundBuffer.return_last_n_seconds(n) (wakeword.py:498-513) as float32 (ring values are the float32 input). */
int ewk_read_last(ewk_engine* e, int32_t stream, int64_t n_samples, float* out, int64_t* n_out);
/* Copy the samples of a queued/polled event (ring must not have wrapped over it). */
int ewk_read_segment(ewk_engine* e, int32_t stream, int64_t ring_start, int32_t length, float* out);
/* Reset all stream state (ring, threshold, FSM, event queue). */
int ewk_reset_streams(ewk_engine* e);

/* ---- either side of the path --------------------------------------- */
/* Level-3 input: WakeWord._transcribe_audio's normalisation (wakeword.py:1019-1025)
 * y = x - mean(x); y /= max|y| if > 0; y *= 1.5; clip to [-1, 1], float64 and
 * bit-identical to numpy (pairwise mean), on the device.  Outputs are packed:
 * segment i starts at out[sum of the previous lengths].  out is host memory unless
 * flags has EWK_OUT_DEVICE.  Segments of a float32 batch (pcm host memory unless
 * EWK_PCM_DEVICE) ... */
int ewk_normalize_segments(ewk_engine* e, const float* pcm, int64_t n_pcm, const int64_t* offsets,
                           const int32_t* lengths, int32_t n_seg, double* out, int32_t flags);
/* ... or gated segments straight from the stream rings (polled events: stream,
 * ring_start, length), the reference's word_audio of each event. */
int ewk_normalize_events(ewk_engine* e, const ewk_event* events, int32_t n, double* out, int32_t flags);
/* Positives for the level-3 confirm gather (SURVEY.md 8b `ewk_gather_detections`, 8e):
 * the reference confirms every detection (wakeword.py:1120-1130); on N GPUs only the
 * positives cross xGMI.  Compacts the matched segments of a scored batch -- d_score /
 * d_match as ewk_score_segments_device wrote them -- into d_out (device memory,
 * capacity >= n, or >= *d_count + n with EWK_COMPACT_APPEND) in segment order, record
 * i = {first_id + segment index, score, step}, and leaves the count in *d_count (device
 * memory): no host sync, so a C/C++ host can hand d_out / d_count straight to its own
 * RCCL collective.  EWK_COMPACT_APPEND keeps the *d_count
 * records already there (K steps batched into one gather, the batch step of
 * easywakeword_amd.shard.MatchGather); otherwise *d_count is overwritten.
 * Asynchronous on `stream` (NULL = the engine's stream); the engine's scratch is shared,
 * so calls on different streams must be ordered by the caller. */
#define EWK_COMPACT_APPEND 1
typedef struct ewk_positive {
    int64_t id;                   /* first_id + index of the segment in its batch */
    double score;                 /* its scaled similarity (>= threshold) */
    int64_t step;                 /* caller's step tag (e.g. the batch number) */
} ewk_positive;
int ewk_compact_positives(ewk_engine* e, const double* d_score, const uint8_t* d_match, int32_t n,
                          int64_t first_id, int64_t step, ewk_positive* d_out, int32_t* d_count,
                          int32_t flags, void* stream);
/* WAV / PCM16 ingest (librosa.load of a 16 kHz PCM16 file = int16 / 32768 as float32):
 * host arrays unless EWK_PCM_DEVICE (then both are device memory, asynchronous). */
int ewk_decode_pcm16(ewk_engine* e, const int16_t* in, int64_t n, float* out, int32_t flags);

/* ---- measurement ------------------------------------------------------------ */
/* When enabled, every scorer / gate launch is bracketed by hipEvents on the
 * stream it runs on; ewk_profile_read resolves them (synchronizing) and returns
 * the summed device time and launch count per kernel family, then clears.
 * kind: 0 = fp32 MFCC scorer (k_score_f32), 1 = fp64 re-scorer, 2 = gate ticks. */
int ewk_profile_enable(ewk_engine* e, int32_t on);
int ewk_profile_read(ewk_engine* e, int32_t kind, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* EWK_H */
