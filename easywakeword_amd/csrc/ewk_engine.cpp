// ewk_engine.cpp -- the C ABI (include/ewk.h): engine lifetime, device memory,
// the level-2 batch scorer entry points and the level-1+2 streaming tick path.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "ewk_gate.h"
#include "ewk_internal.h"

using namespace ewk;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return fail(EWK_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));          \
    } while (0)

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;   // elements
    unsigned flags = 0;   // hipExtMallocWithFlags flags (0: hipMalloc)
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        hipError_t e = flags ? hipExtMallocWithFlags((void**)&p, bytes, flags) : hipMalloc(&p, bytes);
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

constexpr int kWorkInts = 32;          // ewk_engine::d_work
constexpr int32_t kPollChunk = 1024;   // events copied speculatively with the counters
constexpr size_t kPollRegion = 16 + (size_t)kPollChunk * sizeof(ewk_event);   // per bank: counters + chunk

// Scoped temporary device buffer (freed on return; callers synchronize before).
template <typename T>
struct TmpBuf : DevBuf<T> {
    ~TmpBuf() { this->release(); }
};

}  // namespace

struct ewk_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    ewk_config cfg{};
    int32_t n_streams = 0;
    int64_t ring_len = 0;           // the reference ring (buffer_seconds * sample_rate)
    int64_t sring_len = 0;          // samples stored per stream (ring_len, or cfg.ring_samples)
    int32_t n_blocks = 0;
    int64_t n_last = 0;

    Tables* d_tab = nullptr;
    Tables64* d_tab64 = nullptr;
    float* d_tmpl = nullptr;
    float h_tmpl[2 * NMFCC];
    float uu_m32 = 0.f, uu_s32 = 0.f;   // numpy float32 dot of the template with itself
    bool has_tmpl = false;

    // fp64 re-score (ewk_rescore.h): slots of listed segments and the chunk part pool, shared
    // by linear and ring launches (which never run concurrently: join_scoring)
    DevBuf<RsSlot> rs_slots;
    DevBuf<int32_t> rs_serial;      // serial slots of a launch
    DevBuf<RsPart> rs_parts;        // uncached (ScoreArgs::rs_ctl)
    int32_t rs_cap = 0;             // slots
    int32_t rs_part_cap = 0;        // part records (a slot that finds the pool full runs serially)
    // [0] linear work, [1] ring work, [4..5] event-count snapshots, [16..23] ring re-score
    // counters (ScoreArgs::rs_ctl), [24..31] linear re-score counters
    int32_t* d_work = nullptr;
    int32_t* d_compact = nullptr;   // ewk_compact_positives block counts / offsets
    int32_t compact_cap = 0;        // ... in blocks
    DevBuf<int32_t> order;          // linear batches: longest-first work order (k_lpt_order)

    // host-API staging
    DevBuf<float> pcm;
    DevBuf<int64_t> offsets;
    DevBuf<int32_t> lengths;
    DevBuf<float> mean, stdv;
    DevBuf<double> score;
    DevBuf<uint8_t> match;
    DevBuf<double> mean64, std64;

    // streaming
    void* d_ring = nullptr;         // float32 or int16 samples (cfg.ring_format)
    size_t ring_es = sizeof(float); // bytes per ring sample
    float* ring_f32() const { return ring_es == sizeof(float) ? static_cast<float*>(d_ring) : nullptr; }
    int16_t* ring_i16() const { return ring_es == sizeof(int16_t) ? static_cast<int16_t*>(d_ring) : nullptr; }
    double* d_brms = nullptr;
    double* d_sorted = nullptr;     // [streams][2][n_blocks] sorted block RMS (double-buffered)
    PwTree* d_trees = nullptr;      // numpy pairwise-sum trees for the block and the last 0.1 s
    GateStream* d_st = nullptr;
    // Two event banks (ev_cap events + 4 counters each: [0] count, [1] dropped,
    // [2] scored watermark): pushes append to `bank`; ewk_poll_lagged drains the
    // other bank while the GPU still works on this one.  The counters only grow (wrapping
    // uint32): a drained bank is re-armed by moving its epoch base to the count the host
    // read -- event i of an epoch is at slot count - base -- so no fill launch per tick.
    ewk_event* d_events = nullptr;   // [2][ev_cap]
    int32_t* d_evc = nullptr;        // [2][4]
    uint32_t ev_base0[2] = {0, 0};   // per bank: count at the start of the current epoch
    uint32_t drop_base0[2] = {0, 0}; // per bank: dropped count at the start of the epoch
    int32_t ev_cap = 0;
    int bank = 0;
    bool bank_used[2] = {false, false};
    hipEvent_t bank_done[2] = {nullptr, nullptr};   // recorded after the last push into a bank
    hipStream_t cstream = nullptr;                  // D2H copies of drained banks
    // Ring-mode scoring of tick t runs on sstream concurrently with the gate of tick t+1
    // on `stream` (the gate only overwrites ring samples older than any scorable segment;
    // see `overlap`).  At most one scoring pass is in flight beside a gate.
    hipStream_t sstream = nullptr;
    hipEvent_t gate_evt[2] = {nullptr, nullptr};
    hipEvent_t score_evt[2] = {nullptr, nullptr};
    bool score_live[2] = {false, false};
    hipEvent_t score_tail = nullptr;                // the latest recorded score_evt
    int64_t push_seq = 0;
    bool overlap = false;
    int32_t ticks_per_launch = 32;                  // gate launch length (segments must outlive it in the ring)
    ewk_event* ev_bank(int b) { return d_events + (size_t)b * ev_cap; }
    int32_t* evc_bank(int b) { return d_evc + 4 * b; }
    DevBuf<float> push_stage;
    float* h_stage = nullptr;       // pinned host staging for ewk_push / ewk_push_many
    unsigned char* h_poll = nullptr;   // pinned: event counters + the first kPollChunk events
    unsigned char* d_poll = nullptr;   // h_poll's device address (k_bank_mirror writes it)
    // mirror[b]: h_poll's region b holds bank b as of bank_done[b], written by k_bank_mirror
    // after the push's last scoring pass (same stream) -- the poll needs no copies
    bool mirror[2] = {false, false};
    size_t h_stage_cap = 0;
    hipEvent_t h_stage_free = nullptr;   // recorded after the last DMA out of h_stage
    int64_t tick = 0;
    int32_t gate_stage = 0;
    int32_t gate_val_len = 0;       // per-wave LDS doubles of the gate (tree values, sort scratch)

    // measurement: (start, stop) event pairs per kernel family
    bool prof = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[3];
    std::vector<hipEvent_t> ev_pool;
};

static hipEvent_t pool_event(ewk_engine* e) {
    if (!e->ev_pool.empty()) {
        hipEvent_t x = e->ev_pool.back();
        e->ev_pool.pop_back();
        return x;
    }
    hipEvent_t x = nullptr;
    if (hipEventCreate(&x) != hipSuccess) return nullptr;
    return x;
}

// RAII bracket: records start/stop events around one launch when profiling.
struct ProfScope {
    ewk_engine* e;
    int kind;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(ewk_engine* e_, int kind_, hipStream_t s_) : e(e_), kind(kind_), s(s_) {
        if (!e->prof) return;
        a = pool_event(e);
        b = pool_event(e);
        if (a) (void)hipEventRecord(a, s);
    }
    ~ProfScope() {
        if (!e->prof || !a || !b) return;
        (void)hipEventRecord(b, s);
        e->ev[kind].push_back({a, b});
    }
};

static void zero_event_state(ewk_engine* e) {
    if (e->d_evc) (void)hipMemsetAsync(e->d_evc, 0, 8 * sizeof(int32_t), e->stream);
    e->ev_base0[0] = e->ev_base0[1] = 0;
    e->drop_base0[0] = e->drop_base0[1] = 0;
    e->bank_used[0] = e->bank_used[1] = false;
    e->mirror[0] = e->mirror[1] = false;
}

static hipError_t ensure_poll_region(ewk_engine* e) {
    if (e->h_poll && e->d_poll) return hipSuccess;
    if (!e->h_poll) {
        hipError_t err = hipHostMalloc((void**)&e->h_poll, 2 * kPollRegion, hipHostMallocDefault);
        if (err != hipSuccess) { e->h_poll = nullptr; return err; }
    }
    hipError_t err = hipHostGetDevicePointer((void**)&e->d_poll, e->h_poll, 0);
    if (err != hipSuccess) {   // never leave a host region without its device alias (the mirror writes through it)
        (void)hipHostFree(e->h_poll);
        e->h_poll = nullptr;
        e->d_poll = nullptr;
    }
    return err;
}

// Order stream s after every ring-mode scoring pass enqueued so far (they run on
// sstream): needed before touching what those passes read or share -- the template,
// the re-score list, the log-mel and fp64 scratch, the event banks.
static hipError_t join_scoring(ewk_engine* e, hipStream_t s) {
    if (!e->overlap || !e->score_tail) return hipSuccess;
    return hipStreamWaitEvent(s, e->score_tail, 0);
}

// The re-score list holds at most one slot per segment of a launch (slots must start zeroed).
static hipError_t reserve_rescore(ewk_engine* e, int32_t n_seg) {
    if (n_seg <= e->rs_cap) return hipSuccess;
    hipError_t err = hipSuccess;
    if (e->stream) err = hipStreamSynchronize(e->stream);
    if (err == hipSuccess && e->sstream) err = hipStreamSynchronize(e->sstream);
    if (err != hipSuccess) return err;
    err = e->rs_slots.reserve((size_t)n_seg);
    if (err == hipSuccess) err = hipMemset(e->rs_slots.p, 0, (size_t)n_seg * sizeof(RsSlot));
    if (err == hipSuccess) err = e->rs_serial.reserve((size_t)n_seg);
    if (err != hipSuccess) return err;
    err = e->order.reserve((size_t)n_seg + kLptScratch);
    if (err != hipSuccess) return err;
    e->rs_cap = n_seg;
    return hipSuccess;
}

// Part records for the chunks of the slots listed in one launch (8 frames each).
static hipError_t reserve_parts(ewk_engine* e, int32_t n) {
    if (n <= e->rs_part_cap) return hipSuccess;
    hipError_t err = hipSuccess;
    if (e->stream) err = hipStreamSynchronize(e->stream);
    if (err == hipSuccess && e->sstream) err = hipStreamSynchronize(e->sstream);
    e->rs_parts.flags = hipDeviceMallocUncached;
    if (err == hipSuccess) err = e->rs_parts.reserve((size_t)n);
    if (err == hipSuccess) e->rs_part_cap = n;
    return err;
}

extern "C" {

void ewk_default_config(ewk_config* c) {
    memset(c, 0, sizeof(*c));
    c->sample_rate = 16000;
    c->buffer_seconds = 10;
    c->block = 1600;
    c->tick_seconds = 0.1;
    c->pre_speech_silence = 0.8;
    c->speech_duration_min = 0.3;
    c->speech_duration_max = 2.0;
    c->post_speech_silence = 0.4;
    c->padding = 0.05;
    c->max_segment_seconds = 3.0;
    c->similarity_threshold = 75.0;
    c->reentry_timeout = 0.0;
    c->min_threshold = 0.005;
    c->initial_threshold = 0.01;
    c->rescore_margin = 1e-3;
}

const char* ewk_last_error(void) { return g_err.c_str(); }
int ewk_abi_version(void) { return EWK_ABI_VERSION; }

int ewk_runtime_info(char* path, int32_t cap, int32_t* hip_version) {
    // the definition hipLaunchKernel resolved to for this library: with RTLD_GLOBAL
    // interposition (e.g. torch's bundled runtime loaded first) it is not the
    // libamdhip64.so.7 libewk.so was linked against
    Dl_info info;
    memset(&info, 0, sizeof(info));
    const void* sym = reinterpret_cast<const void*>(&hipLaunchKernel);
    if (!dladdr(sym, &info) || !info.dli_fname) return fail(EWK_EHIP, "dladdr(hipLaunchKernel) failed");
    if (path && cap > 0) {
        strncpy(path, info.dli_fname, (size_t)cap - 1);
        path[cap - 1] = 0;
    }
    if (hip_version) {
        int v = -1;
        if (hipRuntimeGetVersion(&v) != hipSuccess) v = -1;
        *hip_version = v;
    }
    return EWK_OK;
}

int ewk_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void ewk_destroy(ewk_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->sstream) (void)hipStreamSynchronize(e->sstream);
    (void)hipFree(e->d_tab);
    (void)hipFree(e->d_tab64);
    (void)hipFree(e->d_tmpl);
    e->rs_slots.release();
    e->rs_serial.release();
    e->rs_parts.release();
    (void)hipFree(e->d_work);
    (void)hipFree(e->d_compact);
    e->order.release();
    e->pcm.release();
    e->offsets.release();
    e->lengths.release();
    e->mean.release();
    e->stdv.release();
    e->score.release();
    e->match.release();
    e->mean64.release();
    e->std64.release();
    e->push_stage.release();
    (void)hipFree(e->d_ring);
    (void)hipFree(e->d_brms);
    (void)hipFree(e->d_sorted);
    (void)hipFree(e->d_trees);
    (void)hipFree(e->d_st);
    (void)hipFree(e->d_events);
    (void)hipFree(e->d_evc);
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    if (e->h_poll) (void)hipHostFree(e->h_poll);
    if (e->h_stage_free) (void)hipEventDestroy(e->h_stage_free);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->cstream) (void)hipStreamDestroy(e->cstream);
    if (e->sstream) (void)hipStreamDestroy(e->sstream);
    for (int b = 0; b < 2; ++b) {
        if (e->bank_done[b]) (void)hipEventDestroy(e->bank_done[b]);
        if (e->gate_evt[b]) (void)hipEventDestroy(e->gate_evt[b]);
        if (e->score_evt[b]) (void)hipEventDestroy(e->score_evt[b]);
    }
    delete e;
}

int ewk_reset_streams(ewk_engine* e);

int ewk_create(ewk_engine** out, int device, int32_t n_streams, const ewk_config* cfg) {
    if (!out) return fail(EWK_EINVAL, "out is NULL");
    *out = nullptr;
    ewk_config c;
    if (cfg) c = *cfg;
    else ewk_default_config(&c);
    if (c.sample_rate != 16000) return fail(EWK_EINVAL, "sample_rate must be 16000 (SoundBuffer.FREQUENCY)");
    if (c.buffer_seconds <= 0) return fail(EWK_EINVAL, "buffer_seconds must be positive");
    if (c.block <= 0 || c.block > 8192) return fail(EWK_EINVAL, "block must be in [1, 8192]");
    if (c.tick_seconds <= 0) return fail(EWK_EINVAL, "tick_seconds must be positive");
    if (c.pre_speech_silence <= 0) return fail(EWK_EINVAL, "pre_speech_silence must be positive");
    if (c.speech_duration_min <= 0) return fail(EWK_EINVAL, "speech_duration_min must be positive");
    if (c.speech_duration_max <= 0) return fail(EWK_EINVAL, "speech_duration_max must be positive");
    if (c.speech_duration_min > c.speech_duration_max)
        return fail(EWK_EINVAL, "speech_duration_min must be <= speech_duration_max");
    if (c.post_speech_silence <= 0) return fail(EWK_EINVAL, "post_speech_silence must be positive");
    if (n_streams < 0) return fail(EWK_EINVAL, "n_streams must be >= 0");
    if (c.ring_format != EWK_RING_F32 && c.ring_format != EWK_RING_I16)
        return fail(EWK_EINVAL, "ring_format must be EWK_RING_F32 or EWK_RING_I16");
    const int64_t ring_len = (int64_t)c.buffer_seconds * c.sample_rate;
    if (ring_len > INT32_MAX / 2) return fail(EWK_EINVAL, "buffer_seconds too large");
    // Longest segment request the cut can make (wakeword.py:1100-1111): nreq =
    // int(|sound_start - now - padding| * sr) with now - sound_start <= max speech +
    // (post silence rounded up to a tick), capped at the ring (return_last_n_seconds).
    const int64_t seg_need = std::min<int64_t>(
        ring_len, (int64_t)((c.speech_duration_max + c.post_speech_silence + c.tick_seconds + c.padding) *
                            (double)c.sample_rate) + 2);
    if (c.ring_samples != 0) {
        if (c.ring_samples < 0 || c.ring_samples > ring_len)
            return fail(EWK_EINVAL, "ring_samples must be in [0, buffer_seconds * sample_rate]");
        if (c.ring_samples < ring_len) {
            if (ring_len % c.block != 0 || c.ring_samples % c.block != 0)
                return fail(EWK_EINVAL, "a compact ring (ring_samples) needs block to divide both rings");
            if (gate_stage_len(c.block, (int64_t)(0.1 * (double)c.sample_rate)) < c.block)
                return fail(EWK_EINVAL, "a compact ring (ring_samples) needs block <= 4096");
            if (c.ring_samples < seg_need + c.block || c.ring_samples < (int64_t)(0.1 * (double)c.sample_rate))
                return fail(EWK_EINVAL, "ring_samples must hold the longest segment request plus one tick (" +
                                            std::to_string(seg_need + c.block) + " samples for this config)");
        }
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(EWK_ENODEV, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(EWK_ENODEV, "device index out of range");
    HIP_TRY(hipSetDevice(device));

    ewk_engine* e = new ewk_engine();
    e->device = device;
    e->cfg = c;
    e->n_streams = n_streams;
    e->ring_len = ring_len;
    e->sring_len = c.ring_samples > 0 ? (int64_t)c.ring_samples : ring_len;
    e->ring_es = c.ring_format == EWK_RING_I16 ? sizeof(int16_t) : sizeof(float);
    e->n_blocks = (int32_t)(e->ring_len / c.block);
    e->n_last = (int64_t)(0.1 * (double)c.sample_rate);   // int(0.1 * FREQUENCY)
    auto bail = [&](hipError_t err, const char* what) {
        std::string m = std::string(what) + ": " + hipGetErrorString(err);
        ewk_destroy(e);
        return fail(err == hipErrorOutOfMemory ? EWK_ENOMEM : EWK_EHIP, m);
    };
    hipError_t err;
    if ((err = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking)) != hipSuccess) return bail(err, "stream");
    if ((err = hipStreamCreateWithFlags(&e->cstream, hipStreamNonBlocking)) != hipSuccess) return bail(err, "stream");
    if ((err = hipStreamCreateWithFlags(&e->sstream, hipStreamNonBlocking)) != hipSuccess) return bail(err, "stream");
    for (int b = 0; b < 2; ++b) {
        if ((err = hipEventCreateWithFlags(&e->gate_evt[b], hipEventDisableTiming)) != hipSuccess) return bail(err, "event");
        if ((err = hipEventCreateWithFlags(&e->score_evt[b], hipEventDisableTiming)) != hipSuccess) return bail(err, "event");
    }
    for (int b = 0; b < 2; ++b)
        if ((err = hipEventCreateWithFlags(&e->bank_done[b], hipEventDisableTiming)) != hipSuccess)
            return bail(err, "event");
    {
        std::vector<unsigned char> buf(sizeof(Tables));
        Tables* t = reinterpret_cast<Tables*>(buf.data());
        build_tables(t);
        if (!t->ok) {
            ewk_destroy(e);
            return fail(EWK_EHIP, "mel filterbank does not fit the kernel's band layout");
        }
        if ((err = hipMalloc(&e->d_tab, sizeof(Tables))) != hipSuccess) return bail(err, "tables");
        if ((err = hipMemcpy(e->d_tab, t, sizeof(Tables), hipMemcpyHostToDevice)) != hipSuccess) return bail(err, "tables");
        std::vector<unsigned char> buf64(sizeof(Tables64));
        Tables64* t64 = reinterpret_cast<Tables64*>(buf64.data());
        build_tables64(t64);
        for (int m = 0; m < NMEL; ++m)
            if (t64->mel_off[m + 1] - t64->mel_off[m] > (m < NMEL / 2 ? kRsMelWLo : kRsMelW)) {
                ewk_destroy(e);
                return fail(EWK_EHIP, "mel filterbank band wider than the fp64 path's window (kRsMelWLo / kRsMelW)");
            }
        if ((err = hipMalloc(&e->d_tab64, sizeof(Tables64))) != hipSuccess) return bail(err, "tables64");
        if ((err = hipMemcpy(e->d_tab64, t64, sizeof(Tables64), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(err, "tables64");
    }
    if ((err = hipMalloc(&e->d_tmpl, 2 * NMFCC * sizeof(float))) != hipSuccess) return bail(err, "template");
    if ((err = reserve_rescore(e, 4096)) != hipSuccess) return bail(err, "rescore slots");
    if ((err = reserve_parts(e, 16384)) != hipSuccess) return bail(err, "rescore parts");
    if ((err = hipMalloc(&e->d_work, kWorkInts * sizeof(int32_t))) != hipSuccess) return bail(err, "work counter");
    if ((err = hipMemset(e->d_work, 0, kWorkInts * sizeof(int32_t))) != hipSuccess) return bail(err, "work counter");
    if (n_streams > 0) {
        const size_t ring_bytes = (size_t)n_streams * e->sring_len * e->ring_es;
        if ((err = hipMalloc(&e->d_ring, ring_bytes)) != hipSuccess) return bail(err, "ring");
        if ((err = hipMalloc(&e->d_brms, (size_t)n_streams * std::max(1, e->n_blocks) * sizeof(double))) != hipSuccess)
            return bail(err, "block rms");
        if ((err = hipMalloc(&e->d_sorted, (size_t)n_streams * 2 * std::max(1, e->n_blocks) * sizeof(double))) !=
            hipSuccess)
            return bail(err, "sorted block rms");
        if ((err = hipMalloc(&e->d_st, (size_t)n_streams * sizeof(GateStream))) != hipSuccess) return bail(err, "state");
        {
            std::vector<PwTree> tr(kNumTrees);
            const int64_t lens[2] = {c.block, e->n_last};
            for (int k = 0; k < 2; ++k) {
                const int64_t n = std::min<int64_t>(lens[k], e->ring_len);
                build_pw_tree(n > kPwChunk ? kPwChunk : 0, &tr[2 * k]);
                const int64_t r = n % kPwChunk;
                build_pw_tree((int)(n > kPwChunk ? (r ? r : kPwChunk) : n), &tr[2 * k + 1]);
            }
            if ((err = hipMalloc(&e->d_trees, kNumTrees * sizeof(PwTree))) != hipSuccess) return bail(err, "trees");
            if ((err = hipMemcpy(e->d_trees, tr.data(), kNumTrees * sizeof(PwTree), hipMemcpyHostToDevice)) != hipSuccess)
                return bail(err, "trees");
            e->gate_val_len = gate_val_len(tr.data(), e->n_blocks);
        }
        e->ev_cap = std::max(4096, 4 * n_streams);
        if ((err = reserve_rescore(e, e->ev_cap)) != hipSuccess) return bail(err, "rescore list");
        // a tick lists ~4 % of its events (the configs[2] recipe), ~20 chunks each
        if ((err = reserve_parts(e, std::min(262144, std::max(16384, e->ev_cap / 2)))) != hipSuccess)
            return bail(err, "rescore parts");
        if ((err = hipMalloc(&e->d_events, 2 * (size_t)e->ev_cap * sizeof(ewk_event))) != hipSuccess)
            return bail(err, "events");
        if ((err = hipMalloc(&e->d_evc, 8 * sizeof(int32_t))) != hipSuccess) return bail(err, "event counters");
        e->gate_stage = gate_stage_len(c.block, e->n_last);
        {   // A segment is cut at the tick that ends it and scored after its gate launch,
            // so the ticks of one launch after the cut must not reach its first sample:
            // ticks_per_launch <= (ring - longest request) / block (>= 1: a one-tick launch is
            // always safe, the cut never asks for more than the ring).  Overlapping the
            // scoring with the next gate launch doubles the ticks that may pass.
            const int64_t room = (e->sring_len - std::min(seg_need, e->sring_len)) / (int64_t)c.block;
            const int64_t tpl = std::max<int64_t>(1, std::min<int64_t>(32, room));
            const int64_t tpl_ov = std::min<int64_t>(32, room / 2);
            // opt-in (EWK_SCORE_OVERLAP=1): measured on MI355X the extra stream/event calls
            // per tick cost more host time than the concurrency saves (scripts/mb_stream.py)
            const char* env = getenv("EWK_SCORE_OVERLAP");
            e->overlap = tpl_ov >= 1 && env && env[0] == '1';
            e->ticks_per_launch = (int32_t)(e->overlap ? tpl_ov : tpl);
        }
        int rc = ewk_reset_streams(e);
        if (rc != EWK_OK) {
            std::string m = g_err;
            ewk_destroy(e);
            return fail(rc, m);
        }
    }
    if ((err = hipStreamSynchronize(e->stream)) != hipSuccess) return bail(err, "sync");
    *out = e;
    return EWK_OK;
}

int ewk_sync(ewk_engine* e) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipStreamSynchronize(e->sstream));
    return EWK_OK;
}

void* ewk_stream_handle(ewk_engine* e) { return e ? (void*)e->stream : nullptr; }

int ewk_set_template(ewk_engine* e, const float* mean20, const float* std20) {
    if (!e || !mean20 || !std20) return fail(EWK_EINVAL, "NULL argument");
    memcpy(e->h_tmpl, mean20, NMFCC * sizeof(float));
    memcpy(e->h_tmpl + NMFCC, std20, NMFCC * sizeof(float));
    {   // cblas_sdot for n = 20: float products accumulated in double, rounded to float
        double am = 0.0, as = 0.0;
        for (int i = 0; i < NMFCC; ++i) {
            const float pm = mean20[i] * mean20[i], ps = std20[i] * std20[i];
            am += (double)pm;
            as += (double)ps;
        }
        e->uu_m32 = (float)am;
        e->uu_s32 = (float)as;
    }
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(join_scoring(e, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_tmpl, e->h_tmpl, sizeof(e->h_tmpl), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->has_tmpl = true;
    return EWK_OK;
}

int ewk_set_similarity_threshold(ewk_engine* e, double threshold) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (!(threshold == threshold)) return fail(EWK_EINVAL, "threshold is NaN");
    e->cfg.similarity_threshold = threshold;
    return EWK_OK;
}

int ewk_get_template(ewk_engine* e, float* mean20, float* std20) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (!e->has_tmpl) return fail(EWK_ENOTEMPLATE, "No reference word set. Call set_reference() first.");
    if (mean20) memcpy(mean20, e->h_tmpl, NMFCC * sizeof(float));
    if (std20) memcpy(std20, e->h_tmpl + NMFCC, NMFCC * sizeof(float));
    return EWK_OK;
}

static ScoreArgs base_args(ewk_engine* e) {
    ScoreArgs a;
    memset(&a, 0, sizeof(a));
    a.has_template = e->has_tmpl ? 1 : 0;
    a.tmpl = e->d_tmpl;
    a.uu_m32 = e->uu_m32;
    a.uu_s32 = e->uu_s32;
    a.threshold = e->cfg.similarity_threshold;
    a.rescore_margin = e->cfg.rescore_margin;
    a.rs_ctl = e->d_work + 24;
    a.rs_slots = e->has_tmpl ? e->rs_slots.p : nullptr;
    a.rs_serial = e->rs_serial.p;
    a.rs_cap = e->rs_cap;
    a.rs_parts = e->rs_parts.p;
    a.rs_part_cap = e->rs_part_cap;
    a.tab64 = e->d_tab64;
    a.work = e->d_work;
    a.order = e->order.p;
    return a;
}

// f32 scorer + fp64 rescoring of the near-threshold list, all on `s`.
static int score_linear(ewk_engine* e, const float* d_pcm, const int64_t* d_off, const int32_t* d_len, int32_t n,
                        float* d_mean, float* d_std, double* d_score, uint8_t* d_match, int32_t flags,
                        hipStream_t s) {
    ScoreArgs a = base_args(e);
    a.cand_f32 = (flags & EWK_SCORE_F32_CANDIDATES) ? 1 : 0;
    a.pcm = d_pcm;
    a.offsets = d_off;
    a.lengths = d_len;
    a.n_seg = n;
    a.out_mean = d_mean;
    a.out_std = d_std;
    a.out_score = d_score;
    a.out_match = d_match;
    {   // (launch_score_f32 zeroes the work and re-score counters)
        ProfScope ps(e, 0, s);
        HIP_TRY(launch_score_f32(e->d_tab, a, 0, s));
    }
    {
        ProfScope ps(e, 1, s);
        HIP_TRY(launch_rescore_linear(a, s));
    }
    return EWK_OK;
}

int ewk_score_segments_device(ewk_engine* e, const float* d_pcm, const int64_t* d_offsets, const int32_t* d_lengths,
                              int32_t n_seg, float* d_mean, float* d_std, double* d_score, uint8_t* d_match,
                              int32_t flags, void* stream) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (n_seg < 0) return fail(EWK_EINVAL, "n_seg must be >= 0");
    if (n_seg == 0) return EWK_OK;
    if (!d_pcm || !d_offsets || !d_lengths) return fail(EWK_EINVAL, "NULL device pointer");
    if ((flags & EWK_SCORE_REQUIRE_TEMPLATE) && !e->has_tmpl)
        return fail(EWK_ENOTEMPLATE, "No reference word set. Call set_reference() first.");
    if (e->has_tmpl && !d_score) return fail(EWK_EINVAL, "d_score is required when a template is set");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(reserve_rescore(e, n_seg));
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    HIP_TRY(join_scoring(e, s));
    return score_linear(e, d_pcm, d_offsets, d_lengths, n_seg, d_mean, d_std, d_score, d_match, flags, s);
}

static int check_segments(const int64_t* offsets, const int32_t* lengths, int32_t n_seg, int64_t n_pcm,
                          int32_t* max_len) {
    int32_t mx = 0;
    for (int32_t i = 0; i < n_seg; ++i) {
        if (lengths[i] < 0 || offsets[i] < 0 || offsets[i] + lengths[i] > n_pcm)
            return fail(EWK_EINVAL, "segment " + std::to_string(i) + " out of range of pcm");
        mx = std::max(mx, lengths[i]);
    }
    *max_len = mx;
    return EWK_OK;
}

int ewk_score_segments(ewk_engine* e, const float* pcm, int64_t n_pcm, const int64_t* offsets,
                       const int32_t* lengths, int32_t n_seg, float* out_mean, float* out_std, double* out_score,
                       uint8_t* out_match, int32_t flags) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (n_seg < 0 || n_pcm < 0) return fail(EWK_EINVAL, "negative size");
    if ((flags & EWK_SCORE_REQUIRE_TEMPLATE) && !e->has_tmpl)
        return fail(EWK_ENOTEMPLATE, "No reference word set. Call set_reference() first.");
    if (n_seg == 0) return EWK_OK;
    if (!offsets || !lengths || (n_pcm > 0 && !pcm)) return fail(EWK_EINVAL, "NULL argument");
    int32_t max_len = 0;
    int rc = check_segments(offsets, lengths, n_seg, n_pcm, &max_len);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(reserve_rescore(e, n_seg));
    HIP_TRY(e->pcm.reserve(std::max<int64_t>(n_pcm, 1)));
    HIP_TRY(e->offsets.reserve(n_seg));
    HIP_TRY(e->lengths.reserve(n_seg));
    HIP_TRY(e->mean.reserve((size_t)n_seg * NMFCC));
    HIP_TRY(e->stdv.reserve((size_t)n_seg * NMFCC));
    HIP_TRY(e->score.reserve(n_seg));
    HIP_TRY(e->match.reserve(n_seg));
    hipStream_t s = e->stream;
    HIP_TRY(join_scoring(e, s));
    if (n_pcm > 0) HIP_TRY(hipMemcpyAsync(e->pcm.p, pcm, n_pcm * sizeof(float), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->offsets.p, offsets, n_seg * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->lengths.p, lengths, n_seg * sizeof(int32_t), hipMemcpyHostToDevice, s));
    {
        ScoreArgs a = base_args(e);
        a.pcm = e->pcm.p;
        a.offsets = e->offsets.p;
        a.lengths = e->lengths.p;
        a.n_seg = n_seg;
        a.out_mean = e->mean.p;
        a.out_std = e->stdv.p;
        a.out_score = e->score.p;
        a.out_match = e->match.p;
        a.cand_f32 = (flags & EWK_SCORE_F32_CANDIDATES) ? 1 : 0;
        HIP_TRY(launch_score_f32(e->d_tab, a, 0, s));   // (zeroes the work and re-score counters)
        HIP_TRY(launch_rescore_linear(a, s));
    }
    if (out_mean) HIP_TRY(hipMemcpyAsync(out_mean, e->mean.p, (size_t)n_seg * NMFCC * 4, hipMemcpyDeviceToHost, s));
    if (out_std) HIP_TRY(hipMemcpyAsync(out_std, e->stdv.p, (size_t)n_seg * NMFCC * 4, hipMemcpyDeviceToHost, s));
    if (e->has_tmpl) {
        if (out_score) HIP_TRY(hipMemcpyAsync(out_score, e->score.p, n_seg * sizeof(double), hipMemcpyDeviceToHost, s));
        if (out_match) HIP_TRY(hipMemcpyAsync(out_match, e->match.p, n_seg, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return EWK_OK;
}

int ewk_score_segments_f64(ewk_engine* e, const float* pcm, int64_t n_pcm, const int64_t* offsets,
                           const int32_t* lengths, int32_t n_seg, double* out_mean, double* out_std,
                           double* out_score, int32_t flags) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (n_seg < 0 || n_pcm < 0) return fail(EWK_EINVAL, "negative size");
    if (n_seg == 0) return EWK_OK;
    if (!offsets || !lengths || (n_pcm > 0 && !pcm)) return fail(EWK_EINVAL, "NULL argument");
    int32_t max_len = 0;
    int rc = check_segments(offsets, lengths, n_seg, n_pcm, &max_len);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    HIP_TRY(join_scoring(e, s));
    HIP_TRY(reserve_rescore(e, n_seg));
    HIP_TRY(e->pcm.reserve(std::max<int64_t>(n_pcm, 1)));
    HIP_TRY(e->offsets.reserve(n_seg));
    HIP_TRY(e->lengths.reserve(n_seg));
    HIP_TRY(e->mean64.reserve((size_t)n_seg * NMFCC));
    HIP_TRY(e->std64.reserve((size_t)n_seg * NMFCC));
    HIP_TRY(e->score.reserve(n_seg));
    if (n_pcm > 0) HIP_TRY(hipMemcpyAsync(e->pcm.p, pcm, n_pcm * sizeof(float), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->offsets.p, offsets, n_seg * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->lengths.p, lengths, n_seg * sizeof(int32_t), hipMemcpyHostToDevice, s));
    ScoreArgs a = base_args(e);
    a.pcm = e->pcm.p;
    a.offsets = e->offsets.p;
    a.lengths = e->lengths.p;
    a.n_seg = n_seg;
    a.out_score = e->score.p;
    a.cand_f32 = (flags & EWK_SCORE_F32_CANDIDATES) ? 1 : 0;
    // every segment through the fp64 path: the float32 pass only supplies the speculative
    // top_db clamp of each segment (its own scores are overwritten)
    a.list_all = 1;
    a.rs_slots = e->rs_slots.p;
    a.out_mean64 = e->mean64.p;
    a.out_std64 = e->std64.p;
    HIP_TRY(launch_score_f32(e->d_tab, a, 0, s));
    HIP_TRY(launch_rescore_linear(a, s));
    if (out_mean) HIP_TRY(hipMemcpyAsync(out_mean, e->mean64.p, (size_t)n_seg * NMFCC * 8, hipMemcpyDeviceToHost, s));
    if (out_std) HIP_TRY(hipMemcpyAsync(out_std, e->std64.p, (size_t)n_seg * NMFCC * 8, hipMemcpyDeviceToHost, s));
    if (out_score && e->has_tmpl)
        HIP_TRY(hipMemcpyAsync(out_score, e->score.p, n_seg * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return EWK_OK;
}

int ewk_template_from_pcm(ewk_engine* e, const float* pcm, int64_t n) {
    if (!e || (!pcm && n > 0)) return fail(EWK_EINVAL, "NULL argument");
    if (n <= 0 || n > INT32_MAX) return fail(EWK_EINVAL, "template length must be in [1, 2^31)");
    const int64_t off = 0;
    const int32_t len = (int32_t)n;
    float m[NMFCC], sd[NMFCC];
    const bool had = e->has_tmpl;
    e->has_tmpl = false;   // compute stats only
    int rc = ewk_score_segments(e, pcm, n, &off, &len, 1, m, sd, nullptr, nullptr, EWK_SCORE_F32_CANDIDATES);
    e->has_tmpl = had;
    if (rc) return rc;
    return ewk_set_template(e, m, sd);
}

// ---------------------------------------------------------------- streaming path
int ewk_reset_streams(ewk_engine* e) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (e->n_streams <= 0) return EWK_OK;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    HIP_TRY(join_scoring(e, s));
#ifndef EWK_RING_MEMSET
    HIP_TRY(launch_ring_zero(e->d_ring, (size_t)e->n_streams * e->sring_len * e->ring_es, s));
#else   // (the round-6 fill, kept for the A/B of scripts/gpu_miss_prefix.sh)
    HIP_TRY(hipMemsetAsync(e->d_ring, 0, (size_t)e->n_streams * e->sring_len * e->ring_es, s));
#endif
    HIP_TRY(hipMemsetAsync(e->d_brms, 0, (size_t)e->n_streams * std::max(1, e->n_blocks) * sizeof(double), s));
    std::vector<GateStream> st(e->n_streams);
    for (auto& x : st) {
        memset(&x, 0, sizeof(x));
        x.threshold = e->cfg.initial_threshold;
        x.last_silent = 1;
    }
    HIP_TRY(hipMemcpyAsync(e->d_st, st.data(), st.size() * sizeof(GateStream), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(e->d_work, 0, kWorkInts * sizeof(int32_t), s));
    zero_event_state(e);
    HIP_TRY(hipStreamSynchronize(s));
    e->tick = 0;
    return EWK_OK;
}

// Score the events queued since the last scoring pass (ring mode), then advance the watermark.
// Score the current bank's events [ev_base, *n_events) on stream ss; n_events is the
// live counter (same stream as the gate) or a snapshot of it taken after the gate.
static int score_pending(ewk_engine* e, hipStream_t ss, const int32_t* n_events) {
    if (!e->has_tmpl) return EWK_OK;   // events keep NaN scores until a template exists
    ScoreArgs a = base_args(e);
    a.pcm = e->ring_f32();
    a.pcm16 = e->ring_i16();
    a.ring_len = e->sring_len;
    a.events = e->ev_bank(e->bank);
    a.n_events = n_events;
    a.ev_base = e->evc_bank(e->bank) + 2;
    a.ev_base0 = e->ev_base0[e->bank];
    a.n_seg = e->ev_cap;
    a.work = e->d_work + 1;            // ring-mode counters (zeroed at create, re-armed by the tick end)
    a.rs_ctl = e->d_work + 16;
    // k_rescore_ring (after the scorer) re-scores the listed segments in fp64 and its last
    // workgroup out advances the watermark and writes the poll mirror
    a.adv_ev_base = e->evc_bank(e->bank) + 2;
    HIP_TRY(ensure_poll_region(e));
    a.mirror = e->d_poll + e->bank * kPollRegion;
    a.evc = e->evc_bank(e->bank);
    a.mirror_chunk = std::min<int32_t>(kPollChunk, e->ev_cap);
    {
        ProfScope ps(e, 0, ss);
        HIP_TRY(launch_score_f32(e->d_tab, a, e->n_streams >= kRingWaveStreams ? 2 : 1, ss));
    }
    {
        ProfScope ps(e, 1, ss);
        HIP_TRY(launch_rescore_ring(a, ss));
    }
    return EWK_OK;
}

static int push_impl(ewk_engine* e, const void* pcm_any, int64_t stride, int64_t tick_stride, int32_t n_ticks,
                     int32_t flags, bool pcm16) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (e->n_streams <= 0) return fail(EWK_EINVAL, "engine has no streams");
    if (!pcm_any) return fail(EWK_EINVAL, "pcm is NULL");
    if (n_ticks <= 0) return fail(EWK_EINVAL, "n_ticks must be positive");
    if (!pcm16 && e->ring_es == sizeof(int16_t))
        return fail(EWK_EINVAL, "an int16 ring (EWK_RING_I16) takes PCM16 pushes (ewk_push_pcm16)");
    const size_t es = pcm16 ? sizeof(int16_t) : sizeof(float);
    const unsigned char* pcm = static_cast<const unsigned char*>(pcm_any);
    if (stride < e->cfg.block && e->n_streams > 1) return fail(EWK_EINVAL, "stride must be >= block");
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    const void* src = pcm_any;
    int64_t st_stride = stride, tk_stride = tick_stride;
    if (!(flags & EWK_PUSH_DEVICE)) {
        // Gather the caller's (pageable) blocks into pinned staging on the CPU, then
        // DMA asynchronously: the caller's buffer may die as soon as we return.
        const size_t per_stream = (size_t)n_ticks * e->cfg.block;
        const size_t total = per_stream * e->n_streams;
        if (e->h_stage_free) HIP_TRY(hipEventSynchronize(e->h_stage_free));   // previous DMA done
        if (total > e->h_stage_cap) {
            if (e->h_stage) HIP_TRY(hipHostFree(e->h_stage));
            e->h_stage = nullptr;
            e->h_stage_cap = 0;
            HIP_TRY(hipHostMalloc((void**)&e->h_stage, total * sizeof(float), hipHostMallocDefault));   // >= es bytes each
            e->h_stage_cap = total;
        }
        if (!e->h_stage_free) HIP_TRY(hipEventCreateWithFlags(&e->h_stage_free, hipEventDisableTiming));
        for (int32_t st = 0; st < e->n_streams; ++st)
            for (int32_t t = 0; t < n_ticks; ++t)
                memcpy(reinterpret_cast<unsigned char*>(e->h_stage) + ((size_t)st * per_stream + (size_t)t * e->cfg.block) * es,
                       pcm + ((size_t)st * stride + (size_t)t * tick_stride) * es, e->cfg.block * es);
        HIP_TRY(e->push_stage.reserve(total));
        HIP_TRY(hipMemcpyAsync(e->push_stage.p, e->h_stage, total * es, hipMemcpyHostToDevice, s));
        HIP_TRY(hipEventRecord(e->h_stage_free, s));
        src = e->push_stage.p;
        st_stride = (int64_t)per_stream;
        tk_stride = e->cfg.block;
    }
    // Segments must be scored before the ring overwrites them: <= ticks_per_launch ticks per gate launch.
    for (int32_t t0 = 0; t0 < n_ticks; t0 += e->ticks_per_launch) {
        const int32_t nt = std::min<int32_t>(e->ticks_per_launch, n_ticks - t0);
        GateArgs g;
        memset(&g, 0, sizeof(g));
        if (pcm16) g.pcm16 = static_cast<const int16_t*>(src) + (int64_t)t0 * tk_stride;
        else g.pcm = static_cast<const float*>(src) + (int64_t)t0 * tk_stride;
        g.stride = st_stride;
        g.tick_stride = tk_stride;
        g.n_ticks = nt;
        g.n_streams = e->n_streams;
        g.tick0 = e->tick;
        g.ring = e->ring_f32();
        g.ring16 = e->ring_i16();
        g.ring_len = e->ring_len;
        g.sring_len = e->sring_len;
        g.compact = e->sring_len < e->ring_len ? 1 : 0;
        g.block_rms = e->d_brms;
        g.sorted_rms = e->d_sorted;
        g.trees = e->d_trees;
        g.st = e->d_st;
        g.block = e->cfg.block;
        g.n_blocks = e->n_blocks;
        g.n_last = e->n_last;
        g.sample_rate = e->cfg.sample_rate;
        g.stage = e->gate_stage;
        g.val_len = e->gate_val_len;
        g.tick_seconds = e->cfg.tick_seconds;
        g.pre_speech_silence = e->cfg.pre_speech_silence;
        g.speech_duration_min = e->cfg.speech_duration_min;
        g.speech_duration_max = e->cfg.speech_duration_max;
        g.post_speech_silence = e->cfg.post_speech_silence;
        g.padding = e->cfg.padding;
        g.max_segment_seconds = e->cfg.max_segment_seconds;
        g.reentry_timeout = e->cfg.reentry_timeout;
        g.min_threshold = e->cfg.min_threshold;
        g.events = e->ev_bank(e->bank);
        g.ev_count = e->evc_bank(e->bank);
        g.ev_dropped = e->evc_bank(e->bank) + 1;
        g.ev_cap = e->ev_cap;
        g.ev_base0 = e->ev_base0[e->bank];
        const int k = (int)(e->push_seq & 1);
        // the scoring pass two launches back must be done: it read snapshot slot k, and
        // at most one pass runs beside a gate
        if (e->overlap && e->score_live[k]) HIP_TRY(hipStreamWaitEvent(s, e->score_evt[k], 0));
        {
            ProfScope ps(e, 2, s);
            HIP_TRY(launch_gate(g, s));
        }
        e->tick += nt;
        if (e->overlap) {
            int32_t* snap = e->d_work + 4 + k;
            HIP_TRY(launch_snapshot(e->evc_bank(e->bank), snap, s));
            HIP_TRY(hipEventRecord(e->gate_evt[k], s));
            HIP_TRY(hipStreamWaitEvent(e->sstream, e->gate_evt[k], 0));
            int rc = score_pending(e, e->sstream, snap);
            if (rc) return rc;
            HIP_TRY(hipEventRecord(e->score_evt[k], e->sstream));
            e->score_live[k] = true;
            e->score_tail = e->score_evt[k];
        } else {
            int rc = score_pending(e, s, e->evc_bank(e->bank));
            if (rc) return rc;
        }
        e->push_seq += 1;
    }
    // the poll mirror of this bank: written by the last scoring pass's tick end, or (no template
    // yet: no scoring pass) by k_bank_mirror behind the gate
    if (!e->has_tmpl) {
        hipStream_t ms = e->overlap ? e->sstream : s;
        HIP_TRY(ensure_poll_region(e));
        HIP_TRY(launch_bank_mirror(e->evc_bank(e->bank), e->ev_bank(e->bank), e->ev_base0[e->bank], e->ev_cap,
                                   std::min<int32_t>(kPollChunk, e->ev_cap), e->d_poll + e->bank * kPollRegion, ms));
    }
    e->mirror[e->bank] = true;
    HIP_TRY(hipEventRecord(e->bank_done[e->bank], e->overlap ? e->sstream : s));
    e->bank_used[e->bank] = true;
    return EWK_OK;
}

int ewk_push(ewk_engine* e, const float* pcm, int64_t stride, int32_t flags) {
    return push_impl(e, pcm, stride, 0, 1, flags, false);
}

int ewk_push_many(ewk_engine* e, const float* pcm, int64_t stride, int64_t tick_stride, int32_t n_ticks,
                  int32_t flags) {
    return push_impl(e, pcm, stride, tick_stride, n_ticks, flags, false);
}

int ewk_push_pcm16(ewk_engine* e, const int16_t* pcm, int64_t stride, int32_t flags) {
    return push_impl(e, pcm, stride, 0, 1, flags, true);
}

int ewk_push_many_pcm16(ewk_engine* e, const int16_t* pcm, int64_t stride, int64_t tick_stride, int32_t n_ticks,
                        int32_t flags) {
    return push_impl(e, pcm, stride, tick_stride, n_ticks, flags, true);
}

// ---------------------------------------------------------------- level-3 input / PCM16 decode
static int normalize_impl(ewk_engine* e, const float* d_pcm, const int64_t* offsets, const int32_t* lengths,
                          const ewk_event* events, int32_t n, double* out, int32_t flags) {
    hipStream_t s = e->stream;
    HIP_TRY(join_scoring(e, s));
    std::vector<int64_t> oo(n);
    int64_t total = 0;
    for (int32_t i = 0; i < n; ++i) {
        const int32_t len = events ? events[i].length : lengths[i];
        if (len < 0) return fail(EWK_EINVAL, "negative segment length");
        oo[i] = total;
        total += len;
    }
    TmpBuf<int64_t> d_oo, d_off;
    TmpBuf<int32_t> d_len;
    TmpBuf<ewk_event> d_ev;
    TmpBuf<double> d_out;
    HIP_TRY(d_oo.reserve(std::max<int32_t>(1, n)));
    HIP_TRY(hipMemcpyAsync(d_oo.p, oo.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, s));
    L3Args a;
    memset(&a, 0, sizeof(a));
    a.n = n;
    a.out_offsets = d_oo.p;
    if (events) {
        HIP_TRY(d_ev.reserve(std::max<int32_t>(1, n)));
        HIP_TRY(hipMemcpyAsync(d_ev.p, events, n * sizeof(ewk_event), hipMemcpyHostToDevice, s));
        a.events = d_ev.p;
        a.pcm = e->ring_f32();
        a.pcm16 = e->ring_i16();
        a.ring_len = e->sring_len;
    } else {
        HIP_TRY(d_off.reserve(std::max<int32_t>(1, n)));
        HIP_TRY(d_len.reserve(std::max<int32_t>(1, n)));
        HIP_TRY(hipMemcpyAsync(d_off.p, offsets, n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_len.p, lengths, n * sizeof(int32_t), hipMemcpyHostToDevice, s));
        a.pcm = d_pcm;
        a.offsets = d_off.p;
        a.lengths = d_len.p;
    }
    if (flags & EWK_OUT_DEVICE) {
        a.out = out;
    } else {
        HIP_TRY(d_out.reserve(std::max<int64_t>(1, total)));
        a.out = d_out.p;
    }
    HIP_TRY(launch_normalize(a, s));
    if (!(flags & EWK_OUT_DEVICE) && total > 0)
        HIP_TRY(hipMemcpyAsync(out, d_out.p, total * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return EWK_OK;
}

int ewk_normalize_segments(ewk_engine* e, const float* pcm, int64_t n_pcm, const int64_t* offsets,
                           const int32_t* lengths, int32_t n_seg, double* out, int32_t flags) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (n_seg < 0 || n_pcm < 0) return fail(EWK_EINVAL, "negative size");
    if (n_seg == 0) return EWK_OK;
    if (!pcm || !offsets || !lengths || !out) return fail(EWK_EINVAL, "NULL argument");
    for (int32_t i = 0; i < n_seg; ++i)
        if (offsets[i] < 0 || lengths[i] < 0 || offsets[i] + lengths[i] > n_pcm)
            return fail(EWK_EINVAL, "segment " + std::to_string(i) + " outside pcm");
    HIP_TRY(hipSetDevice(e->device));
    const float* d_pcm = pcm;
    TmpBuf<float> tmp;
    if (!(flags & EWK_PCM_DEVICE)) {
        HIP_TRY(tmp.reserve(std::max<int64_t>(1, n_pcm)));
        HIP_TRY(hipMemcpyAsync(tmp.p, pcm, n_pcm * sizeof(float), hipMemcpyHostToDevice, e->stream));
        d_pcm = tmp.p;
    }
    return normalize_impl(e, d_pcm, offsets, lengths, nullptr, n_seg, out, flags);
}

int ewk_normalize_events(ewk_engine* e, const ewk_event* events, int32_t n, double* out, int32_t flags) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (n < 0) return fail(EWK_EINVAL, "negative size");
    if (n == 0) return EWK_OK;
    if (!events || !out) return fail(EWK_EINVAL, "NULL argument");
    if (e->n_streams <= 0) return fail(EWK_EINVAL, "engine has no streams");
    for (int32_t i = 0; i < n; ++i) {
        const ewk_event& ev = events[i];
        if (ev.stream < 0 || ev.stream >= e->n_streams || ev.length < 0 || ev.length > e->sring_len ||
            ev.ring_start < 0 || ev.ring_start >= e->sring_len)
            return fail(EWK_EINVAL, "event " + std::to_string(i) + " outside the rings");
        // The segment is the last nreq >= length samples before the write position of its
        // tick (ewk_gate.hip, the cut), and every later tick writes one block: it is intact
        // while nreq + (ticks since) * block <= ring.  (The write position after tick k is
        // k * block mod ring for every stream.)
        const int64_t Rs = e->sring_len, blk = e->cfg.block;
        if (ev.tick < 0 || ev.tick > e->tick)
            return fail(EWK_EINVAL, "event " + std::to_string(i) + " is from a tick this engine has not pushed");
        int64_t nreq = ((ev.tick % Rs) * (blk % Rs) % Rs - ev.ring_start) % Rs;
        if (nreq < 0) nreq += Rs;
        if (nreq == 0 && ev.length > 0) nreq = Rs;
        if (nreq + (e->tick - ev.tick) * blk > Rs)
            return fail(EWK_EOVERWRITTEN, "event " + std::to_string(i) + " (tick " + std::to_string(ev.tick) +
                                        "): the ring has overwritten its samples since (now tick " +
                                        std::to_string(e->tick) + "); read positives right after their poll");
    }
    HIP_TRY(hipSetDevice(e->device));
    return normalize_impl(e, nullptr, nullptr, nullptr, events, n, out, flags);
}

int ewk_compact_positives(ewk_engine* e, const double* d_score, const uint8_t* d_match, int32_t n, int64_t first_id,
                          int64_t step, ewk_positive* d_out, int32_t* d_count, int32_t flags, void* stream) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (n < 0) return fail(EWK_EINVAL, "negative size");
    if (!d_count || (n > 0 && (!d_score || !d_match || !d_out))) return fail(EWK_EINVAL, "NULL argument");
    if (flags & ~EWK_COMPACT_APPEND) return fail(EWK_EINVAL, "unknown flags");
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    const int nb = std::max(1, compact_blocks(n));
    if (nb > e->compact_cap) {   // grown rarely (stream-ordered: the old scratch may be in use)
        HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(e->d_compact);
        e->d_compact = nullptr;
        e->compact_cap = 0;
        HIP_TRY(hipMalloc(&e->d_compact, 2 * (size_t)nb * sizeof(int32_t)));
        e->compact_cap = nb;
    }
    HIP_TRY(launch_compact_positives(d_score, d_match, n, first_id, step, d_out, d_count, e->d_compact,
                                     (flags & EWK_COMPACT_APPEND) ? 1 : 0, s));
    return EWK_OK;
}

int ewk_decode_pcm16(ewk_engine* e, const int16_t* in, int64_t n, float* out, int32_t flags) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (n < 0) return fail(EWK_EINVAL, "negative size");
    if (n == 0) return EWK_OK;
    if (!in || !out) return fail(EWK_EINVAL, "NULL argument");
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    if (flags & EWK_PCM_DEVICE) {   // both pointers device memory; asynchronous
        HIP_TRY(launch_decode_pcm16(in, out, n, s));
        return EWK_OK;
    }
    TmpBuf<int16_t> d_in;
    TmpBuf<float> d_out;
    HIP_TRY(d_in.reserve(n));
    HIP_TRY(d_out.reserve(n));
    HIP_TRY(hipMemcpyAsync(d_in.p, in, n * sizeof(int16_t), hipMemcpyHostToDevice, s));
    HIP_TRY(launch_decode_pcm16(d_in.p, d_out.p, n, s));
    HIP_TRY(hipMemcpyAsync(out, d_out.p, n * sizeof(float), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return EWK_OK;
}

// Event banks are drained in two steps so a failing poll consumes nothing:
// peek_bank waits for the pushes into bank b (copy stream only, no wait on later
// work) and fetches its counters with the first kPollChunk events; take_bank copies
// the rest out and re-arms the bank's counters on the engine stream.
struct BankPeek {
    int32_t n = 0;         // queued events (<= ev_cap)
    int32_t dropped = 0;   // events lost to a full bank
    uint32_t count = 0, dropped_total = 0;   // the raw counters (the next epoch's bases)
    bool used = false;
};

static int peek_bank(ewk_engine* e, int b, BankPeek* pk) {
    *pk = BankPeek();
    if (!e->bank_used[b]) return EWK_OK;
    HIP_TRY(ensure_poll_region(e));
    unsigned char* reg = e->h_poll + b * kPollRegion;
    int32_t* cnt = reinterpret_cast<int32_t*>(reg);
    const int32_t chunk = std::min<int32_t>(kPollChunk, e->ev_cap);
    if (e->mirror[b]) {   // written by k_bank_mirror behind the bank's last push
        HIP_TRY(hipEventSynchronize(e->bank_done[b]));
    } else {
        HIP_TRY(hipStreamWaitEvent(e->cstream, e->bank_done[b], 0));
        HIP_TRY(hipMemcpyAsync(cnt, e->evc_bank(b), 4 * sizeof(int32_t), hipMemcpyDeviceToHost, e->cstream));
        HIP_TRY(hipMemcpyAsync(reg + 16, e->ev_bank(b), (size_t)chunk * sizeof(ewk_event), hipMemcpyDeviceToHost,
                               e->cstream));
        HIP_TRY(hipStreamSynchronize(e->cstream));
    }
    pk->count = (uint32_t)cnt[0];
    pk->dropped_total = (uint32_t)cnt[1];
    pk->n = (int32_t)std::min<uint32_t>(pk->count - e->ev_base0[b], (uint32_t)e->ev_cap);
    pk->dropped = (int32_t)(pk->dropped_total - e->drop_base0[b]);
    pk->used = true;
    return EWK_OK;
}

// Re-arm bank b: its next epoch starts at the counters the host just read (no device work;
// the scorer's watermark is at or behind the new base and is clamped to it).
static int rearm_bank(ewk_engine* e, int b, const BankPeek& pk) {
    e->ev_base0[b] = pk.count;
    e->drop_base0[b] = pk.dropped_total;
    e->bank_used[b] = false;
    e->mirror[b] = false;
    return EWK_OK;
}

static int take_bank(ewk_engine* e, int b, const BankPeek& pk, ewk_event* out) {
    if (!pk.used) return EWK_OK;
    const int32_t chunk = std::min<int32_t>(kPollChunk, e->ev_cap);
    if (pk.n > 0 && out) {
        memcpy(out, e->h_poll + b * kPollRegion + 16, (size_t)std::min(pk.n, chunk) * sizeof(ewk_event));
        if (pk.n > chunk) {
            HIP_TRY(hipMemcpyAsync(out + chunk, e->ev_bank(b) + chunk, (size_t)(pk.n - chunk) * sizeof(ewk_event),
                                   hipMemcpyDeviceToHost, e->cstream));
            HIP_TRY(hipStreamSynchronize(e->cstream));
        }
    }
    return rearm_bank(e, b, pk);
}

// An overflowed bank cannot be delivered whole: re-arm it (its events are lost, the
// engine keeps running) and report how many were dropped.
static int overflow(ewk_engine* e, const BankPeek* pk, const int* banks, int nb) {
    int64_t lost = 0;
    for (int i = 0; i < nb; ++i)
        if (pk[i].used && pk[i].dropped > 0) {
            lost += (int64_t)pk[i].n + pk[i].dropped;
            int rc = rearm_bank(e, banks[i], pk[i]);
            if (rc) return rc;
        }
    return fail(EWK_ENOMEM, "event queue overflow: " + std::to_string(lost) +
                                " events of the overflowed bank(s) dropped; the queue was re-armed");
}

static void sort_events(ewk_event* out, int32_t n) {   // deterministic order: (tick, stream)
    std::sort(out, out + n, [](const ewk_event& x, const ewk_event& y) {
        return x.tick != y.tick ? x.tick < y.tick : x.stream < y.stream;
    });
}

static int poll_banks(ewk_engine* e, const int* banks, int nb, ewk_event* out, int32_t cap, int32_t* n_out) {
    BankPeek pk[2];
    int64_t total = 0;
    bool over = false;
    for (int i = 0; i < nb; ++i) {
        int rc = peek_bank(e, banks[i], &pk[i]);
        if (rc) return rc;
        total += pk[i].n;
        over = over || pk[i].dropped > 0;
    }
    if (over) return overflow(e, pk, banks, nb);
    // validated before either bank is consumed: a short `cap` loses nothing
    if (out && total > std::max(0, cap))
        return fail(EWK_EINVAL, "poll capacity " + std::to_string(cap) + " is smaller than the " +
                                    std::to_string(total) + " queued events (nothing was drained)");
    int32_t n = 0;
    for (int i = 0; i < nb; ++i) {
        int rc = take_bank(e, banks[i], pk[i], out ? out + n : nullptr);
        if (rc) return rc;
        n += pk[i].n;
    }
    if (out) sort_events(out, n);
    *n_out = n;
    return EWK_OK;
}

int ewk_poll(ewk_engine* e, ewk_event* out, int32_t cap, int32_t* n_out) {
    if (!e || !n_out) return fail(EWK_EINVAL, "NULL argument");
    *n_out = 0;
    if (e->n_streams <= 0) return EWK_OK;
    HIP_TRY(hipSetDevice(e->device));
    const int banks[2] = {e->bank ^ 1, e->bank};   // older first
    return poll_banks(e, banks, 2, out, cap, n_out);
}

int ewk_poll_lagged(ewk_engine* e, ewk_event* out, int32_t cap, int32_t* n_out) {
    if (!e || !n_out) return fail(EWK_EINVAL, "NULL argument");
    *n_out = 0;
    if (e->n_streams <= 0) return EWK_OK;
    HIP_TRY(hipSetDevice(e->device));
    const int older = e->bank ^ 1;
    const int banks[1] = {older};
    int rc = poll_banks(e, banks, 1, out, cap, n_out);
    if (rc == EWK_OK || !e->bank_used[older])   // drained (or re-armed after an overflow)
        e->bank = older;   // later pushes append to the drained bank; the newest one drains next time
    return rc;
}

int ewk_reenter(ewk_engine* e, int32_t stream, double reentry_timeout) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    if (e->n_streams <= 0) return fail(EWK_EINVAL, "engine has no streams");
    if (stream < -1 || stream >= e->n_streams) return fail(EWK_EINVAL, "stream index out of range");
    if (!(reentry_timeout == reentry_timeout)) return fail(EWK_EINVAL, "reentry_timeout is NaN");
    HIP_TRY(hipSetDevice(e->device));
    e->cfg.reentry_timeout = reentry_timeout;   // read by every later gate launch
    const int32_t first = stream < 0 ? 0 : stream;
    const int32_t n = stream < 0 ? e->n_streams : 1;
    HIP_TRY(launch_reenter(e->d_st, first, n, e->cfg.tick_seconds, e->stream));
    return EWK_OK;
}

int ewk_get_stream_state(ewk_engine* e, int32_t stream, ewk_stream_state* out) {
    if (!e || !out) return fail(EWK_EINVAL, "NULL argument");
    if (stream < 0 || stream >= e->n_streams) return fail(EWK_EINVAL, "stream index out of range");
    HIP_TRY(hipSetDevice(e->device));
    GateStream st;
    HIP_TRY(hipMemcpyAsync(&st, e->d_st + stream, sizeof(st), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    out->samples_collected = st.collected;
    out->tick = st.tick;
    out->silence_threshold = st.threshold;
    out->last_rms = st.last_rms;
    out->silence_start_time = st.silence_start;
    out->sound_start_time = st.sound_start;
    out->sound_end_time = st.sound_end;
    out->start_time = st.start_time;
    out->pointer = st.pointer;
    out->state = st.state;
    out->started = st.started;
    out->last_silent = st.last_silent;
    return EWK_OK;
}

int ewk_read_segment(ewk_engine* e, int32_t stream, int64_t ring_start, int32_t length, float* out) {
    if (!e || !out) return fail(EWK_EINVAL, "NULL argument");
    if (stream < 0 || stream >= e->n_streams) return fail(EWK_EINVAL, "stream index out of range");
    if (length < 0 || length > e->sring_len || ring_start < 0 || ring_start >= e->sring_len)
        return fail(EWK_EINVAL, "segment out of range");
    HIP_TRY(hipSetDevice(e->device));
    const size_t es = e->ring_es;
    const unsigned char* base = static_cast<const unsigned char*>(e->d_ring) + (size_t)stream * e->sring_len * es;
    const int64_t first = std::min<int64_t>(length, e->sring_len - ring_start);
    // int16 rings: copied to a host staging buffer, then widened (x / 32768, exact)
    std::vector<int16_t> q(es == sizeof(int16_t) ? (size_t)length : 0);
    unsigned char* dst = es == sizeof(float) ? reinterpret_cast<unsigned char*>(out)
                                             : reinterpret_cast<unsigned char*>(q.data());
    HIP_TRY(hipMemcpyAsync(dst, base + ring_start * es, first * es, hipMemcpyDeviceToHost, e->stream));
    if (length > first)
        HIP_TRY(hipMemcpyAsync(dst + first * es, base, (length - first) * es, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (size_t i = 0; i < q.size(); ++i) out[i] = (float)q[i] * (1.0f / 32768.0f);
    return EWK_OK;
}

int ewk_read_last(ewk_engine* e, int32_t stream, int64_t n_samples, float* out, int64_t* n_out) {
    if (!e || !out || !n_out) return fail(EWK_EINVAL, "NULL argument");
    if (stream < 0 || stream >= e->n_streams) return fail(EWK_EINVAL, "stream index out of range");
    // return_last_n_seconds: at most the reference ring (wakeword.py:500-502)
    int64_t n = std::min<int64_t>(std::max<int64_t>(n_samples, 0), e->ring_len);
    *n_out = 0;
    if (n > e->sring_len)
        return fail(EWK_EINVAL, "the compact ring keeps only the last " + std::to_string(e->sring_len) + " samples");
    HIP_TRY(hipSetDevice(e->device));
    GateStream st;
    HIP_TRY(hipMemcpyAsync(&st, e->d_st + stream, sizeof(st), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    *n_out = n;
    if (n == 0) return EWK_OK;
    int64_t start = st.spos - n;
    if (start < 0) start += e->sring_len;
    return ewk_read_segment(e, stream, start, (int32_t)n, out);
}

int ewk_profile_enable(ewk_engine* e, int32_t on) {
    if (!e) return fail(EWK_EINVAL, "engine is NULL");
    e->prof = on != 0;
    return EWK_OK;
}

int ewk_profile_read(ewk_engine* e, int32_t kind, double* total_ms, int64_t* launches) {
    if (!e || !total_ms || !launches) return fail(EWK_EINVAL, "NULL argument");
    if (kind < 0 || kind > 2) return fail(EWK_EINVAL, "kind must be 0, 1 or 2");
    HIP_TRY(hipSetDevice(e->device));
    double tot = 0.0;
    for (auto& p : e->ev[kind]) {
        HIP_TRY(hipEventSynchronize(p.second));
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, p.first, p.second));
        tot += ms;
        e->ev_pool.push_back(p.first);
        e->ev_pool.push_back(p.second);
    }
    *total_ms = tot;
    *launches = (int64_t)e->ev[kind].size();
    e->ev[kind].clear();
    return EWK_OK;
}

}  // extern "C"
