// A C-style host of libewk.so with no Python: scores K batches of segments on the device,
// compacts each batch's positives with ewk_compact_positives (append mode, the records and
// their count stay in device memory), then runs the gather INTEGRATION.md section 4 shows --
// an RCCL all_gather of the per-rank counts and the records to rank 0 -- and checks the
// records on the host.  This is the C-side counterpart of easywakeword_amd.shard.MatchGather
// (SURVEY.md 8b `ewk_gather_detections`; the reference's consumer of positives is the level-3
// confirm, wakeword.py:1120-1130).
//
// One process per GPU: rank/world from RANK / WORLD_SIZE (default 0 / 1), the RCCL unique id
// passed through a file named by EWK_NCCL_ID_FILE when world > 1.  tests/test_gpu_c_host.py
// runs it with world 1 on one MI355X.
//
// Usage: c_positives_rccl <reference_word.wav> [n_segments] [steps]
// Build: __graft_entry__.build() (hipcc, links libewk.so and librccl).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <vector>

#include "ewk.h"

#define HIP_CHECK(x)                                                                    \
    do {                                                                                \
        hipError_t err_ = (x);                                                          \
        if (err_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(err_)); \
            exit(2);                                                                    \
        }                                                                               \
    } while (0)
#define EWK_CHECK(x)                                                                    \
    do {                                                                                \
        int rc_ = (x);                                                                  \
        if (rc_ != EWK_OK) {                                                            \
            fprintf(stderr, "%s:%d %s: %d %s\n", __FILE__, __LINE__, #x, rc_, ewk_last_error()); \
            exit(3);                                                                    \
        }                                                                               \
    } while (0)
#define NCCL_CHECK(x)                                                                   \
    do {                                                                                \
        ncclResult_t r_ = (x);                                                          \
        if (r_ != ncclSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); \
            exit(4);                                                                    \
        }                                                                               \
    } while (0)

// 16 kHz mono PCM16 WAV -> float32 k / 32768 (librosa.load's scaling for such files)
static std::vector<float> read_wav16(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    std::vector<unsigned char> b;
    unsigned char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
    fclose(f);
    size_t p = 12;
    while (p + 8 <= b.size()) {   // walk the RIFF chunks to "data"
        const uint32_t sz = b[p + 4] | (b[p + 5] << 8) | (b[p + 6] << 16) | ((uint32_t)b[p + 7] << 24);
        if (memcmp(&b[p], "data", 4) == 0) {
            std::vector<float> out(sz / 2);
            for (size_t i = 0; i < out.size(); ++i)
                out[i] = (float)(int16_t)(b[p + 8 + 2 * i] | (b[p + 9 + 2 * i] << 8)) / 32768.0f;
            return out;
        }
        p += 8 + sz + (sz & 1);
    }
    fprintf(stderr, "%s: no data chunk\n", path);
    exit(1);
}

static uint32_t lcg(uint32_t& s) { return s = s * 1664525u + 1013904223u; }
static float noise(uint32_t& s) { return ((float)(lcg(s) >> 8) / 16777216.0f - 0.5f) * 2e-3f; }

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s reference_word.wav [n_segments] [steps]\n", argv[0]); return 1; }
    const int n_seg = argc > 2 ? atoi(argv[2]) : 4096;
    const int steps = argc > 3 ? atoi(argv[3]) : 3;
    const int rank = getenv("RANK") ? atoi(getenv("RANK")) : 0;
    const int world = getenv("WORLD_SIZE") ? atoi(getenv("WORLD_SIZE")) : 1;
    int ndev = 0;
    HIP_CHECK(hipGetDeviceCount(&ndev));
    const int dev = ndev ? rank % ndev : 0;
    HIP_CHECK(hipSetDevice(dev));

    const std::vector<float> word = read_wav16(argv[1]);
    ewk_config cfg;
    ewk_default_config(&cfg);
    ewk_engine* e = nullptr;
    EWK_CHECK(ewk_create(&e, dev, 0, &cfg));
    EWK_CHECK(ewk_template_from_pcm(e, word.data(), (int64_t)word.size()));

    // segments: even i = the word at a per-segment gain plus noise (mostly matches), odd i =
    // noise only (no match), lengths ragged around the word's
    std::vector<int64_t> off(n_seg);
    std::vector<int32_t> len(n_seg);
    std::vector<float> pcm;
    uint32_t s = 1234u + 1000u * (uint32_t)rank;
    for (int i = 0; i < n_seg; ++i) {
        const int pad = 800 + (int)(lcg(s) % 4000);
        off[i] = (int64_t)pcm.size();
        len[i] = (int32_t)word.size() + pad;
        const float gain = 0.8f + (float)(lcg(s) % 1000) / 2500.0f;
        for (int k = 0; k < pad / 2; ++k) pcm.push_back(noise(s));
        for (size_t k = 0; k < word.size(); ++k) pcm.push_back((i % 2 == 0 ? gain * word[k] : 0.0f) + noise(s));
        for (int k = pad / 2; k < pad; ++k) pcm.push_back(noise(s));
    }
    hipStream_t st = (hipStream_t)ewk_stream_handle(e);
    float* d_pcm;
    int64_t* d_off;
    int32_t* d_len;
    double* d_score;
    uint8_t* d_match;
    ewk_positive* d_pos;
    int32_t* d_cnt;
    int32_t* d_counts;
    HIP_CHECK(hipMalloc(&d_pcm, pcm.size() * sizeof(float)));
    HIP_CHECK(hipMalloc(&d_off, n_seg * sizeof(int64_t)));
    HIP_CHECK(hipMalloc(&d_len, n_seg * sizeof(int32_t)));
    HIP_CHECK(hipMalloc(&d_score, n_seg * sizeof(double)));
    HIP_CHECK(hipMalloc(&d_match, n_seg));
    HIP_CHECK(hipMalloc(&d_pos, (size_t)steps * n_seg * sizeof(ewk_positive)));
    HIP_CHECK(hipMalloc(&d_cnt, sizeof(int32_t)));
    HIP_CHECK(hipMalloc(&d_counts, world * sizeof(int32_t)));
    HIP_CHECK(hipMemcpyAsync(d_pcm, pcm.data(), pcm.size() * sizeof(float), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_off, off.data(), n_seg * sizeof(int64_t), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_len, len.data(), n_seg * sizeof(int32_t), hipMemcpyHostToDevice, st));

    // K steps: score + compact, no host sync
    for (int k = 0; k < steps; ++k) {
        EWK_CHECK(ewk_score_segments_device(e, d_pcm, d_off, d_len, n_seg, nullptr, nullptr, d_score, d_match,
                                            EWK_SCORE_REQUIRE_TEMPLATE, st));
        EWK_CHECK(ewk_compact_positives(e, d_score, d_match, n_seg, (int64_t)rank * n_seg, k, d_pos, d_cnt,
                                        k ? EWK_COMPACT_APPEND : 0, st));
    }

    // the gather: counts to every rank (RCCL), then each rank's records to rank 0
    ncclUniqueId id;
    if (rank == 0) NCCL_CHECK(ncclGetUniqueId(&id));
    if (world > 1) {   // share the id through a file (a real host uses its own bootstrap)
        const char* path = getenv("EWK_NCCL_ID_FILE");
        if (!path) { fprintf(stderr, "EWK_NCCL_ID_FILE is required for world > 1\n"); return 1; }
        if (rank == 0) {
            FILE* f = fopen(path, "wb");
            fwrite(&id, sizeof id, 1, f);
            fclose(f);
        } else {
            FILE* f = nullptr;
            for (int t = 0; t < 600 && !(f = fopen(path, "rb")); ++t) usleep(100000);
            if (!f || fread(&id, sizeof id, 1, f) != 1) { fprintf(stderr, "no id\n"); return 1; }
            fclose(f);
        }
    }
    ncclComm_t comm;
    NCCL_CHECK(ncclCommInitRank(&comm, world, id, rank));
    NCCL_CHECK(ncclAllGather(d_cnt, d_counts, 1, ncclInt32, comm, st));
    std::vector<int32_t> counts(world);
    HIP_CHECK(hipMemcpyAsync(counts.data(), d_counts, world * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));   // the gather's one host sync
    int64_t total = 0;
    for (int r = 0; r < world; ++r) total += counts[r];
    ewk_positive* d_all = nullptr;
    if (rank == 0) HIP_CHECK(hipMalloc(&d_all, (size_t)(total > 0 ? total : 1) * sizeof(ewk_positive)));
    NCCL_CHECK(ncclGroupStart());
    if (rank != 0) {
        if (counts[rank]) NCCL_CHECK(ncclSend(d_pos, counts[rank] * sizeof(ewk_positive), ncclUint8, 0, comm, st));
    } else {
        int64_t o = counts[0];
        for (int r = 1; r < world; ++r) {
            if (counts[r])
                NCCL_CHECK(ncclRecv(d_all + o, counts[r] * sizeof(ewk_positive), ncclUint8, r, comm, st));
            o += counts[r];
        }
    }
    NCCL_CHECK(ncclGroupEnd());
    if (rank == 0 && counts[0])
        HIP_CHECK(hipMemcpyAsync(d_all, d_pos, counts[0] * sizeof(ewk_positive), hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));

    // rank 0 checks: the records of every rank are valid (step in range, score >= threshold,
    // no duplicate), and its own are exactly the matched segments of each step with their
    // scores (the scorer's outputs of the last step; every step scores the same batch)
    int bad = 0;
    if (rank == 0) {
        std::vector<ewk_positive> rec(total);
        std::vector<double> score(n_seg);
        std::vector<uint8_t> match(n_seg);
        HIP_CHECK(hipMemcpy(rec.data(), d_all, total * sizeof(ewk_positive), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(score.data(), d_score, n_seg * sizeof(double), hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(match.data(), d_match, n_seg, hipMemcpyDeviceToHost));
        std::vector<int> seen((size_t)world * n_seg * steps, 0);
        int64_t own = 0;
        for (const ewk_positive& p : rec) {
            const int64_t r = p.id / n_seg, i = p.id % n_seg;
            const bool ok = p.id >= 0 && r < world && p.step >= 0 && p.step < steps &&
                            p.score >= cfg.similarity_threshold && !seen[(size_t)(r * n_seg + i) * steps + p.step]++ &&
                            (r != 0 || (match[i] && p.score == score[i]));
            own += r == 0;
            if (!ok && bad++ < 5)
                fprintf(stderr, "bad record: id %lld step %lld score %.17g\n", (long long)p.id, (long long)p.step, p.score);
        }
        int64_t want = 0;
        for (int i = 0; i < n_seg; ++i) want += match[i];
        want *= steps;
        printf("world %d, %d segments x %d steps per rank: %lld positives gathered, rank 0's %lld (want %lld), "
               "%d bad\n", world, n_seg, steps, (long long)total, (long long)own, (long long)want, bad);
        if (own != want || want == 0) bad++;
        printf(bad ? "FAILED\n" : "OK\n");
    }
    NCCL_CHECK(ncclCommDestroy(comm));
    for (void* q : {(void*)d_all, (void*)d_pcm, (void*)d_off, (void*)d_len, (void*)d_score, (void*)d_match,
                    (void*)d_pos, (void*)d_cnt, (void*)d_counts})
        if (q) (void)hipFree(q);
    ewk_destroy(e);
    return bad ? 5 : 0;
}
