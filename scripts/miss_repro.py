"""Rate of the ring-path score miss (tests/test_gpu_gate.py::test_many_streams_vs_oracle's scenario).
(GPU box; diagnostic.  A wrong score, not a GPU fault: every run is checked and recorded.)

    python scripts/miss_repro.py [runs] [--load] [--fresh]

Each run creates a StreamEngine of the 32 scenario streams (like the test), pushes 16 ticks per
call, polls after each push and checks every scored event against the oracle (1e-4).  --load
runs a 65,536-segment batch scorer launch and a 4-stream engine between runs (the GPU state the
earlier tests of a session leave); --fresh keeps one engine per run (default) vs --reuse one
engine re-armed by ewk_reset_streams.  Failures (run, event, engine score, oracle) go to
gpurun_out/miss_repro.json.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import synth
    from golden_io import matcher_fixture, template_arrays
    from oracle import mfcc_ref
    from oracle.gate_ref import GateConfig, run_stream
    from easywakeword_amd import Engine, StreamEngine
    runs = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
    load = "--load" in sys.argv
    fx, _ = matcher_fixture()
    tm, ts = template_arrays(fx)
    pcms = []
    for i in range(32):
        rng = np.random.default_rng(500 + i)
        p, _ = synth.make_stream(seed=2000 + i, n_words=4, sigma=float(rng.uniform(1e-4, 5e-3)),
                                 gain=float(rng.uniform(0.2, 3.0)), distractors=bool(i % 2))
        pcms.append(p)
    L = min(len(p) for p in pcms)
    L -= L % 1600
    data = np.stack([p[:L] for p in pcms]).astype(np.float32)
    cfg = GateConfig(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0, post_speech_silence=0.4)
    ref = {}
    for i in range(32):
        for e in run_stream(data[i], cfg).events:
            if not e.skipped:
                cm, cs = mfcc_ref.extract_mfcc(e.audio)
                ref[(i, e.tick)] = (e.length, float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs)))
    print(f"{len(ref)} oracle events; {runs} runs, load={load}", flush=True)
    bad = []
    dev = torch.device("cuda", 0)
    word = synth.load_word()
    for r in range(runs):
        if load:   # a batch launch and a small engine between runs (other tests' GPU state)
            g = torch.Generator(device="cpu").manual_seed(r)
            n = 65536
            lens = torch.randint(6400, 33600, (n,), generator=g, dtype=torch.int32)
            offs = torch.zeros(n, dtype=torch.int64)
            offs[1:] = torch.cumsum(lens[:-1].to(torch.int64), 0)
            pcm = (torch.randn(int(offs[-1] + lens[-1]), generator=g) * 0.1).to(dev)
            offs_d, lens_d = offs.to(dev), lens.to(dev)
            mean = torch.empty((n, 20), device=dev); std = torch.empty((n, 20), device=dev)
            sc = torch.empty(n, device=dev, dtype=torch.float64); mt = torch.empty(n, device=dev, dtype=torch.uint8)
            eb = Engine()
            eb.template_from_pcm(word)
            eb.score_device(pcm.data_ptr(), offs_d.data_ptr(), lens_d.data_ptr(), n, mean.data_ptr(), std.data_ptr(),
                            sc.data_ptr(), mt.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize()
            eb.close()
            del pcm
        eng = StreamEngine(32, pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0,
                           post_speech_silence=0.4)
        eng.set_template(tm, ts)
        got = []
        for c in range(0, L, 16 * 1600):
            eng.push_many(data[:, c:c + 16 * 1600])
            got.extend(eng.poll().tolist())
        eng.close()
        nb = 0
        for g in got:
            if g[7] & 1:
                continue
            key = (g[0], g[2])
            if key not in ref:
                bad.append(dict(run=r, why="unknown event", mine=list(map(repr, g))))
                nb += 1
                continue
            s = ref[key][1]
            if not (abs(g[5] - s) <= 1e-4 or (np.isnan(g[5]) and np.isnan(s))):
                bad.append(dict(run=r, stream=int(g[0]), tick=int(g[2]), length=int(g[1]), ring_start=int(g[3]),
                                score=repr(float(g[5])), oracle=repr(s), flags=int(g[7])))
                nb += 1
        print(f"run {r}: {len(got)} events, {nb} wrong", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "miss_repro.json"), "w") as f:
        json.dump(bad, f, indent=1)
    print(f"total wrong: {len(bad)} over {runs} runs")
    for b in bad[:20]:
        print("  ", b)


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"({time.time() - t0:.0f} s)")
