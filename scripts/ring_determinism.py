"""Determinism of the ring path's scores: tests/test_gpu_gate.py::test_many_streams_vs_oracle's
32-stream scenario (16 ticks per push) run REPS times in one process; every run's events must
be identical to the first, and their scores within 1e-4 of the oracle.

    EWK_LIB=... python scripts/ring_determinism.py [reps]
"""
import os
import sys

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402
from oracle import mfcc_ref  # noqa: E402
from oracle.gate_ref import GateConfig, run_stream  # noqa: E402
from easywakeword_amd import StreamEngine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
gate = dict(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0, post_speech_silence=0.4)
pcms = []
for i in range(32):
    rng = np.random.default_rng(500 + i)
    p, _ = synth.make_stream(seed=2000 + i, n_words=4, sigma=float(rng.uniform(1e-4, 5e-3)),
                             gain=float(rng.uniform(0.2, 3.0)), distractors=bool(i % 2))
    pcms.append(p)
L = min(len(p) for p in pcms)
L -= L % 1600
data = np.stack([p[:L] for p in pcms]).astype(np.float32)
tm, ts = mfcc_ref.extract_mfcc(synth.load_word())
ref = {}
for i in range(32):
    for e in run_stream(data[i], GateConfig(**gate)).events:
        if not e.skipped:
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            ref[(i, e.tick)] = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
runs = []
for r in range(reps):
    eng = StreamEngine(32, **gate)
    eng.set_template(tm, ts)
    got = []
    for c in range(0, L, 16 * 1600):
        eng.push_many(data[:, c:c + 16 * 1600])
        got.append(eng.poll())
    eng.close()
    ev = np.concatenate(got)
    ev = ev[np.lexsort((ev["tick"], ev["stream"]))]
    bad = [(int(x["stream"]), int(x["tick"]), float(x["score"]), ref[(int(x["stream"]), int(x["tick"]))])
           for x in ev if (int(x["stream"]), int(x["tick"])) in ref
           and not abs(float(x["score"]) - ref[(int(x["stream"]), int(x["tick"]))]) <= 1e-4]
    same = r == 0 or np.array_equal(ev.view(np.uint8), runs[0].view(np.uint8))
    print(f"run {r}: {len(ev)} events, identical to run 0: {same}, off the oracle by > 1e-4: {bad[:5]}")
    runs.append(ev)
