"""Diagnostic (pytest-style, GPU box): test_gpu_gate.py::test_many_streams_vs_oracle's scenario
K times in the calling pytest process, after whatever tests ran before it in that process (the
ring-path miss appears only after a session's earlier tests).  Records every wrong score
(engine vs oracle > 1e-4) with the ring read-back check, in gpurun_out/diag_loop.json; never
fails (it measures a rate).  EWK_DIAG_K sets K (default 20).

    python -m pytest -q <earlier tests> scripts/diag_many_streams_loop.py
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

pytestmark = pytest.mark.gpu


def test_many_streams_loop():
    import synth
    from golden_io import matcher_fixture, template_arrays
    from oracle import mfcc_ref
    from oracle.gate_ref import GateConfig, run_stream
    from easywakeword_amd import StreamEngine
    K = int(os.environ.get("EWK_DIAG_K", "20"))
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
                ref[(i, e.tick)] = (float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs)), np.asarray(e.audio, np.float32))
    bad = []
    poll_kind = os.environ.get("EWK_DIAG_POLLUTE")   # fill every CU's LDS / VGPRs before each run
    pol = None
    if poll_kind is not None:
        import ctypes
        pol = ctypes.CDLL(os.path.join(ROOT, "scripts", "probes", "lds_polluter.so"))
    for r in range(K):
        if pol is not None:
            assert pol.pollute(int(poll_kind)) == 0
        eng = StreamEngine(32, pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0,
                           post_speech_silence=0.4)
        eng.set_template(tm, ts)
        got = []
        for c in range(0, L, 16 * 1600):
            eng.push_many(data[:, c:c + 16 * 1600])
            got.extend(eng.poll().tolist())
        for g in got:
            if g[7] & 1 or (g[0], g[2]) not in ref:
                continue
            s, audio = ref[(g[0], g[2])]
            ok = abs(g[5] - s) <= 1e-4
            p0 = g[2] * 1600 - (g[2] * 1600 - g[3]) % 160000
            ring_ok = None
            if p0 >= L - 160000:
                ring_ok = bool(np.array_equal(eng.read_segment(g[0], g[3], g[1]), audio))
            if not ok or ring_ok is False:
                bad.append(dict(run=r, stream=int(g[0]), tick=int(g[2]), length=int(g[1]), ring_start=int(g[3]),
                                score=repr(float(g[5])), oracle=repr(s), flags=int(g[7]), ring_ok=ring_ok))
        eng.close()
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, f"diag_loop_{os.environ.get('EWK_DIAG_TAG', 'x')}.json")
    with open(path, "w") as f:
        json.dump(dict(K=K, lib=os.environ.get("EWK_LIB", ""), pollute=poll_kind, bad=bad), f, indent=1)
    print(f"\n[diag] {K} runs, {len(bad)} wrong events: {bad[:6]}")
