"""Randomised streaming configurations on the GPU against the oracle gate
(oracle/gate_ref.py, the reference's SoundBuffer + _detect_word restated).

Each case draws a block size (20-125 ms callbacks on a real-time virtual clock), a ring
length, the detector's durations, a push granularity, the ring format (float32 or int16,
full or compact) and a handful of streams with words, distractors and rejects.  Bar: the
event list (tick, length, skip flag) identical to the oracle's and scores within 1e-4 with
identical decisions -- the same bar as the fixed-configuration tests.
"""
import numpy as np
import pytest

import synth
from golden_io import matcher_fixture, score_close, template_arrays
from oracle import mfcc_ref
from oracle.gate_ref import GateConfig, run_stream

pytestmark = pytest.mark.gpu

SR = 16000


@pytest.fixture(scope="module")
def template():
    fx, _ = matcher_fixture()
    return template_arrays(fx)


def _case(seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    block = int(rng.choice([320, 512, 800, 1000, 1600, 2000]))
    buf = int(rng.choice([4, 6, 10]))
    smin = float(rng.uniform(0.2, 0.5))
    smax = float(rng.uniform(1.2, 2.6))
    pre = float(rng.uniform(0.3, 1.0))
    post = float(rng.uniform(0.2, 0.6))
    per_push = int(rng.choice([1, 5, 13]))
    int16 = bool(rng.integers(0, 2))
    compact = bool(rng.integers(0, 2)) and (buf * SR) % block == 0
    return dict(block=block, buf=buf, smin=smin, smax=smax, pre=pre, post=post, per_push=per_push,
                int16=int16, compact=compact)


@pytest.mark.parametrize("seed", [11, 12, 13, 14, 15, 16])
def test_random_stream_configs_vs_oracle(seed, template):
    from easywakeword_amd import StreamEngine
    c = _case(seed)
    block = c["block"]
    n = 4
    pcms = []
    for i in range(n):
        rng = np.random.default_rng(seed * 100 + i)
        p, _ = synth.make_stream(seed=seed * 1000 + i, n_words=3, prefill=float(c["buf"]) + 0.5,
                                 sigma=float(rng.uniform(1e-4, 3e-3)), gain=float(rng.uniform(0.3, 2.0)),
                                 distractors=bool(i % 2), block=block)
        pcms.append(p)
    L = min(len(p) for p in pcms)
    L -= L % block
    data = np.stack([p[:L] for p in pcms]).astype(np.float32)
    if c["int16"]:   # PCM16 values x / 32768 (a 16-bit source): exact in both the oracle and the ring
        q = np.clip(np.round(data * 32768.0), -32768, 32767).astype(np.int16)
        data = q.astype(np.float32) / np.float32(32768.0)
    cfg = dict(block=block, tick_seconds=block / SR, buffer_seconds=c["buf"], speech_duration_min=c["smin"],
               speech_duration_max=c["smax"], pre_speech_silence=c["pre"], post_speech_silence=c["post"])
    if c["compact"]:
        need = int((c["smax"] + c["post"] + block / SR + 0.05) * SR) + 2 + block
        ring = -(-need // block) * block
        if ring < c["buf"] * SR:
            cfg["ring_samples"] = ring
    if c["int16"]:
        cfg["ring_format"] = 1
    eng = StreamEngine(n, **cfg)
    eng.set_template(*template)
    got = []
    step = c["per_push"] * block
    for t0 in range(0, L, step):
        if c["int16"]:
            eng.push_pcm16(q[:, t0:t0 + step])
        else:
            eng.push_many(data[:, t0:t0 + step])
        got.append(eng.poll())
    eng.close()
    ev = np.concatenate(got)
    tm, ts = template
    gcfg = GateConfig(block=block, tick_seconds=block / SR, buffer_seconds=c["buf"], speech_duration_min=c["smin"],
                      speech_duration_max=c["smax"], pre_speech_silence=c["pre"], post_speech_silence=c["post"])
    n_scored = 0
    for i in range(n):
        ref = run_stream(data[i], gcfg).events
        mine = ev[ev["stream"] == i]
        assert [(int(m["tick"]), int(m["length"]), bool(m["flags"] & 1)) for m in mine] == \
               [(e.tick, e.length, e.skipped) for e in ref], (c, i)
        for m, e in zip(mine, ref):
            if e.skipped:
                continue
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            assert score_close(float(m["score"]), s, 1e-4), (c, i, int(m["tick"]), float(m["score"]), s)
            assert bool(m["match"]) == (s >= 75.0), (c, i)
            n_scored += 1
    assert n_scored >= 1, c


@pytest.mark.parametrize("overlap", ["0", "1"])
def test_lagged_polls_late_template_and_overlap_vs_oracle(overlap, template, monkeypatch):
    """One tick per push with lagged polls (the serving cadence), the template set only after
    tick 150 (the polls before it read the k_bank_mirror copy, after it the scorer's tick-end
    copy), with the scorer on the engine stream and in the opt-in overlap mode
    (EWK_SCORE_OVERLAP=1, scoring of tick t beside the gate of tick t+1): the event list equals
    the oracle's, every scored event within 1e-4 of it, every event after the template scored."""
    from easywakeword_amd import StreamEngine
    monkeypatch.setenv("EWK_SCORE_OVERLAP", overlap)
    block, n = 1600, 4
    pcms = [synth.make_stream(seed=7100 + i, n_words=4, prefill=10.5, sigma=1e-3, gain=1.0,
                              distractors=bool(i % 2), block=block)[0] for i in range(n)]
    L = min(len(p) for p in pcms)
    L -= L % block
    data = np.stack([p[:L] for p in pcms]).astype(np.float32)
    eng = StreamEngine(n, block=block, tick_seconds=block / SR, buffer_seconds=10)
    t_tmpl = 150
    got = []
    for t in range(L // block):
        if t == t_tmpl:
            eng.set_template(*template)
        eng.push_many(data[:, t * block:(t + 1) * block])
        got.append(eng.poll(lagged=True))
    got.append(eng.poll())
    eng.close()
    ev = np.concatenate(got)
    tm, ts = template
    gcfg = GateConfig(block=block, tick_seconds=block / SR, buffer_seconds=10)
    n_scored = 0
    for i in range(n):
        ref = run_stream(data[i], gcfg).events
        mine = ev[ev["stream"] == i]
        assert [(int(m["tick"]), int(m["length"]), bool(m["flags"] & 1)) for m in mine] == \
               [(e.tick, e.length, e.skipped) for e in ref], (overlap, i)
        for m, e in zip(mine, ref):
            if e.skipped:
                continue
            if np.isnan(float(m["score"])) and int(m["tick"]) <= t_tmpl:
                continue   # drained before the template existed: never scored
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            assert score_close(float(m["score"]), s, 1e-4), (overlap, i, int(m["tick"]), float(m["score"]), s)
            assert bool(m["match"]) == (s >= 75.0), (overlap, i)
            n_scored += 1
    assert n_scored >= 1
