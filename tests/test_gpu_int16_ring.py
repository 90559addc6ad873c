"""int16 sample rings (ewk_config.ring_format = EWK_RING_I16) on the GPU.

A PCM16 source (PortAudio paInt16, a 16-bit WAV) delivers x = k / 32768; an int16
ring stores k exactly, in half the HBM.  Bar: the same PCM16 pushes into float32 and
int16 rings (full and compact) give identical events field for field (score bits
included), identical thresholds, identical segment samples and level-3 input, and
the oracle's events; float32 pushes into an int16 ring are refused.  The 65,536-stream
case runs the one-segment-per-wave ring scorer (k_score_f32<2, 1>).
"""
import numpy as np
import pytest

import synth
from golden_io import matcher_fixture, score_close, template_arrays
from oracle import mfcc_ref
from oracle.gate_ref import GateConfig, run_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def template():
    fx, _ = matcher_fixture()
    return template_arrays(fx)


def _pcm16_streams(n, seed0, n_words=4):
    rows = []
    for i in range(n):
        rng = np.random.default_rng(seed0 + i)
        p, _ = synth.make_stream(seed=seed0 + 500 + i, n_words=n_words, sigma=float(rng.uniform(2e-4, 4e-3)),
                                 gain=float(rng.uniform(0.3, 2.5)), distractors=bool(i % 2))
        rows.append(p)
    L = min(len(p) for p in rows) // 1600 * 1600
    x = np.stack([p[:L] for p in rows])
    return np.clip(np.round(x.astype(np.float64) * 32768.0), -32768, 32767).astype(np.int16)


def _run(q, template, **cfg):
    from easywakeword_amd import StreamEngine
    eng = StreamEngine(q.shape[0], **cfg)
    eng.set_template(*template)
    got = []
    for c in range(0, q.shape[1], 9 * 1600):
        eng.push_pcm16(q[:, c:c + 9 * 1600])
        got.append(eng.poll())
    ev = np.concatenate(got)
    thr = [eng.state(i)["silence_threshold"] for i in range(q.shape[0])]
    if cfg.get("ring_samples"):
        # ticks after their cut, a compact ring no longer holds the last events' first
        # samples: the level-3 read is refused instead of returning overwritten audio
        with pytest.raises(ValueError, match="overwritten"):
            eng.normalize_events(ev[:1])
        return eng, ev, thr, None, None
    segs = [eng.read_segment(int(e["stream"]), int(e["ring_start"]), int(e["length"])) for e in ev[-6:]]
    l3 = eng.normalize_events(ev[-6:])
    return eng, ev, thr, segs, l3


def test_int16_ring_equals_float32_ring_and_oracle(template):
    q = _pcm16_streams(10, 4100)
    results = [_run(q, template),
               _run(q, template, ring_format=1),
               _run(q, template, ring_format=1, ring_samples=43200)]
    _, ev_f, thr_f, seg_f, l3_f = results[0]
    assert len(ev_f) > 15
    for k, (eng, ev, thr, segs, l3) in enumerate(results[1:]):
        for f in ("stream", "tick", "length", "flags", "match"):
            np.testing.assert_array_equal(ev[f], ev_f[f], err_msg=f)
        np.testing.assert_array_equal(ev["score"].view(np.int64), ev_f["score"].view(np.int64))
        assert thr == thr_f
        if k == 0:   # full rings still hold the last events' samples (a compact ring may not, ticks later)
            for a, b in zip(segs, seg_f):
                np.testing.assert_array_equal(a, b)
            for a, b in zip(l3, l3_f):
                np.testing.assert_array_equal(a, b)
        with pytest.raises(ValueError, match="PCM16"):
            eng.push(np.zeros((q.shape[0], 1600), np.float32))
        eng.close()
    results[0][0].close()
    x = q.astype(np.float32) / np.float32(32768.0)
    tm, ts = template
    n_checked = 0
    for i in range(q.shape[0]):
        ref = run_stream(x[i], GateConfig()).events
        mine = ev_f[ev_f["stream"] == i]
        assert [(int(m["tick"]), int(m["length"]), bool(m["flags"] & 1)) for m in mine] == \
               [(e.tick, e.length, e.skipped) for e in ref], i
        for m, e in zip(mine, ref):
            if e.skipped or n_checked >= 12:
                continue
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            assert score_close(float(m["score"]), s, 1e-4)
            assert bool(m["match"]) == (s >= 75.0)
            n_checked += 1


def test_int16_ring_65536_streams_per_wave_scorer():
    import torch
    import bench
    from easywakeword_amd import StreamEngine
    dev = torch.device("cuda", 0)
    word = bench.load_word()
    n, ticks = 65536, 220
    sig = bench.make_shifted_signal(torch, dev, n, ticks, 99, word, pcm16=True)
    out = []
    for fmt, ring in ((0, 0), (1, 48000)):
        se = StreamEngine(n, ring_format=fmt, ring_samples=ring)
        se.template_from_pcm(word)
        got = []
        for t in range(0, ticks, 4):
            se.push_device_pcm16(sig.data_ptr() + t * 1600 * 2, 1600, 1600, 4)
            got.append(se.poll())
        ev = np.concatenate(got)
        out.append(ev[np.lexsort((ev["stream"], ev["tick"]))])
        se.close()
    a, b = out
    assert len(a) > n // 4
    for f in ("stream", "tick", "length", "flags", "match"):
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)
    np.testing.assert_array_equal(a["score"].view(np.int64), b["score"].view(np.int64))
