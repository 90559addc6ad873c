"""Loud segments whose MFCC mean vector nearly vanishes, through the streaming (ring) path.

Loud white-noise events (gain 1-2 over a quiet floor) give log-mel values averaging near
0 dB: c0's positive and negative frames cancel and |mean| drops to ~8-60.  The float32
pipeline's small absolute mean error then turns the mean vector's direction by up to ~4e-4
in the score (round 3: 341 of 8,192 configs[2] events, DESIGN.md numerics).  Such segments
(|mean| < RESCORE_TINY_MEAN: 32 since round 5, 64 before) go to the fp64 re-score in every
path -- linear batches, the cooperative ring scorer (StreamEngine, MODE 1) and the WakeWord
facade's 1-stream engine -- and must meet the 1e-4 bar against the oracle (oracle/mfcc_ref.py, the float64 candidate path of
wakeword.py:509-513 -> 544-567) like every other segment.
"""
import numpy as np
import pytest

import synth
from golden_io import score_close
from oracle import mfcc_ref
from oracle.gate_ref import GateConfig, run_stream
from easywakeword_amd._lib import RESCORE_TINY_MEAN

pytestmark = pytest.mark.gpu

SCORE_TOL = 1e-4
GATE = dict(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0, post_speech_silence=0.4)
RECIPE = [(g, s) for g in (1.0, 1.5, 2.0) for s in (1e-4, 1e-3, 3e-3)]


def _streams():
    pcms = [synth.make_stream(seed=8100 + i, n_words=4, sigma=s, gain=g, kinds=["white", "word"])[0]
            for i, (g, s) in enumerate(RECIPE)]
    L = min(len(p) for p in pcms) // 1600 * 1600
    return np.stack([p[:L] for p in pcms]).astype(np.float32)


@pytest.fixture(scope="module")
def streams():
    return _streams()


@pytest.fixture(scope="module")
def template():
    return mfcc_ref.extract_mfcc(synth.load_word())


def _check(events, pcm, template, threshold=75.0):
    """events of one stream (tick order) vs the oracle gate + scorer; returns the number of
    |mean| < RESCORE_TINY_MEAN events checked (each finite-scored one must carry EWK_EV_RESCORED;
    a NaN one is not listed when its float32 similarity is negative beyond the float32 error);
    every event, listed or not, must meet the 1e-4 bar (NaN == NaN)."""
    tm, ts = template
    ref = run_stream(pcm, GateConfig(**GATE)).events
    assert [(int(e["tick"]), int(e["length"]), bool(e["flags"] & 1)) for e in events] == \
           [(r.tick, r.length, r.skipped) for r in ref]
    small = 0
    for e, r in zip(events, ref):
        if r.skipped:
            continue
        cm, cs = mfcc_ref.extract_mfcc(r.audio)
        s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
        assert score_close(float(e["score"]), s, SCORE_TOL), (int(e["tick"]), float(e["score"]), s)
        assert bool(e["match"]) == (s >= threshold)
        # (the engine lists |float32 mean| < RESCORE_TINY_MEAN unless the score is NaN beyond the
        # float32 error: a finite oracle score is never such a case)
        if np.linalg.norm(cm) < RESCORE_TINY_MEAN - 0.5:
            small += 1
            if np.isfinite(s):
                assert e["flags"] & 2, "a vanishing-mean event must be decided by the fp64 path"
    return small


def test_vanishing_mean_many_streams_ring(streams, template):
    """9 streams in one engine (cooperative ring scorer), pushed 8 ticks at a time."""
    from easywakeword_amd import StreamEngine
    eng = StreamEngine(len(streams), **GATE)
    eng.set_template(*template)
    got = []
    for c in range(0, streams.shape[1], 8 * 1600):
        eng.push_many(streams[:, c:c + 8 * 1600])
        got.append(eng.poll())
    eng.close()
    ev = np.concatenate(got)
    small = 0
    for i in range(len(streams)):
        mine = ev[ev["stream"] == i]
        small += _check(mine[np.argsort(mine["tick"], kind="stable")], streams[i], template)
    assert small >= 8, small


@pytest.mark.parametrize("i", [4, 6, 8])
def test_vanishing_mean_one_stream_engine(streams, template, i):
    """StreamEngine(1), one tick per push (the facade's engine shape).  The oracle's |mean| of
    the streams' events: 4 -> 11.2 (listed) and 38.0 (float32 alone, inside round 4's |mean| < 64
    criterion), 6 -> 8.0 and 20.3, 8 -> 8.7 and 9.3; every event must meet 1e-4 either way."""
    from easywakeword_amd import StreamEngine
    eng = StreamEngine(1, **GATE)
    eng.set_template(*template)
    got = []
    for c in range(0, streams.shape[1], 1600):
        eng.push(streams[i:i + 1, c:c + 1600])
        got.append(eng.poll())
    eng.close()
    ev = np.concatenate(got)
    assert _check(ev, streams[i], template) >= 1


def test_vanishing_mean_wakeword_facade(streams, template):
    """WakeWord(...).waitforit() over one loud stream: every level-2 call the facade makes
    (its _handle_events sees the polled events) scores like the oracle within 1e-4."""
    import os
    from easywakeword_amd import ArraySource, WakeWord
    from golden_io import GOLD
    i = 5
    pcm = streams[i]
    ww = WakeWord("hello", os.path.join(GOLD, "reference_word.wav"), similarity_threshold=101.0,
                  timeout=int(len(pcm) / 16000) - 9, source=ArraySource(pcm), **GATE)
    seen = []
    handle = ww._handle_events

    def spy(events):
        seen.extend(events.tolist())
        return handle(events)

    ww._handle_events = spy
    with pytest.raises(TimeoutError):
        ww.waitforit()
    from easywakeword_amd._lib import EVENT_DTYPE
    ev = np.array([tuple(x) for x in seen], dtype=EVENT_DTYPE)
    ev = ev[ev["tick"] <= len(pcm) // 1600]   # the source goes on with zeros past the stream's end
    assert len(ev) == len(run_stream(pcm, GateConfig(**GATE)).events)
    tm, ts = ww._matcher.reference_mfcc_mean, ww._matcher.reference_mfcc_std
    assert _check(ev, pcm, (tm, ts), threshold=101.0) >= 1   # the facade's threshold: nothing matches


def test_mean_band_four_recipes_vs_oracle():
    """600 segments whose ORACLE |mean| lies in [32, 64) -- the band the
    round-5 criterion (|mean| < 32) no longer re-scores -- from four recipes other than the
    streaming bench's (tests/golden/mean_band_cases.json, made by make_mean_band.py: loud white
    and pink noise, a tone plus noise, the word in loud noise), scored by the linear batch
    scorer (float64 candidates).  Every score within 1e-4 of the oracle with the same decision;
    the worst error per recipe goes to gpurun_out/ (the criterion's evidence)."""
    import json
    import os
    from easywakeword_amd import Engine
    from evidence import dump
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mean_band_cases.json")) as f:
        cases = json.load(f)["cases"]
    segs = [synth.mean_band_segment(c["kind"], c["seed"], c["gain"], c["length"]) for c in cases]
    eng = Engine()
    eng.template_from_pcm(synth.load_word())
    m, _, sc, mt = eng.score(segs, candidate_dtype="float64")
    ref = np.array([c["score"] for c in cases])
    d = np.abs(sc - ref)
    kinds = sorted(set(c["kind"] for c in cases))
    per = {}
    for k in kinds:
        sel = np.array([c["kind"] == k for c in cases])
        j = int(np.argmax(np.where(sel, d, -1.0)))
        per[k] = dict(n=int(sel.sum()), max_err=float(d[sel].max()), median_err=float(np.median(d[sel])),
                      worst=dict(cases[j], gpu=float(sc[j])),
                      gpu_listed=int((np.linalg.norm(m[sel], axis=1) < RESCORE_TINY_MEAN).sum()))
    dump("mean_band", dict(criterion=RESCORE_TINY_MEAN, max_err=float(d.max()), per_recipe=per,
                           err_by_mean=[[c["mean_norm"], float(e)] for c, e in zip(cases, d)]))
    print("mean band [32, 64):", {k: (v["n"], v["max_err"]) for k, v in per.items()})
    assert len(kinds) >= 3 and len(cases) >= 500
    assert float(d.max()) <= SCORE_TOL, per
    np.testing.assert_array_equal(mt, ref >= 75.0)
    eng.close()
