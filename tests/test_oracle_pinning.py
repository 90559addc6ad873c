"""Pin the CPU oracle before trusting it (CPU only).

* a6/a7 (oracle/mfcc_ref.py, librosa 0.11.0 restatement) against the golden
  outputs recorded from the reference WordMatcher and against the reference's
  own test expectations and LEARNINGS.md:92-94 observations;
* a1-a5 (oracle/gate_ref.py) against traces of the REAL reference SoundBuffer +
  _detect_word driven on the virtual clock (tests/golden/gate_traces.json);
* numpy's summation / percentile orders that the HIP gate kernel restates.
"""
import math

import numpy as np
import pytest

import synth
from golden_io import gate_fixture, matcher_fixture, sha, stream_pcm, template_arrays
from oracle import mfcc_ref
from oracle.gate_ref import GateConfig, pairwise_sum_f64, run_stream


def test_oracle_reproduces_reference_matcher_outputs():
    fx, audio = matcher_fixture()
    tm, ts = template_arrays(fx)
    word = mfcc_ref.load_wav_pcm16(synth.WAV)
    m, s = mfcc_ref.extract_mfcc(word)
    assert np.array_equal(m.astype(np.float32), tm) and np.array_equal(s.astype(np.float32), ts)
    for c in fx["cases"]:
        for dt in ("float64", "float32"):
            y = audio[c["name"]].astype(dt)
            cm, cs = mfcc_ref.extract_mfcc(y)
            sc = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            ref = c[dt]["score"]
            if ref is None:
                assert math.isnan(sc), c["name"]
            else:
                assert sc == ref, (c["name"], dt, sc, ref)


def test_reference_test_expectations_hold_on_oracle():
    """test_wakeword_simulated.py:104-205 / 330-360, test_cross_platform.py:69-109,
    LEARNINGS.md:92-94."""
    m = mfcc_ref.WordMatcherRef()
    a440 = synth.tone(440)
    m.set_reference(a440)
    assert m.matches(a440) == (True, 100.0)
    s880 = float(m.calculate_similarity(synth.tone(880)))
    assert s880 < 100.0 and 89.0 < s880 < 90.5
    rs = np.random.RandomState(42)
    sn = float(m.calculate_similarity(rs.randn(16000).astype(np.float32) * np.float32(0.1)))
    assert 77.0 < sn < 100.0
    assert float(m.calculate_similarity(a440 * np.float32(0.5))) > 50.0
    assert math.isnan(float(m.calculate_similarity(np.zeros(16000))))
    sp = synth.speech_like()
    m.set_reference(sp)
    assert m.matches(sp)[1] == 100.0
    mm = mfcc_ref.mfcc(sp)
    assert mm.shape[0] == 20 and np.all(np.isfinite(mm))
    with pytest.raises(ValueError, match="No reference word set"):
        mfcc_ref.WordMatcherRef().calculate_similarity(np.zeros(100))


def test_template_of_reference_word_matches_survey_values():
    m, s = mfcc_ref.extract_mfcc(mfcc_ref.load_wav_pcm16(synth.WAV))
    np.testing.assert_allclose(m[:5], [-530.337, 98.579, -19.178, 25.856, -26.941], atol=2e-3)
    np.testing.assert_allclose(s[:5], [78.331, 39.104, 40.963, 30.343, 17.543], atol=2e-3)


@pytest.mark.parametrize("rec", gate_fixture(), ids=lambda r: r["name"])
def test_gate_oracle_reproduces_reference_traces(rec):
    pcm = stream_pcm(rec)
    g = rec["gate"]
    cfg = GateConfig(pre_speech_silence=g["pre_speech_silence"], speech_duration_min=g["speech_duration_min"],
                     speech_duration_max=g["speech_duration_max"], post_speech_silence=g["post_speech_silence"],
                     reentry_timeout=g.get("reentry_timeout"), block=g.get("block", 1600),
                     buffer_seconds=g.get("buffer_seconds", 10))
    det = run_stream(pcm, cfg)
    evs = [e for e in det.events if not e.skipped]
    assert [(e.tick, e.length) for e in evs] == [(e["tick"], e["length"]) for e in rec["events"]]
    assert [sha(e.audio) for e in evs] == [e["sha256"] for e in rec["events"]]
    if "reentries" in rec:
        assert det.reentries == rec["reentries"]


@pytest.mark.parametrize("n", [0, 1, 3, 7, 8, 9, 15, 16, 100, 127, 128, 129, 200, 512, 1000, 1600, 8192, 8193, 20000])
def test_pairwise_order_is_numpys(n):
    rng = np.random.default_rng(n)
    for _ in range(5):
        a = rng.standard_normal(n).astype(np.float32).astype(np.float64) ** 2
        assert pairwise_sum_f64(a) == float(np.add.reduce(a))


@pytest.mark.parametrize("nb", [1, 2, 3, 4, 5, 99, 100, 101, 102, 312])
def test_percentile_restatement(nb):
    rng = np.random.default_rng(nb)
    v = rng.random(nb)
    q = 0.25
    vi = nb * q + (1 + q * (1 - 1 - 1)) - 1
    prev = int(np.floor(vi))
    if vi >= nb - 1:
        a = b = np.sort(v)[-1]
    else:
        a, b = np.sort(v)[prev], np.sort(v)[prev + 1]
    g = vi - np.floor(vi)
    r = a + (b - a) * g
    if g >= 0.5:
        r = b - (b - a) * (1 - g)
    assert r == np.percentile(v, 25)
