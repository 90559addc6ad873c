"""The fp64 re-score's speculative top_db clamp on values AT the threshold (ewk_rescore.h).

The re-score splits each chunk's DCT at theta_s, the float32 pass's max - 80 dB, and is exact
for the fp64 theta when no log-mel value lies within kRsWindow (2e-4 dB since round 6, measured
|theta - theta_s| <= 2e-5 dB: scripts/rs_window_probe.py) of theta_s; a chunk holding such a
value is recomputed with the exact theta by the slot's finishing wave.  Natural audio puts a
value there about once per 1,000-5,000 chunks, so this builds segments that do it on purpose:
a loud tone sets the segment max M, a second tone in other frames is scaled (from the oracle's
own float64 log-mel) so that its peak band lands at M - 80 dB, or a few 1e-6..1e-4 dB either
side of it, in chunk 0, a middle chunk or the last (partial) one.  Both fp64 paths -- serial
slots (`score_f64`, ewk_score_segments_f64) and chunked slots through the part pool
(rescore_margin = 1e9: every segment listed) -- must give the oracle's float64 mean / std /
score within 1e-9 (wakeword.py:544-567, 591-625).
"""
import numpy as np
import pytest

from golden_io import score_close
from oracle import mfcc_ref

pytestmark = pytest.mark.gpu

SR = 16000


def _tone(L, f, a, s0, s1):
    y = np.zeros(L)
    t = np.arange(s1 - s0) / SR
    y[s0:s1] = a * np.sin(2 * np.pi * f * t) * np.hanning(s1 - s0)
    return y


def _raw_log_mel(y):
    """oracle float64 log-mel [128, T] before the top_db clamp."""
    mel_basis, _ = mfcc_ref._tables()
    S = mfcc_ref.power_spectrogram(y.astype(np.float64))
    return 10.0 * np.log10(np.maximum(mfcc_ref.AMIN, np.einsum("ft,mf->mt", S, mel_basis)))


def _segments():
    rng = np.random.default_rng(20261018)
    segs = []
    for i in range(18):
        L = int([6400, 16000, 16037 + 160 * i, 33600][i % 4])
        fa, fb = float(rng.uniform(300, 2000)), float(rng.uniform(2500, 6000))
        la, lb = int(rng.integers(800, 1500)), 1200
        # the quiet tone in chunk 0, a middle chunk or the last (partial) one; the loud tone
        # >= 600 samples away (no shared STFT window)
        where = i % 3
        sb = [0, L // 2 - lb // 2, L - lb][where]
        sa = L - la - 600 if where == 0 else 100
        loud = _tone(L, fa, float(rng.uniform(0.2, 0.9)), sa, sa + la)
        quiet1 = _tone(L, fb, 1.0, sb, sb + lb)
        M = _raw_log_mel(loud).max()
        b0 = _raw_log_mel(quiet1).max()
        delta = [0.0, 3e-6, -3e-6, 5e-5, -5e-5, 1.5e-4][i % 6]       # dB from M - 80
        quiet = quiet1 * 10 ** ((M - 80.0 + delta - b0) / 20.0)
        assert abs(_raw_log_mel(quiet).max() - (M - 80.0 + delta)) < 1e-9
        y = loud + quiet
        assert abs(_raw_log_mel(y).max() - M) < 1e-9                 # the quiet tone does not move the max
        segs.append(y.astype(np.float32))
    return segs


@pytest.fixture(scope="module")
def segments():
    return _segments()


def _template():
    from synth import load_word
    return mfcc_ref.extract_mfcc(load_word().astype(np.float32))


def _check(mean, std, score, segs, tm, ts):
    for i, y in enumerate(segs):
        cm, cs = mfcc_ref.extract_mfcc(y.astype(np.float64))
        np.testing.assert_allclose(mean[i], cm, rtol=1e-9, atol=1e-9, err_msg=str(i))
        np.testing.assert_allclose(std[i], cs, rtol=1e-9, atol=1e-9, err_msg=str(i))
        s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
        assert score_close(score[i], s, 1e-9), (i, score[i], s)


def test_values_at_the_threshold_serial_slots(segments):
    from easywakeword_amd import Engine
    tm, ts = _template()
    e = Engine()
    e.set_template(tm.astype(np.float32), ts.astype(np.float32))
    mean, std, score = e.score_f64(segments)
    e.close()
    _check(mean, std, score, segments, tm.astype(np.float32), ts.astype(np.float32))


def test_values_at_the_threshold_chunked_slots(segments):
    from easywakeword_amd import Engine
    tm, ts = _template()
    e = Engine(rescore_margin=1e9)
    e.set_template(tm.astype(np.float32), ts.astype(np.float32))
    _, _, score, _ = e.score(segments, candidate_dtype="float64")
    e.close()
    tm32, ts32 = tm.astype(np.float32), ts.astype(np.float32)   # (scipy's uu of a float32 template is float32)
    for i, y in enumerate(segments):
        cm, cs = mfcc_ref.extract_mfcc(y.astype(np.float64))
        s = float(mfcc_ref.similarity_from_stats(tm32, ts32, cm, cs))
        assert score_close(score[i], s, 1e-9), (i, score[i], s)
