"""WAV ingest: librosa.load(sr=16000) semantics of load_wav.
16 kHz PCM16 is bit-exact (int16 / 32768); other rates are resampled on the host
(polyphase FIR; librosa's soxr is absent -- parity unpinned, checked here only for
length, band-limited accuracy on a tone, and that the result scores like the
original through the oracle)."""
import numpy as np
import pytest

import synth
from easywakeword_amd.audio import load_wav, resample, write_wav


def test_16k_pcm16_is_bit_exact(tmp_path):
    p = tmp_path / "w.wav"
    x = synth.load_word()
    write_wav(str(p), x)
    y = load_wav(str(p))
    assert y.dtype == np.float32
    np.testing.assert_array_equal(y, x)        # x is already int16 / 32768: the round trip is exact


@pytest.mark.parametrize("sr", [8000, 22050, 44100, 48000])
def test_other_rates_are_resampled(tmp_path, sr):
    t = np.arange(int(sr * 0.5)) / sr
    tone = 0.4 * np.sin(2 * np.pi * 440.0 * t)
    p = tmp_path / f"t{sr}.wav"
    import wave
    q = np.round(tone * 32767).astype("<i2")
    with wave.open(str(p), "wb") as w:
        w.setnchannels(1); w.setsampwidth(2); w.setframerate(sr); w.writeframes(q.tobytes())
    y = load_wav(str(p))
    assert len(y) == int(np.ceil(len(q) * 16000 / sr))
    tt = np.arange(len(y)) / 16000
    ref = 0.4 * np.sin(2 * np.pi * 440.0 * tt)
    mid = slice(400, len(y) - 400)                 # away from the filter's edge transients
    assert np.max(np.abs(y[mid] - ref[mid])) < 2e-3


def test_resampled_word_scores_like_the_original():
    from oracle import mfcc_ref
    x = synth.load_word()
    up = resample(x, 16000, 44100)
    back = resample(up, 44100, 16000)
    assert abs(len(back) - len(x)) <= 1
    tm, ts = mfcc_ref.extract_mfcc(x)
    cm, cs = mfcc_ref.extract_mfcc(back[:len(x)].astype(np.float64))
    assert float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs)) > 99.0
