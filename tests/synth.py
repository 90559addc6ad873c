"""Deterministic synthetic audio for parity tests and golden generation (test infra).

Stream recipe: ``prefill`` seconds of
N(0, sigma) noise, then ``n_words`` x [U(0.9, 2.0) s of noise, one *event*,
1.0 s of noise].  Events are the reference word scaled by ``gain`` or, when
``distractors`` is on, an 880 Hz burst, a noise burst, or the time-reversed
word.  Everything is float32 and generated from numpy PCG64 with a fixed seed,
so the same recipe reproduces the same samples on any box with this image.
"""
from __future__ import annotations

import os
import wave

import numpy as np

SR = 16000
HERE = os.path.dirname(os.path.abspath(__file__))
WAV = os.path.join(HERE, "golden", "reference_word.wav")


def load_word() -> np.ndarray:
    with wave.open(WAV, "rb") as w:
        raw = w.readframes(w.getnframes())
    return np.frombuffer(raw, dtype="<i2").astype(np.float32) / np.float32(32768.0)


def make_stream(seed: int, n_words: int = 8, prefill: float = 10.0, sigma: float = 1e-3,
                gain: float = 1.0, distractors: bool = False, block: int = 1600, kinds=None):
    """Returns (pcm float32 padded to a multiple of `block`, list of (start, kind)).

    kinds: explicit event kinds, cycled (no random kind draw), including the level-2
    rejects: "hp" (differenced white noise x 0.1: scores ~68 < 75), "hp_near" (x 0.05:
    ~73-75, near the threshold), "white" (loud white noise: negative similarity -> NaN)
    "burst" (the word's first 0.3 s) and "long" (a 3.2 s harmonic hum: longer than max_segment_seconds when the gate's
    speech_duration_max allows it, so the reference skips level 2, wakeword.py:1113-1118)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    word = load_word()
    parts = [rng.normal(0.0, sigma, int(prefill * SR)).astype(np.float32)]
    pos = len(parts[0])
    events = []
    for i in range(n_words):
        gap = rng.normal(0.0, sigma, int(rng.uniform(0.9, 2.0) * SR)).astype(np.float32)
        parts.append(gap)
        pos += len(gap)
        kind = "word"
        if kinds:
            kind = kinds[i % len(kinds)]
        elif distractors:
            kind = ["word", "tone880", "noise", "reversed"][int(rng.integers(0, 4))]
        if kind == "word":
            ev = word * np.float32(gain)
        elif kind == "reversed":
            ev = word[::-1] * np.float32(gain)
        elif kind in ("hp", "hp_near"):
            ev = (np.diff(rng.standard_normal(len(word) + 1)) * (0.1 if kind == "hp" else 0.05) * gain)
            ev = ev.astype(np.float32)
        elif kind == "burst":
            ev = word[:4800] * np.float32(gain)
        elif kind == "white":
            ev = (rng.standard_normal(len(word)) * 0.8 * gain).astype(np.float32)
        elif kind == "long":
            t = np.arange(int(3.2 * SR)) / SR
            env = np.minimum(1.0, np.minimum(t, t[-1] - t) / 0.05)
            ev = ((0.3 * np.sin(2 * np.pi * 150 * t) + 0.2 * np.sin(2 * np.pi * 500 * t)
                   + 0.1 * np.sin(2 * np.pi * 1500 * t)) * env * gain).astype(np.float32)
        elif kind == "tone880":
            t = np.arange(len(word)) / SR
            env = np.sin(np.pi * t / t[-1]) ** 0.5
            ev = (0.3 * gain * env * np.sin(2 * np.pi * 880 * t)).astype(np.float32)
        else:
            t = np.arange(len(word)) / SR
            env = np.sin(np.pi * t / t[-1]) ** 0.5
            ev = (0.15 * gain * env * rng.standard_normal(len(word))).astype(np.float32)
        ev = ev + rng.normal(0.0, sigma, len(ev)).astype(np.float32)
        parts.append(ev.astype(np.float32))
        events.append((pos, kind))
        pos += len(ev)
        tail = rng.normal(0.0, sigma, SR).astype(np.float32)
        parts.append(tail)
        pos += len(tail)
    pcm = np.concatenate(parts).astype(np.float32)
    pad = (-len(pcm)) % block
    if pad:
        pcm = np.concatenate([pcm, rng.normal(0.0, sigma, pad).astype(np.float32)])
    return pcm, events


def tone(freq: float, seconds: float = 1.0, amp: float = 0.5) -> np.ndarray:
    """generate_wav() of tests/test_wakeword_simulated.py:46-51 followed by the
    soundfile PCM16 write/read round trip (write x*32767 rounded, read /32768)."""
    t = np.linspace(0, seconds, int(SR * seconds), endpoint=False)
    a = (amp * np.sin(2 * np.pi * freq * t)).astype(np.float32)
    return pcm16_roundtrip(a)


def speech_like(seconds: float = 1.0) -> np.ndarray:
    """generate_speech_like_audio() of tests/test_wakeword_simulated.py:54-67 (+ PCM16 round trip)."""
    t = np.linspace(0, seconds, int(SR * seconds), endpoint=False)
    a = (0.3 * np.sin(2 * np.pi * 150 * t) + 0.2 * np.sin(2 * np.pi * 500 * t)
         + 0.15 * np.sin(2 * np.pi * 1500 * t) + 0.1 * np.sin(2 * np.pi * 2500 * t))
    env = np.sin(np.pi * t / seconds) ** 0.5
    return pcm16_roundtrip((a * env).astype(np.float32))


def pcm16_roundtrip(x: np.ndarray) -> np.ndarray:
    q = np.clip(np.round(np.asarray(x, np.float64) * 32767.0), -32768, 32767).astype(np.int16)
    return q.astype(np.float32) / np.float32(32768.0)


def ragged_segments(seed: int, n: int, lo: int = 6400, hi: int = 33600, sigma=(1e-4, 5e-3)):
    """Segment batch like the kernel microbench: lengths U{lo..hi}, half positives
    (gain-scaled word embedded in noise), half distractors."""
    rng = np.random.Generator(np.random.PCG64(seed))
    word = load_word()
    segs = []
    for i in range(n):
        L = int(rng.integers(lo, hi + 1))
        s = float(rng.uniform(*sigma))
        x = rng.normal(0.0, s, L).astype(np.float32)
        kind = int(rng.integers(0, 4))
        g = float(rng.uniform(0.2, 3.0))
        off = int(rng.integers(0, max(1, L - len(word))))
        if kind == 0 or kind == 1:
            w = word[: L - off] * np.float32(g)
            x[off:off + len(w)] += w
        elif kind == 2:
            t = np.arange(min(L - off, len(word))) / SR
            x[off:off + len(t)] += (0.3 * g * np.sin(2 * np.pi * 880 * t)).astype(np.float32)
        else:
            w = word[::-1][: L - off] * np.float32(g)
            x[off:off + len(w)] += w
        segs.append(x.astype(np.float32))
    return segs


def matcher_cases():
    """The named segment set of tests/golden/matcher_cases.json (inputs are
    regenerated here; the fixture stores their sha256 and the reference outputs)."""
    cases = []
    word = load_word()
    cases.append(("word_self", word))
    cases.append(("word_half", word * np.float32(0.5)))
    cases.append(("word_reversed", word[::-1].copy()))
    cases.append(("tone440", tone(440)))
    cases.append(("tone880", tone(880)))
    cases.append(("speech_like", speech_like()))
    rs = np.random.RandomState(42)          # test_wakeword_simulated.py:165-166
    cases.append(("noise_seed42", rs.randn(16000).astype(np.float32) * np.float32(0.1)))
    cases.append(("short_1", np.full(1, 0.25, np.float32)))
    cases.append(("short_159", ragged_segments(7, 1, 159, 159)[0]))
    cases.append(("short_160", ragged_segments(8, 1, 160, 160)[0]))
    cases.append(("short_511", ragged_segments(9, 1, 511, 511)[0]))
    cases.append(("len_16000", ragged_segments(10, 1, 16000, 16000)[0]))
    cases.append(("len_48000", ragged_segments(11, 1, 48000, 48000)[0]))
    # digital silence around speech forces the top_db clamp (max - 80 dB)
    cases.append(("word_zero_padded",
                  np.concatenate([np.zeros(4000, np.float32), word, np.zeros(4000, np.float32)])))
    for i, seg in enumerate(ragged_segments(1234, 40)):
        cases.append((f"ragged_{i:02d}", seg))
    cases.append(("silence_6400", np.zeros(6400, np.float32)))
    cases.append(("silence_16000", np.zeros(16000, np.float32)))
    # audible level-2 rejects and near-threshold cases (differenced / twice-differenced
    # white noise: high-passed spectra score 0-75 against the word; loud white noise
    # drives the similarity negative -> NaN)
    rng = np.random.Generator(np.random.PCG64(4242))
    n = len(word)
    for g in (0.03, 0.04, 0.045, 0.05, 0.055, 0.06, 0.1, 0.2, 0.5, 1.0):
        cases.append((f"hp_noise_{g:g}", (np.diff(rng.standard_normal(n + 1)) * g).astype(np.float32)))
    for g in (0.05, 0.2):
        cases.append((f"hp2_noise_{g:g}", (np.diff(rng.standard_normal(n + 2), 2) * g).astype(np.float32)))
    for g in (0.5, 1.5):
        cases.append((f"white_{g:g}", (rng.standard_normal(n) * g).astype(np.float32)))
    # a word buried in high-passed noise (mixtures near the decision)
    for g in (0.3, 0.6):
        cases.append((f"word_in_hp_{g:g}", (word * np.float32(g) + np.diff(rng.standard_normal(n + 1)) * 0.08)
                      .astype(np.float32)))
    return [(n, np.ascontiguousarray(x, dtype=np.float32)) for n, x in cases]


def fuzz_segments(seed: int, n: int, word: np.ndarray) -> list:
    """The top_db fuzz recipe (tests/test_gpu_scorer.py): lengths 1-60000, a noise floor of
    1e-7..1e-2, 0-4 bursts (the word, a tone or white noise, 0-100 dB above the floor) at
    random places, a 3000-sample digital-silence stretch every 7th segment and two identical
    2560-sample tiles (a scout tie) every 11th."""
    rng = np.random.Generator(np.random.PCG64(seed))
    segs = []
    for k in range(n):
        L = int(rng.integers(1, 60001))
        x = (rng.normal(0, 1, L) * 10 ** rng.uniform(-7, -2)).astype(np.float32)
        for _ in range(int(rng.integers(0, 5))):
            m = int(rng.integers(200, 12000))
            s0 = int(rng.integers(0, max(1, L - m)))
            amp = np.float32(10 ** rng.uniform(-5, 0))
            kind = int(rng.integers(0, 3))
            if kind == 0:
                src = word[:m] if m <= len(word) else np.resize(word, m)
            elif kind == 1:
                src = np.sin(2 * np.pi * rng.uniform(100, 7000) * np.arange(m) / 16000).astype(np.float32)
            else:
                src = rng.normal(0, 1, m).astype(np.float32)
            c = min(m, L - s0)
            x[s0:s0 + c] += amp * src[:c]
        if k % 7 == 0 and L > 4000:       # digital silence stretch
            a = int(rng.integers(0, L - 3000))
            x[a:a + 3000] = 0.0
        if k % 11 == 0 and L > 5120:      # two identical tiles: a tie in the scout ranking
            x[2560:5120] = x[0:2560]
        segs.append(x)
    return segs


MEAN_BAND_KINDS = ("white", "pink", "tone_noise", "word_noise")


def mean_band_segment(kind: str, seed: int, gain: float, length: int) -> np.ndarray:
    """Loud segments of four recipes other than the streaming bench's, for the vanishing-mean
    criterion's evidence (tests/golden/make_mean_band.py picks parameters
    whose oracle MFCC mean vector has |mean| in [32, 64)): white noise, pink (1/f power) noise,
    a tone plus white noise, and the reference word (looped, x 4) in white noise.  (High-passed
    noise and a clipped word never get there: their spectral shape alone keeps |mean| above
    ~110.)  Deterministic in (kind, seed, gain, length)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = int(length)
    if kind == "white":
        x = rng.standard_normal(n) * gain
    elif kind == "pink":
        w = np.fft.rfft(rng.standard_normal(n))
        f = np.arange(len(w), dtype=np.float64)
        f[0] = 1.0
        x = np.fft.irfft(w / np.sqrt(f), n) * gain * np.sqrt(n / 16.0)
    elif kind == "tone_noise":
        t = np.arange(n) / SR
        f0 = float(rng.uniform(150.0, 3000.0))
        x = gain * (np.sin(2 * np.pi * f0 * t) + 0.3 * rng.standard_normal(n))
    elif kind == "word_noise":
        word = load_word().astype(np.float64)
        x = 4.0 * np.resize(word, n) + gain * rng.standard_normal(n)
    else:
        raise ValueError(kind)
    return x.astype(np.float32)
