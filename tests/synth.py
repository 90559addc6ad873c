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
                gain: float = 1.0, distractors: bool = False, block: int = 1600):
    """Returns (pcm float32 padded to a multiple of `block`, list of (start, kind))."""
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
        if distractors:
            kind = ["word", "tone880", "noise", "reversed"][int(rng.integers(0, 4))]
        if kind == "word":
            ev = word * np.float32(gain)
        elif kind == "reversed":
            ev = word[::-1] * np.float32(gain)
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
    return [(n, np.ascontiguousarray(x, dtype=np.float32)) for n, x in cases]
