"""The data formats either side of the path on the GPU:

* level-3 input: WakeWord._transcribe_audio's normalisation (reference
  wakeword.py:1019-1025), bit-identical to the reference's numpy expression,
  for linear batches and for gated events read straight from the stream rings;
* PCM16 ingest: int16 -> float32 decode (librosa.load / soundfile value for a
  16 kHz PCM16 WAV: int16 / 32768) and int16 streaming pushes, which must gate
  exactly like the float32 pushes of the decoded audio.
"""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


def _numpy_normalize(x):
    """wakeword.py:1019-1025 verbatim on the float64 ring slice."""
    a = np.asarray(x, dtype=np.float64)
    a = a - np.mean(a)
    max_val = np.max(np.abs(a))
    if max_val > 0:
        a = a / max_val
    a = a * 1.5
    return np.clip(a, -1.0, 1.0)


LENGTHS = [1, 2, 7, 8, 9, 100, 127, 128, 129, 1000, 4097, 8191, 8192, 8193, 16384, 16391, 24577, 48000]


def test_normalize_linear_bit_exact():
    from easywakeword_amd import Engine
    rng = np.random.default_rng(5)
    segs = []
    for i, n in enumerate(LENGTHS):
        x = (rng.standard_normal(n) * 10 ** rng.uniform(-4, 0) + rng.uniform(-0.1, 0.1)).astype(np.float32)
        segs.append(x)
    segs.append(np.full(3000, 0.25, np.float32))      # constant: max|y| == 0, no scaling
    segs.append(np.zeros(1600, np.float32))           # silence
    segs.append(synth.load_word())                     # the reference word
    out = Engine().normalize(segs)
    assert len(out) == len(segs)
    for x, y in zip(segs, out):
        want = _numpy_normalize(x)
        assert y.dtype == np.float64 and y.shape == want.shape
        np.testing.assert_array_equal(y, want)


def test_normalize_events_from_rings_bit_exact():
    from easywakeword_amd import StreamEngine
    parts = [synth.make_stream(seed, n_words=4)[0] for seed in (1, 2, 3)]
    n = min(len(p) for p in parts) // 1600 * 1600
    pcm = np.stack([p[:n] for p in parts]).astype(np.float32)
    n_ticks = pcm.shape[1] // 1600
    eng = StreamEngine(3)
    eng.template_from_pcm(synth.load_word())
    evs = []
    for t0 in range(0, n_ticks, 16):
        nt = min(16, n_ticks - t0)
        eng.push_many(pcm[:, t0 * 1600:(t0 + nt) * 1600])
        ev = eng.poll()
        ev = ev[(ev["flags"] & 1) == 0]
        if len(ev):   # normalise before the rings move on
            outs = eng.normalize_events(ev)
            outs_dev = eng.normalize_events_device(ev)   # the confirm stage's device-resident copy
            for e, y, yd in zip(ev, outs, outs_dev):
                audio = eng.read_segment(int(e["stream"]), int(e["ring_start"]), int(e["length"]))
                np.testing.assert_array_equal(y, _numpy_normalize(audio))
                np.testing.assert_array_equal(yd.cpu().numpy(), y)
            evs.extend(ev)
    assert len(evs) >= 6


def test_decode_pcm16_exact():
    from easywakeword_amd import Engine
    rng = np.random.default_rng(9)
    x = rng.integers(-32768, 32768, 100003).astype(np.int16)
    x[:4] = [-32768, 32767, 0, -1]
    y = Engine().decode_pcm16(x)
    np.testing.assert_array_equal(y, x.astype(np.float32) / np.float32(32768.0))


def test_push_pcm16_gates_like_float32():
    from easywakeword_amd import StreamEngine
    streams = [synth.make_stream(seed, n_words=3)[0] for seed in (11, 12)]
    n = min(len(x) for x in streams) // 1600 * 1600
    streams = [x[:n] for x in streams]
    pcm16 = np.stack([np.clip(np.round(s * 32768.0), -32768, 32767).astype(np.int16) for s in streams])
    pcm32 = pcm16.astype(np.float32) / np.float32(32768.0)
    n_ticks = pcm16.shape[1] // 1600
    a, b = StreamEngine(2), StreamEngine(2)
    for e in (a, b):
        e.template_from_pcm(synth.load_word())
    ev_a, ev_b = [], []
    for t0 in range(0, n_ticks, 8):
        nt = min(8, n_ticks - t0)
        a.push_pcm16(pcm16[:, t0 * 1600:(t0 + nt) * 1600])
        b.push_many(pcm32[:, t0 * 1600:(t0 + nt) * 1600])
        ev_a.append(a.poll())
        ev_b.append(b.poll())
    ev_a, ev_b = np.concatenate(ev_a), np.concatenate(ev_b)
    assert len(ev_a) >= 4
    np.testing.assert_array_equal(ev_a, ev_b)
    for s in range(2):
        assert a.state(s) == b.state(s)
