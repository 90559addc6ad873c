"""Compact sample rings (ewk_config.ring_samples) and the ring-overwrite bound of a
gate launch, on the GPU.

* A compact ring keeps only the samples a segment cut can ask for; the block RMSs
  of the reference's full ring (wakeword.py:472-486) are kept per block as they
  arrive.  Bar: every event field (tick, length, skip flag, score bits, match) and
  every stream's threshold identical to a full-ring engine on the same pushes, and
  the event list identical to the oracle (oracle/gate_ref.py).
* ticks_per_launch: with a short buffer (buffer_seconds 4 or 5) one push_many of a
  whole stream must still score every segment from intact samples (the gate
  launch is cut so later ticks cannot overwrite a segment before it is scored).
* Event queue: an overflowed bank is re-armed (later polls work) and a short poll
  capacity consumes nothing.
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


def _streams(n, block, seed0, n_words=4):
    pcms = []
    for i in range(n):
        rng = np.random.default_rng(seed0 + i)
        p, _ = synth.make_stream(seed=seed0 + 1000 + i, n_words=n_words, sigma=float(rng.uniform(1e-4, 4e-3)),
                                 gain=float(rng.uniform(0.3, 2.5)), distractors=bool(i % 2), block=block)
        pcms.append(p)
    L = min(len(p) for p in pcms)
    L -= L % block
    return np.stack([p[:L] for p in pcms]).astype(np.float32)


def _min_ring(block, max_speech=2.0, post=0.4, pad=0.05):
    need = int((max_speech + post + block / 16000 + pad) * 16000) + 2 + block
    return -(-need // block) * block


def _run(data, block, template, ticks_per_call, **cfg):
    from easywakeword_amd import StreamEngine
    n = data.shape[0]
    eng = StreamEngine(n, block=block, tick_seconds=block / 16000, **cfg)
    eng.set_template(*template)
    got = []
    step = ticks_per_call * block
    for c in range(0, data.shape[1], step):
        eng.push_many(data[:, c:c + step])
        got.append(eng.poll())
    ev = np.concatenate(got)
    thr = [eng.state(i)["silence_threshold"] for i in range(n)]
    eng.close()
    return ev, thr


@pytest.mark.parametrize("block", [1600, 800, 400, 3200])
def test_compact_ring_equals_full_ring_and_oracle(block, template):
    """Blocks of 25-200 ms, each on a real-time virtual clock (tick_seconds = block / 16000)."""
    data = _streams(12, block, 7000 + block)
    ring = _min_ring(block)
    full, thr_f = _run(data, block, template, 7)
    comp, thr_c = _run(data, block, template, 7, ring_samples=ring)
    assert len(full) > 20
    for f in ("stream", "tick", "length", "flags", "match"):
        np.testing.assert_array_equal(comp[f], full[f], err_msg=f)
    np.testing.assert_array_equal(comp["score"].view(np.int64), full["score"].view(np.int64))
    assert thr_c == thr_f
    tm, ts = template
    checked = 0
    for i in range(data.shape[0]):
        ref = run_stream(data[i], GateConfig(block=block, tick_seconds=block / 16000)).events
        mine = comp[comp["stream"] == i]
        assert [(int(m["tick"]), int(m["length"]), bool(m["flags"] & 1)) for m in mine] == \
               [(e.tick, e.length, e.skipped) for e in ref], i
        for m, e in zip(mine, ref):
            if e.skipped or checked >= 12:
                continue
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            assert score_close(float(m["score"]), s, 1e-4), (i, int(m["tick"]), float(m["score"]), s)
            assert bool(m["match"]) == (s >= 75.0)
            checked += 1


def test_compact_ring_read_last_and_segments(template):
    from easywakeword_amd import StreamEngine
    data = _streams(2, 1600, 9100, n_words=3)
    ring = _min_ring(1600)
    eng = StreamEngine(2, ring_samples=ring)
    eng.set_template(*template)
    eng.push_many(data)
    ev = eng.poll()
    assert len(ev) > 0
    # segment samples straight from the compact ring equal the oracle's cut
    ref = run_stream(data[0], GateConfig()).events
    last = [e for e in ref if not e.skipped][-1]
    m = [x for x in ev if x["stream"] == 0 and int(x["tick"]) == last.tick][0]
    seg = eng.read_segment(0, int(m["ring_start"]), int(m["length"]))
    np.testing.assert_array_equal(seg.astype(np.float64), last.audio)
    np.testing.assert_array_equal(eng.read_last(1, 1600), data[1, -1600:])
    np.testing.assert_array_equal(eng.read_last(1, ring), data[1, -ring:])
    with pytest.raises(ValueError):
        eng.read_last(1, ring + 1)           # more than the compact ring keeps
    eng.close()


@pytest.mark.parametrize("buffer_seconds", [4, 5])
def test_short_buffer_push_many_scores_intact_segments(buffer_seconds, template):
    """a 32-tick gate launch would overwrite segments of a 4-5 s ring before
    the scorer reads them; the launch is now cut to what the ring can hold."""
    block = 1600
    data = _streams(6, block, 9300 + buffer_seconds, n_words=5)
    ev, _ = _run(data, block, template, data.shape[1] // block, buffer_seconds=buffer_seconds)
    tm, ts = template
    n_scored = 0
    for i in range(data.shape[0]):
        ref = run_stream(data[i], GateConfig(buffer_seconds=buffer_seconds)).events
        mine = ev[ev["stream"] == i]
        assert [(int(m["tick"]), int(m["length"]), bool(m["flags"] & 1)) for m in mine] == \
               [(e.tick, e.length, e.skipped) for e in ref], i
        for m, e in zip(mine, ref):
            if e.skipped:
                continue
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            assert score_close(float(m["score"]), s, 1e-4), (i, int(m["tick"]), float(m["score"]), s)
            assert bool(m["match"]) == (s >= 75.0)
            n_scored += 1
    assert n_scored >= 10


def test_event_overflow_rearms_and_short_cap_consumes_nothing(template):
    """after an overflow every later poll used to fail; a short poll buffer
    used to lose the older bank."""
    from easywakeword_amd import StreamEngine
    import bench
    import torch
    dev = torch.device("cuda", 0)
    n = 1024                                   # event bank capacity max(4096, 4n) = 4096
    sig = bench.make_shifted_signal(torch, dev, n, 1200, 77, synth.load_word())
    eng = StreamEngine(n)
    eng.set_template(*template)
    t = 0

    def push(nt):
        nonlocal t
        eng.push_device(sig.data_ptr() + t * 1600 * 4, 1600, 1600, nt)
        t += nt

    push(100)
    eng.poll()
    push(1000)                                 # ~ 0.3 events/s/stream x 100 s x 1024 streams >> 4096
    with pytest.raises(MemoryError):
        eng.poll()
    push(40)                                   # the engine keeps working after the overflow
    ev = eng.poll()
    assert 0 < len(ev) < 4096
    push(40)
    with pytest.raises(ValueError):
        eng.poll(cap=1)                        # too small: nothing consumed
    ev2 = eng.poll()
    assert len(ev2) > 1
    assert (ev2["tick"] > ev["tick"].max()).all()
    eng.close()
