"""Level-1 (+2) parity on the GPU: the streaming engine vs traces of the REAL
reference SoundBuffer + WakeWord._detect_word (tests/golden/gate_traces.json)
and vs the oracle restatement (oracle/gate_ref.py) on many streams.

Bar: bit-identical gate decisions (per-tick is_silent, thresholds, segment
ticks/lengths/samples), scores within 1e-4, identical match decisions.
"""
import numpy as np
import pytest

import synth
from golden_io import gate_fixture, matcher_fixture, score_close, sha, stream_pcm, template_arrays
from oracle import mfcc_ref
from oracle.gate_ref import GateConfig, run_stream

pytestmark = pytest.mark.gpu


def _engine(n, gate, **extra):
    from easywakeword_amd import StreamEngine
    kw = dict(pre_speech_silence=gate["pre_speech_silence"], speech_duration_min=gate["speech_duration_min"],
              speech_duration_max=gate["speech_duration_max"], post_speech_silence=gate["post_speech_silence"],
              buffer_seconds=gate.get("buffer_seconds", 10), block=gate.get("block", 1600),
              reentry_timeout=float(gate.get("reentry_timeout") or 0.0))
    kw.update(extra)
    return StreamEngine(n, **kw)


@pytest.fixture(scope="module")
def template():
    fx, _ = matcher_fixture()
    return template_arrays(fx)


@pytest.mark.parametrize("rec", gate_fixture(), ids=lambda r: r["name"])
def test_reference_trace_tick_by_tick(rec, template):
    pcm = stream_pcm(rec)
    eng = _engine(1, rec["gate"])
    eng.set_template(*template)
    block = rec["gate"]["block"]
    silent = {}
    thr = {}
    for (k, s), t in zip(rec["silent"], rec["threshold"]):
        silent.setdefault(k, []).append(s)
        thr.setdefault(k, []).append(t)
    events = []
    for k in range(len(pcm) // block):
        eng.push(pcm[k * block:(k + 1) * block].reshape(1, -1))
        st = eng.state(0)
        tick = k + 1
        if tick in silent:   # every is_silent() the reference made at this clock value
            assert all(bool(st["last_silent"]) == s for s in silent[tick]), (tick, st, silent[tick])
            assert all(st["silence_threshold"] == t for t in thr[tick]), (tick, st["silence_threshold"], thr[tick])
        for ev in eng.poll():
            if ev["flags"] & 1:
                continue
            audio = eng.read_segment(0, int(ev["ring_start"]), int(ev["length"]))
            events.append((int(ev["tick"]), int(ev["length"]), sha(audio.astype(np.float64)), float(ev["score"]),
                           bool(ev["match"])))
    ref = [(e["tick"], e["length"], e["sha256"], e["score"], e["match"]) for e in rec["events"]]
    assert [e[:3] for e in events] == [r[:3] for r in ref]
    for e, r in zip(events, ref):
        assert score_close(e[3], r[3], 1e-4), (e, r)
        assert e[4] == r[4]


def _oracle_events(pcm, gate):
    cfg = GateConfig(pre_speech_silence=gate["pre_speech_silence"], speech_duration_min=gate["speech_duration_min"],
                     speech_duration_max=gate["speech_duration_max"],
                     post_speech_silence=gate["post_speech_silence"], block=gate.get("block", 1600),
                     reentry_timeout=gate.get("reentry_timeout"))
    return run_stream(pcm, cfg).events


def test_many_streams_vs_oracle(template):
    """32 streams with different gains / noise / distractors, pushed 16 ticks at a time."""
    gate = dict(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0, post_speech_silence=0.4)
    n = 32
    pcms = []
    for i in range(n):
        rng = np.random.default_rng(500 + i)
        p, _ = synth.make_stream(seed=2000 + i, n_words=4, sigma=float(rng.uniform(1e-4, 5e-3)),
                                 gain=float(rng.uniform(0.2, 3.0)), distractors=bool(i % 2))
        pcms.append(p)
    L = min(len(p) for p in pcms)
    L -= L % 1600
    data = np.stack([p[:L] for p in pcms]).astype(np.float32)
    eng = _engine(n, gate)
    eng.set_template(*template)
    got = []
    step = 16 * 1600
    for c in range(0, L, step):
        eng.push_many(data[:, c:c + step])
        got.extend(eng.poll().tolist())
    tm, ts = template
    n_ev = 0
    bad = []   # every mismatch, not the first: the evidence is dumped before the test fails
    for i in range(n):
        ref = _oracle_events(data[i], gate)
        mine = sorted([g for g in got if g[0] == i], key=lambda g: g[2])
        if [(g[2], g[1], bool(g[7] & 1)) for g in mine] != [(e.tick, e.length, e.skipped) for e in ref]:
            bad.append(dict(stream=i, why="identity", mine=mine, want=[(e.tick, e.length, e.skipped) for e in ref]))
            continue
        for g, e in zip(mine, ref):
            if e.skipped:
                continue
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            if not score_close(g[5], s, 1e-4) or bool(g[6]) != (s >= 75.0):
                bad.append(dict(stream=i, why="score", mine=g, oracle=s))
            n_ev += 1
            # the ring still holding this segment (the last 10 s): its samples, bit for bit
            p0 = g[2] * 1600 - (g[2] * 1600 - g[3]) % 160000        # segment start in the stream
            if p0 >= L - 160000:
                back = eng.read_segment(i, g[3], g[1])
                want = np.asarray(e.audio, np.float32)
                diff = np.nonzero(back != want)[0]
                if len(diff):
                    j = p0 + diff[:64]
                    bad.append(dict(stream=i, why="ring", mine=g, n_diff=int(len(diff)), first=int(diff[0]),
                                    last=int(diff[-1]), idx=diff[:64], got=back[diff[:64]], want=want[diff[:64]],
                                    stale=data[i][np.maximum(j - 160000, 0)], tick_before=data[i][np.maximum(j - 1600, 0)],
                                    other_streams=[int(k) for k in np.nonzero((data[:, j[0]] == back[diff[0]]))[0]]))
    if bad:
        from evidence import dump
        from easywakeword_amd import Engine
        lin = Engine()
        lin.set_template(tm, ts)
        for b in bad:   # the ring's samples now (if not yet overwritten) and the linear scorer's view
            g = b["mine"]
            p0 = g[2] * 1600 - (g[2] * 1600 - g[3]) % 160000        # segment start in the stream
            if b["why"] == "score" and p0 >= L - 150000:                   # not yet overwritten
                back = eng.read_segment(g[0], g[3], g[1])
                b["ring_back_linear_score"] = float(lin.score([back], candidate_dtype="float64")[2][0])
        lin.close()
        from easywakeword_amd import _lib
        lib = _lib.load()
        if hasattr(lib, "ewk_debug_coop"):   # -DEWK_COOP_DEBUG builds: what each wave of the scorer saw
            ev = np.zeros((8192, 8, 4), np.int32)
            th = np.zeros((8192, 8, 4), np.float32)
            pd = np.zeros((8192, 8, 60), np.float64)
            ms = np.zeros((8192, 40), np.float32)
            import ctypes
            vp = lambda a: ctypes.c_void_p(a.ctypes.data)   # (a bare int would pass as a 32-bit C int)
            if lib.ewk_debug_coop(vp(ev), vp(th), vp(pd), vp(ms)) == 0:
                for b in bad:
                    g = b["mine"]
                    key = (g[0] & 31) * 256 + (g[2] & 255)
                    b["coop"] = dict(ev=ev[key], th=th[key], pd=pd[key], ms=ms[key])
                    if key < 1024 and hasattr(lib, "ewk_debug_coop_tile"):
                        tl = np.zeros((8, 512, 4), np.uint32)
                        if lib.ewk_debug_coop_tile(ctypes.c_int(key), vp(tl)) == 0:
                            b["coop"]["tile"] = tl
        path = dump("many_streams", dict(bad=bad, events=got))
        pytest.fail(f"{len(bad)} mismatches (evidence {path}): {bad[:4]}")
    assert n_ev > 20


def test_ring_tick_fp64_rescore_in_last_workgroup(template):
    """rescore_margin = 1e9: every ring segment is queued for the fp64 re-score, which the
    tick's re-score launch (k_rescore_ring, right after the scorer) drains: all events carry
    EWK_EV_RESCORED and the float64 reference score within 1e-9, over several ticks per
    push and several pushes (the watermark advances in the same tick end)."""
    gate = dict(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0, post_speech_silence=0.4)
    n = 12
    pcms = []
    for i in range(n):
        rng = np.random.default_rng(900 + i)
        p, _ = synth.make_stream(seed=4000 + i, n_words=3, sigma=float(rng.uniform(1e-4, 3e-3)),
                                 gain=float(rng.uniform(0.3, 2.0)), distractors=bool(i % 2))
        pcms.append(p)
    L = min(len(p) for p in pcms)
    L -= L % 1600
    data = np.stack([p[:L] for p in pcms]).astype(np.float32)
    eng = _engine(n, gate, rescore_margin=1e9)
    eng.set_template(*template)
    got = []
    for c in range(0, L, 8 * 1600):
        eng.push_many(data[:, c:c + 8 * 1600])
        got.extend(eng.poll().tolist())
    tm, ts = template
    n_ev = 0
    for i in range(n):
        ref = _oracle_events(data[i], gate)
        mine = sorted([g for g in got if g[0] == i], key=lambda g: g[2])
        assert [(g[2], g[1], bool(g[7] & 1)) for g in mine] == [(e.tick, e.length, e.skipped) for e in ref], i
        for g, e in zip(mine, ref):
            if e.skipped:
                continue
            # EWK_EV_RESCORED (a NaN score is listed by the margin only through another criterion,
            # and a vanishing-mean NaN beyond the float32 error not at all: kNanMarginA)
            assert g[7] & 2 or np.isnan(g[5]), (i, g)
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            assert score_close(g[5], s, 1e-9), (i, g, s)
            assert bool(g[6]) == (s >= 75.0)
            n_ev += 1
    assert n_ev >= 12


def test_unaligned_block_512_thresholds():
    """frame_size 512: 312 physical blocks, the write pointer is not block-aligned
    after the first wrap -> exercises the incremental block-RMS refresh."""
    gate = dict(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0,
                post_speech_silence=0.4, block=512)
    pcm, _ = synth.make_stream(seed=77, n_words=3, sigma=2e-3, gain=1.0, block=512)
    eng = _engine(1, gate)
    cfg = GateConfig(block=512)
    from oracle.gate_ref import DetectorRef
    det = DetectorRef(cfg)
    for k in range(len(pcm) // 512):
        blk = pcm[k * 512:(k + 1) * 512]
        eng.push(blk.reshape(1, -1))
        det.push_tick(blk)
        st = eng.state(0)
        assert st["silence_threshold"] == det.buf.silence_threshold, k
        if det.started and det.buf.is_buffer_full():
            assert bool(st["last_silent"]) == det.buf.is_silent(), k
            assert st["state"] == det.state, k


def test_lagged_poll_pipelines_one_call_behind():
    """ewk_poll_lagged returns exactly the events a blocking poll returns, one push call later."""
    from easywakeword_amd import StreamEngine
    parts = [synth.make_stream(seed, n_words=4)[0] for seed in (31, 32, 33, 34)]
    n = min(len(p) for p in parts) // 1600 * 1600
    pcm = np.stack([p[:n] for p in parts]).astype(np.float32)
    word = synth.load_word()
    a, b = StreamEngine(4), StreamEngine(4)
    for e in (a, b):
        e.template_from_pcm(word)
    blocking, lagged = [], []
    for t0 in range(0, n // 1600, 4):
        blk = pcm[:, t0 * 1600:(t0 + 4) * 1600]
        if blk.shape[1] < 4 * 1600:
            break
        a.push_many(blk)
        blocking.append(a.poll())
        b.push_many(blk)
        lagged.append(b.poll(lagged=True))
    lagged.append(b.poll())          # drain the last call
    assert len(lagged[0]) == 0
    for k, ev in enumerate(blocking):
        np.testing.assert_array_equal(lagged[k + 1], ev)
    assert sum(len(e) for e in blocking) >= 8


def test_long_segments_cooperative_scorer(template):
    """Segments of 8 s and 26 s through the ring-mode scorer: a workgroup's waves
    share each segment (7 and 21 tiles per wave: each wave's last tile waits in LDS
    for the segment max, earlier ones are clamped speculatively and recomputed when
    top_db bites), scores vs the oracle."""
    gate = dict(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=40.0,
                post_speech_silence=0.4, buffer_seconds=60)
    sr = 16000
    streams = []
    for i, dur in enumerate((26.0, 8.0)):
        rng = np.random.default_rng(70 + i)
        n = int(90.0 * sr)   # the gate starts once the 60 s ring is full
        x = (rng.standard_normal(n) * 1e-4).astype(np.float64)
        a, b = int(61.5 * sr), int((61.5 + dur) * sr)
        t = np.arange(b - a) / sr
        x[a:b] += 0.3 * np.sin(2 * np.pi * (440.0 + 60 * i) * t) * (1.0 + 0.3 * np.sin(2 * np.pi * 0.7 * t))
        streams.append(x.astype(np.float32))
    L = min(len(s) for s in streams)
    L -= L % 1600
    data = np.stack([s[:L] for s in streams])
    eng = _engine(2, gate, max_segment_seconds=40.0)
    eng.set_template(*template)
    got = []
    step = 16 * 1600
    for c in range(0, L, step):
        eng.push_many(data[:, c:c + step])
        got.extend(eng.poll().tolist())
    tm, ts = template
    cfg = GateConfig(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=40.0,
                     post_speech_silence=0.4, buffer_seconds=60, max_segment_seconds=40.0)
    n_long = 0
    for i in range(2):
        ref = run_stream(data[i], cfg).events
        mine = sorted([g for g in got if g[0] == i], key=lambda g: g[2])
        assert [(g[2], g[1], bool(g[7] & 1)) for g in mine] == [(e.tick, e.length, e.skipped) for e in ref], i
        for g, e in zip(mine, ref):
            if e.skipped:
                continue
            cm, cs = mfcc_ref.extract_mfcc(e.audio)
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            assert score_close(g[5], s, 1e-4), (i, g[1], g[5], s)
            n_long += e.length > 7 * sr
    assert n_long == 2


def test_corrupt_stream_does_not_disturb_the_others(template):
    """NaN / Inf samples in one stream (a broken capture) must not change any other
    stream's events: streams are independent in the gate, the scorer and the queue."""
    gate = dict(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0, post_speech_silence=0.4)
    parts = [synth.make_stream(seed, n_words=4)[0] for seed in (61, 62, 63)]
    L = min(len(p) for p in parts) // 1600 * 1600
    data = np.stack([p[:L] for p in parts]).astype(np.float32)
    bad = data.copy()
    bad[1, 20 * 16000:20 * 16000 + 4800] = np.nan
    bad[1, 30 * 16000:30 * 16000 + 100] = np.inf
    got = {}
    for name, d in (("clean", data), ("bad", bad)):
        eng = _engine(3, gate)
        eng.set_template(*template)
        ev = []
        for c in range(0, L, 8 * 1600):
            eng.push_many(d[:, c:c + 8 * 1600])
            ev.extend(eng.poll().tolist())
        eng.close()
        got[name] = ev
    for s in (0, 2):
        a = np.array([x[1:3] + x[5:8] for x in got["clean"] if x[0] == s], dtype=np.float64)
        b = np.array([x[1:3] + x[5:8] for x in got["bad"] if x[0] == s], dtype=np.float64)
        assert len(a) > 0
        np.testing.assert_array_equal(a, b)   # (length, tick, score, match, flags); NaN == NaN
