"""N>1 layout of the hot path on CPU: world_size 2 and 3 over gloo, the same sharding
and positives gathers bench.py runs over RCCL (easywakeword_amd/shard.py).

The per-rank scorer / gate here is the oracle (CPU, test-only): the point is that
the stream partition plus the gathers reproduce on rank 0 exactly the positives a
single process finds over all streams -- batch decisions (MatchGather: device-side
compaction, counts all_gather, point-to-point records) and the streaming level-3 feed
(PositiveCollector: per-tick positives batched every K ticks, with the normalised PCM).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from easywakeword_amd.shard import MatchGather, PositiveCollector, gather_positives, shard_streams

N_STREAMS = 5
SEG_PER_STREAM = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _segments(stream: int):
    """SEG_PER_STREAM short segments per stream: the word (match) or noise (no match)."""
    from tests.synth import load_word
    word = load_word()
    rng = np.random.default_rng(100 + stream)
    out = []
    for k in range(SEG_PER_STREAM):
        noise = rng.normal(0, 2e-3, 8000).astype(np.float32)
        if (stream + k) % 2 == 0:
            seg = noise.copy()
            seg[: min(len(word), 8000)] += word[:8000]
        else:   # differenced (high-passed) noise: scores ~70, below the default 75
            w = rng.normal(0, 1.0, 8001).astype(np.float32)
            seg = (w[1:] - w[:-1]) * np.float32(0.1)
        out.append(seg.astype(np.float64))
    return out


def _score_streams(streams):
    from oracle.mfcc_ref import WordMatcherRef
    from tests.synth import load_word
    m = WordMatcherRef()
    m.set_reference(load_word())
    sc, mt = [], []
    for s in streams:
        for seg in _segments(s):
            ok, v = m.matches(seg)
            sc.append(v)
            mt.append(1 if ok else 0)
    return np.array(sc, np.float64), np.array(mt, np.uint8)


def _run_world(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, payload = q.get(timeout=300)
        results[r] = payload
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return results


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker_match(rank, world, port, q):
    _init(rank, world, port)
    try:
        first, count = shard_streams(N_STREAMS, rank, world)     # uneven shards
        sc, mt = _score_streams(range(first, first + count))
        g = MatchGather(len(sc), first * SEG_PER_STREAM, torch.device("cpu"))
        rec = g(torch.from_numpy(sc), torch.from_numpy(mt))
        q.put((rank, None if rec is None else rec.numpy()))
    finally:
        dist.destroy_process_group()


def _worker_match_ksteps(rank, world, port, q):
    """K = 3 steps: per-step gathers vs one batched flush of three device-side adds."""
    _init(rank, world, port)
    try:
        first, count = shard_streams(N_STREAMS, rank, world)
        sc, mt = _score_streams(range(first, first + count))
        steps = [(torch.from_numpy(sc + k), torch.from_numpy(np.roll(mt, k))) for k in range(3)]
        g1 = MatchGather(len(sc), first * SEG_PER_STREAM, torch.device("cpu"))
        per_step = [g1(s, m) for s, m in steps]
        g3 = MatchGather(len(sc), first * SEG_PER_STREAM, torch.device("cpu"), steps=3)
        for s, m in steps:
            g3.add(s, m)
        with pytest.raises(RuntimeError):
            g3.add(*steps[0])
        batched = g3.flush()
        again = [g1(s, m) for s, m in steps[:1]]   # the buffer re-arms after a flush
        q.put((rank, None if batched is None else (batched.numpy(), [p.numpy() for p in per_step],
                                                    again[0].numpy())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_match_gather_k_steps_equals_per_step(world):
    """A K-step batched gather (records held on the device, one flush) delivers exactly
    the per-step gathers' records, each tagged with its step index."""
    res = _run_world(_worker_match_ksteps, world)
    batched, per_step, again = res[0]
    assert all(res[r] is None for r in range(1, world))
    want = []
    for k, rec in enumerate(per_step):
        r = rec.copy()
        r[:, 2] = k
        want.append(r)
    # per rank: steps in order; ranks concatenated -> compare as sorted record sets and per step
    got = sorted(map(tuple, batched.tolist()))
    assert got == sorted(map(tuple, np.concatenate(want).tolist()))
    assert len(batched) == sum(len(w) for w in want) > 0
    np.testing.assert_array_equal(again, per_step[0])


def test_shard_streams_partition():
    for n in (0, 1, 5, 1024, 8193):
        for world in (1, 2, 3, 8):
            spans = [shard_streams(n, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == n
            assert [s for s, _ in spans] == [sum(c for _, c in spans[:r]) for r in range(world)]
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard_streams(4, 2, 2)
    with pytest.raises(ValueError):
        shard_streams(-1, 0, 1)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_match_gather_equals_single_process(world):
    """Only the matched segments reach rank 0: (global segment id, score bits), in order."""
    res = _run_world(_worker_match, world)
    ref_s, ref_m = _score_streams(range(N_STREAMS))
    assert ref_m.any() and not ref_m.all()     # both decisions occur
    idx = np.nonzero(ref_m)[0]
    want = np.stack([idx.astype(np.int64), ref_s[idx].view(np.int64), np.zeros(len(idx), np.int64)], 1)
    np.testing.assert_array_equal(res[0], want)
    assert all(res[r] is None for r in range(1, world))


def _rank_positives(rank):
    """Rank-dependent positives: rank 0 has 2, rank 1 has 3, rank 2 none (ragged, incl. empty)."""
    n = [2, 3, 0][rank]
    g = torch.Generator().manual_seed(10 + rank)
    rec, audio = [], []
    for i in range(n):
        ln = 1000 + 137 * i + 50 * rank
        rec.append([rank * 100 + i, 7 + i, ln, i])
        audio.append(torch.randn(ln, generator=g))
    return torch.tensor(rec, dtype=torch.int64).reshape(n, 4), audio


def _worker_pos(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rec, audio = _rank_positives(rank)
        out_rec, out_audio = gather_positives(rec, audio)
        q.put((rank, None if out_rec is None else out_rec.numpy(),
               None if out_audio is None else [a.numpy() for a in out_audio]))
    finally:
        dist.destroy_process_group()


def test_gloo_world3_gather_positives_with_pcm():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pos, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {r: (rec, aud) for r, rec, aud in [q.get(timeout=300) for _ in range(world)]}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_rec = np.concatenate([_rank_positives(r)[0].numpy() for r in range(world)])
    want_aud = [a.numpy() for r in range(world) for a in _rank_positives(r)[1]]
    rec, aud = results[0]
    np.testing.assert_array_equal(rec, want_rec)
    assert len(aud) == len(want_aud) == 5
    for a, b in zip(aud, want_aud):
        np.testing.assert_array_equal(a, b)
    assert results[1] == (None, None) and results[2] == (None, None)


# ---------------------------------------------------------------- streaming level-3 feed
STREAMS_S = 5
EVERY = 10


def _stream_audio():
    import synth
    pcms = [synth.make_stream(seed=6100 + s, n_words=5, sigma=1e-3, gain=[1.0, 3.0, 0.6, 2.0, 1.2][s],
                              kinds=[["word", "hp"], ["hp", "word", "white"], ["word"], ["word", "hp_near"],
                                     ["word", "hp"]][s])[0] for s in range(STREAMS_S)]
    L = min(len(p) for p in pcms) // 1600 * 1600
    return np.stack([p[:L] for p in pcms])


def _oracle_shard(streams, audio, on_tick):
    """Oracle level 1 + 2 over `streams`, tick by tick; on_tick(events, audio_by_key) per tick."""
    from easywakeword_amd._lib import EVENT_DTYPE
    from oracle import mfcc_ref
    from oracle.gate_ref import DetectorRef, GateConfig
    import synth
    tm, ts = mfcc_ref.extract_mfcc(synth.load_word())
    dets = [DetectorRef(GateConfig()) for _ in streams]
    for t in range(audio.shape[1] // 1600):
        rows, seg = [], {}
        for j, (s, det) in enumerate(zip(streams, dets)):
            ev = det.push_tick(audio[s, t * 1600:(t + 1) * 1600])
            if ev is None:
                continue
            score = np.nan
            if not ev.skipped:
                cm, cs = mfcc_ref.extract_mfcc(ev.audio)
                score = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            rows.append((j, ev.length, ev.tick, 0, ev.time, score, int(score >= 75.0), int(ev.skipped)))
            seg[(j, ev.tick)] = ev.audio
        on_tick(np.array(rows, dtype=EVENT_DTYPE), seg)


def _worker_stream(rank, world, port, q, audio_cap=10000):
    _init(rank, world, port)
    try:
        from oracle.gate_ref import normalize_level3
        audio = _stream_audio()
        first, count = shard_streams(STREAMS_S, rank, world)
        segs = {}

        def audio_fn(ev):
            # only the segments of the tick just polled are readable (a compact ring
            # overwrites older ones): the collector must capture PCM in add()
            return [torch.from_numpy(normalize_level3(segs[(int(e["stream"]), int(e["tick"]))])) for e in ev]

        col = PositiveCollector(first, torch.device("cpu"), every=EVERY, audio_cap=audio_cap, audio_fn=audio_fn)
        got_rec, got_aud = [], []

        def on_tick(ev, seg):
            segs.clear()
            segs.update(seg)
            col.add(ev)
            rec, aud = col.tick()
            if rec is not None:
                got_rec.append(rec.numpy())
                got_aud.extend(a.numpy() for a in aud)

        _oracle_shard(range(first, first + count), audio, on_tick)
        rec, aud = col.flush()
        if rec is not None:
            got_rec.append(rec.numpy())
            got_aud.extend(a.numpy() for a in aud)
        q.put((rank, (np.concatenate(got_rec), got_aud) if rank == 0 else (len(got_rec), len(got_aud))))
    finally:
        dist.destroy_process_group()


def _worker_stream_cap2(rank, world, port, q):
    _worker_stream(rank, world, port, q, audio_cap=1)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_streaming_positives_audio_cap(world):
    """audio_cap = 1 per rank and flush: every positive's record arrives, the PCM rides with
    the newest ones (captured at their poll) and matches each record it is paired with."""
    from oracle.gate_ref import normalize_level3
    res = _run_world(_worker_stream_cap2, world)
    rec, aud = res[0]
    audio = _stream_audio()
    want_aud = {}

    def on_tick(ev, seg):
        for e in ev[(ev["match"] != 0) & ((ev["flags"] & 1) == 0)]:
            key = (int(e["stream"]), int(e["tick"]))
            want_aud[key] = normalize_level3(seg[key])

    _oracle_shard(range(STREAMS_S), audio, on_tick)
    assert sorted((r[0], r[1]) for r in rec.tolist()) == sorted(want_aud)
    assert 0 < len(aud) <= len(rec)
    # gather_positives pairs rank r's PCM with its first records: find each audio's record
    # by length-order consistency -- every PCM equals the segment of some gathered record
    keys = [(r[0], r[1]) for r in rec.tolist()]
    for a in aud:
        assert any(len(a) == len(want_aud[k]) and np.array_equal(a, want_aud[k]) for k in keys)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_streaming_positives_reproduce_single_process(world):
    """Sharded streaming (oracle gate + scorer per rank), positives gathered every 10
    ticks with their level-3 PCM: rank 0 holds exactly the N=1 positives and audio."""
    from oracle.gate_ref import normalize_level3
    res = _run_world(_worker_stream, world)
    rec, aud = res[0]
    assert all(res[r] == (0, 0) for r in range(1, world))
    audio = _stream_audio()
    want, want_aud = [], {}

    def on_tick(ev, seg):
        for e in ev[(ev["match"] != 0) & ((ev["flags"] & 1) == 0)]:
            key = (int(e["stream"]), int(e["tick"]))
            want.append((key[0], key[1], int(e["length"]), int(np.float64(e["score"]).view(np.int64))))
            want_aud[key] = normalize_level3(seg[key])

    _oracle_shard(range(STREAMS_S), audio, on_tick)
    n_ev_all = len(want)
    assert n_ev_all >= 10
    got = sorted(map(tuple, rec.tolist()))
    assert got == sorted(want)
    assert len(aud) == len(rec)
    for r, a in zip(rec.tolist(), aud):
        np.testing.assert_array_equal(a, want_aud[(r[0], r[1])])
