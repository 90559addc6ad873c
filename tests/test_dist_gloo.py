"""N>1 layout of the hot path on CPU: world_size-2 gloo, the same sharding and
decision gather bench.py runs over RCCL (easywakeword_amd/shard.py).

The per-rank scorer here is the oracle (CPU, test-only): the point is that the
stream partition and the all-gather reproduce, on every rank, exactly the
decisions a single process computes over all streams.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from easywakeword_amd.shard import DecisionGather, gather_positives, positives, shard_streams

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


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # equal shards so the fixed-shape all_gather applies (the bench's per-rank shape)
        first, count = shard_streams(N_STREAMS + 1, rank, world)
        sc, mt = _score_streams(range(first, first + count))
        score, match = torch.from_numpy(sc), torch.from_numpy(mt)
        g = DecisionGather(score, match)
        parts_s, parts_m = g(score, match)
        firsts = [shard_streams(N_STREAMS + 1, r, world)[0] for r in range(world)]
        pos = positives(parts_s, parts_m, firsts, SEG_PER_STREAM)
        all_s, all_m = g.concatenated()
        q.put((rank, all_s.numpy(), all_m.numpy(), pos))
    finally:
        dist.destroy_process_group()


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


def test_gloo_world2_gather_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_s, ref_m = _score_streams(range(N_STREAMS + 1))
    assert ref_m.any() and not ref_m.all()     # both decisions occur
    for rank, s, m, pos in sorted(results, key=lambda r: r[0]):
        np.testing.assert_array_equal(s, ref_s)   # same oracle, same inputs: bit-identical
        np.testing.assert_array_equal(m, ref_m)
        want = [(i // SEG_PER_STREAM, i % SEG_PER_STREAM) for i in np.nonzero(ref_m)[0]]
        assert [(a, b) for a, b, _ in pos] == want


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
