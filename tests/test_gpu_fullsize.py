"""Parity at BASELINE.json's full sizes (the bench workloads): EVERY segment and event
checked against the oracle, plus size-independent properties.

* configs[1]: the bench's 65,536-segment ragged batch (bench.make_segments), scored in one
  launch: all 65,536 scores within 1e-4 of the oracle (oracle/mfcc_ref.py, float64
  candidates, over a process pool: tests/oracle_pool.py) with identical decisions; no NaN on
  audible segments; a sample re-scored as its own small batch gives bit-identical outputs
  (a segment's result does not depend on the batch around it or the work order).
* configs[2]: 8,192 streams of the bench's streaming recipe (bench.make_streams) through the
  full engine for 70 s of audio (10 s prefill + 60 s): for 64 streams the event list (tick,
  length, skip flag) equals the oracle gate (oracle/gate_ref.py) exactly; EVERY scored event
  of all 8,192 streams is re-cut from the stream audio and its score checked against the
  oracle within 1e-4 with an identical decision.
"""
import numpy as np
import pytest

from golden_io import score_close
from oracle_pool import oracle_gate_events, oracle_scores
from oracle import mfcc_ref
from oracle.gate_ref import GateConfig, run_stream
from easywakeword_amd._lib import RESCORE_TINY_MEAN

pytestmark = pytest.mark.gpu

SCORE_TOL = 1e-4


@pytest.fixture(scope="module")
def env():
    import torch
    import bench
    import easywakeword_amd as ewa
    dev = torch.device("cuda", 0)
    word = bench.load_word()
    return torch, bench, ewa, dev, word


def test_config2_bench_batch_full_size(env):
    torch, bench, ewa, dev, word = env
    n = 65536
    pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, dev, n, 1234, word)
    eng = ewa.Engine()
    eng.template_from_pcm(word)
    tm, ts = eng.get_template()
    mean = torch.empty((n, 20), device=dev)
    std = torch.empty((n, 20), device=dev)
    score = torch.empty(n, device=dev, dtype=torch.float64)
    match = torch.empty(n, device=dev, dtype=torch.uint8)
    s = torch.cuda.current_stream(dev)
    eng.score_device(pcm.data_ptr(), off.data_ptr(), ln.data_ptr(), n, mean.data_ptr(), std.data_ptr(),
                     score.data_ptr(), match.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    sc, mt = score.cpu().numpy(), match.cpu().numpy().astype(bool)
    assert frames == int((1 + lengths.astype(np.int64) // 160).sum())
    assert not np.isnan(sc).any()                       # every segment is audible
    assert 0.5 < mt.mean() < 1.0                        # both decisions occur (distractors score ~70)

    # every segment against the oracle
    host = pcm.cpu().numpy()
    o0 = int(offsets[0])
    allsegs = [host[int(offsets[i]) - o0:int(offsets[i]) - o0 + int(lengths[i])] for i in range(n)]
    ref = oracle_scores(allsegs, tm, ts)
    del allsegs
    d = np.abs(sc - ref)
    assert np.array_equal(np.isnan(sc), np.isnan(ref))
    worst = int(np.nanargmax(d))
    assert np.nanmax(d) <= SCORE_TOL, (worst, int(lengths[worst]), sc[worst], ref[worst])
    np.testing.assert_array_equal(mt, ref >= 75.0)

    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([rng.choice(n, 40, replace=False),
                                    [int(np.argmax(lengths)), int(np.argmin(lengths)), 0, n - 1]]))
    segs = [host[int(offsets[i]) - o0:int(offsets[i]) - o0 + int(lengths[i])].copy() for i in idx]
    del host
    m2, s2, sc2, mt2 = eng.score(segs, candidate_dtype="float64")
    np.testing.assert_array_equal(sc2, sc[idx])
    np.testing.assert_array_equal(m2, mean.cpu().numpy()[idx])
    np.testing.assert_array_equal(s2, std.cpu().numpy()[idx])
    np.testing.assert_array_equal(mt2.astype(bool), mt[idx])
    eng.close()


def test_config3_streams_full_size_sampled_vs_oracle(env):
    torch, bench, ewa, dev, word = env
    n_streams, ticks = 8192, 700
    period, pcm = bench.make_streams(torch, dev, n_streams, 1234, word)
    se = ewa.StreamEngine(n_streams)
    se.template_from_pcm(word)
    tm, ts = se.get_template()
    got = []
    t = 0
    while t < ticks:                                   # 32 ticks per call, wrapping at the 16 s loop
        k = t % period
        nt = min(32, ticks - t, period - k)
        se.push_device(pcm.data_ptr() + k * 1600 * 4, period * 1600, 1600, nt)
        got.append(se.poll())
        t += nt
    got.append(se.poll())
    ev = np.concatenate(got)
    assert len(ev) > 8 * n_streams                      # ~ 5 events per 16 s per stream after the prefill

    # the gate: 64 streams (the grid's corners and a spread) replayed through the oracle
    sample = sorted(set([0, 1, 2, 777, 4095, 4096, 8190, 8191] +
                        list(np.random.default_rng(11).choice(n_streams, 56, replace=False))))
    host = pcm.cpu().numpy()
    ref_ev = oracle_gate_events([host[s] for s in sample], ticks, tm, ts)
    reps = -(-ticks // period)
    n_checked = 0
    for sid, ref in zip(sample, ref_ev):
        mine = ev[ev["stream"] == sid]
        mine = mine[np.argsort(mine["tick"], kind="stable")]
        assert [(int(m["tick"]), int(m["length"]), bool(m["flags"] & 1)) for m in mine] == \
               [(e[0], e[1], e[2]) for e in ref], sid
        for m, e in zip(mine, ref):
            if e[2]:
                continue
            assert score_close(float(m["score"]), e[3], SCORE_TOL), (sid, int(m["tick"]), float(m["score"]), e[3])
            assert bool(m["match"]) == (e[3] >= 75.0)
            n_checked += 1
    assert n_checked >= 800                             # ~ 17 level-2 calls per stream

    # Every part of the grid: 4,096 events drawn over all streams and ticks (pushes of 32
    # ticks score a few thousand segments per launch: teams of 2 waves in rounds, 4 or 8 on
    # lighter launches) re-scored by the linear batch scorer from the stream audio.  The
    # segment is the `length` samples from tick * 1600 - n_request, where n_request =
    # (tick * 1600 - ring_start) mod ring (checked against the oracle's cut on the samples).
    ring = 160000
    lp = period * 1600

    def cut(row, m):
        n_req = (int(m["tick"]) * 1600 - int(m["ring_start"])) % ring
        s0 = int(m["tick"]) * 1600 - n_req
        return row[np.arange(s0, s0 + int(m["length"])) % lp]

    for sid in sample[:8]:
        row = host[sid]
        mine = ev[(ev["stream"] == sid) & ((ev["flags"] & 1) == 0)]
        ref = [e for e in run_stream(np.tile(row, reps)[: ticks * 1600], GateConfig()).events if not e.skipped]
        for m, e in zip(mine[np.argsort(mine["tick"], kind="stable")], ref):
            np.testing.assert_array_equal(cut(row, m), e.audio.astype(np.float32))
    # EVERY scored event of the 8,192 streams against the oracle: the audio repeats every
    # `period` ticks, so events with equal (stream, tick mod period, request, length) hold the
    # same samples -- each distinct segment is scored once by the oracle
    scored = ev[(ev["flags"] & 1) == 0]
    n_req = (scored["tick"].astype(np.int64) * 1600 - scored["ring_start"].astype(np.int64)) % ring
    key = np.stack([scored["stream"].astype(np.int64), scored["tick"].astype(np.int64) % period, n_req,
                    scored["length"].astype(np.int64)], axis=1)
    uniq, inv = np.unique(key, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    first = np.zeros(len(uniq), np.int64)
    first[inv[::-1]] = np.arange(len(scored))[::-1]
    ref_all = oracle_scores([cut(host[int(scored[i]["stream"])], scored[i]) for i in first], tm, ts)[inv]
    d = np.abs(scored["score"] - ref_all)
    assert np.array_equal(np.isnan(scored["score"]), np.isnan(ref_all))
    assert np.nanmax(d) <= SCORE_TOL, (float(np.nanmax(d)), scored[int(np.nanargmax(d))])
    np.testing.assert_array_equal(scored["match"].astype(bool), ref_all >= 75.0)
    assert len(uniq) > 20000 and len(scored) > 8 * n_streams
    del host

    scored = ev[(ev["flags"] & 1) == 0]
    pick = np.random.Generator(np.random.PCG64(7)).choice(len(scored), size=min(4096, len(scored)), replace=False)
    pick = scored[np.sort(pick)]
    rows = pcm[torch.from_numpy(pick["stream"].astype(np.int64)).to(pcm.device)].cpu().numpy()
    segs = [cut(r, m) for r, m in zip(rows, pick)]
    eng = ewa.Engine()
    eng.template_from_pcm(word)
    bm, _, sc, mt = eng.score(segs, candidate_dtype="float64")
    d = np.abs(sc - pick["score"])
    fin = np.isfinite(sc)
    assert np.array_equal(fin, np.isfinite(pick["score"]))
    # both paths send the same segments (near the threshold, short, stationary, or with a
    # vanishing MFCC mean vector) to the same fp64 re-score: the ring scores and the batch
    # scores of the same segments agree within the 1e-4 bar
    # (a margin for the two paths' float32 means; a NaN score beyond the float32 error is not listed)
    small = (np.linalg.norm(bm, axis=1) < RESCORE_TINY_MEAN - 0.5) & np.isfinite(pick["score"])
    assert small.sum() >= 20, int(small.sum())          # the recipe's loud events are covered
    np.testing.assert_array_equal(pick["flags"][small] & 2, 2)
    bad = fin & (d > SCORE_TOL)
    assert not bad.any(), (float(d[fin].max()), pick[bad][:3])
    np.testing.assert_array_equal(mt.astype(bool), pick["match"].astype(bool))
    eng.close()
    se.close()
