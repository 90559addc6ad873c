"""The CPU oracle over a process pool, for the full-size parity tests (test infrastructure).

VERDICT r5 next #2: check every segment of the full-size configurations against the oracle,
not a sample.  The oracle (oracle/mfcc_ref.py, float64 candidates) does ~3.3 M frames/s on a
GPU box's 16 cores with one BLAS thread per process (bench.py's cpu_baseline): the bench's
8.2 M-frame batch takes a few seconds.  Segments travel to the workers pickled, in balanced
chunks (longest first, round-robin); scores come back in the caller's order.
"""
import numpy as np


def _job(args):
    segs, tm, ts = args
    from oracle import mfcc_ref
    out = np.empty(len(segs), np.float64)
    for k, x in enumerate(segs):
        cm, cs = mfcc_ref.extract_mfcc(np.asarray(x, np.float64))
        out[k] = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
    return out


def _gate_job(args):
    rows, ticks, cfg_kw, tm, ts = args
    from oracle import mfcc_ref
    from oracle.gate_ref import GateConfig, run_stream
    res = []
    for row in rows:
        reps = -(-ticks * 1600 // len(row))
        audio = np.tile(row, reps)[: ticks * 1600]
        evs = []
        for e in run_stream(audio, GateConfig(**cfg_kw)).events:
            s = None
            if not e.skipped:
                cm, cs = mfcc_ref.extract_mfcc(e.audio)
                s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            evs.append((int(e.tick), int(e.length), bool(e.skipped), s))
        res.append(evs)
    return res


def n_procs() -> int:
    import bench
    return max(1, min(16, bench.host_cores()[0]))


def _pool(procs):
    import multiprocessing as mp
    import bench
    return bench._OneThreadEnv(), mp.get_context("spawn").Pool(procs, initializer=bench._pool_init)


def oracle_scores(segs, tm, ts, procs: int = 0) -> np.ndarray:
    """float64-candidate similarity of every segment (wakeword.py:544-567, 591-625)."""
    procs = procs or n_procs()
    n = len(segs)
    order = np.argsort([-len(s) for s in segs], kind="stable")
    n_chunks = min(n, procs * 4)
    chunks = [order[c::n_chunks] for c in range(n_chunks)]
    tm = np.asarray(tm, np.float32)
    ts = np.asarray(ts, np.float32)
    env, pool = _pool(procs)
    with env, pool:
        parts = pool.map(_job, [([segs[i] for i in ch], tm, ts) for ch in chunks], chunksize=1)
    out = np.empty(n, np.float64)
    for ch, p in zip(chunks, parts):
        out[ch] = p
    return out


def oracle_gate_events(rows, ticks, tm, ts, procs: int = 0, **cfg_kw):
    """Per row: the oracle gate's events over `ticks` ticks of the row repeated
    (oracle/gate_ref.py run_stream) with their oracle scores: [(tick, length, skipped, score)]."""
    procs = procs or n_procs()
    idx = list(range(len(rows)))
    chunks = [idx[c::procs] for c in range(min(procs, len(rows)))]
    env, pool = _pool(procs)
    with env, pool:
        parts = pool.map(_gate_job, [([rows[i] for i in ch], ticks, cfg_kw, np.asarray(tm, np.float32),
                                      np.asarray(ts, np.float32)) for ch in chunks], chunksize=1)
    out = [None] * len(rows)
    for ch, p in zip(chunks, parts):
        for i, evs in zip(ch, p):
            out[i] = evs
    return out
