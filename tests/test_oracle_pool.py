"""The oracle process pool (tests/oracle_pool.py) returns exactly the serial oracle's scores and
gate events, in the caller's order (the full-size GPU parity tests rely on it)."""
import numpy as np

import synth
from oracle import mfcc_ref
from oracle.gate_ref import GateConfig, run_stream
from oracle_pool import oracle_gate_events, oracle_scores


def test_pool_equals_serial_oracle():
    word = synth.load_word()
    tm, ts = (x.astype(np.float32) for x in mfcc_ref.extract_mfcc(word))
    segs = synth.ragged_segments(5, 24) + [np.zeros(6400, np.float32)]
    got = oracle_scores(segs, tm, ts, procs=2)
    ref = np.array([float(mfcc_ref.similarity_from_stats(tm, ts, *mfcc_ref.extract_mfcc(s.astype(np.float64))))
                    for s in segs])
    np.testing.assert_array_equal(got, ref)          # NaN == NaN (the silent segment)
    p, _ = synth.make_stream(3, n_words=3)
    row = p[:160 * 1600]
    ev = oracle_gate_events([row, row[::-1].copy()], 300, tm, ts, procs=2)
    for r, e in zip((row, row[::-1].copy()), ev):
        want = run_stream(np.tile(r, 2)[:300 * 1600], GateConfig()).events
        assert [(x[0], x[1], x[2]) for x in e] == [(w.tick, w.length, w.skipped) for w in want]
    assert len(ev[0]) >= 2
