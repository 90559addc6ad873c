"""The vanishing-mean evidence fixture (tests/golden/mean_band_cases.json) regenerates: its
segments come back from tests/synth.py with the oracle |mean| and score the fixture records."""
import json
import os

import numpy as np

import synth
from oracle import mfcc_ref


def test_mean_band_fixture_regenerates():
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mean_band_cases.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) >= 500 and len(set(c["kind"] for c in cases)) >= 3
    tm, ts = (x.astype(np.float32) for x in mfcc_ref.extract_mfcc(synth.load_word()))
    for c in cases[::75]:
        x = synth.mean_band_segment(c["kind"], c["seed"], c["gain"], c["length"])
        cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64))
        assert float(np.linalg.norm(cm)) == c["mean_norm"]
        assert float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs)) == c["score"]
        assert 32.0 <= c["mean_norm"] < 64.0
