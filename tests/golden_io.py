"""Loading helpers for the committed golden fixtures (tests/golden/*.json)."""
import hashlib
import json
import os

import numpy as np

import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(x) -> str:
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def matcher_fixture():
    with open(os.path.join(GOLD, "matcher_cases.json")) as f:
        fx = json.load(f)
    audio = dict(synth.matcher_cases())
    for c in fx["cases"]:
        assert sha(audio[c["name"]]) == c["sha256_f32"], f"regenerated input {c['name']} differs"
    return fx, audio


def template_arrays(fx):
    return (np.array(fx["template"]["mean"], np.float32), np.array(fx["template"]["std"], np.float32))


def gate_fixture():
    with open(os.path.join(GOLD, "gate_traces.json")) as f:
        return json.load(f)


def stream_pcm(rec):
    pcm, _ = synth.make_stream(**rec["stream"])
    assert sha(pcm) == rec["sha256_f32"], f"regenerated stream {rec['name']} differs"
    return pcm


def score_close(a, b, tol=1e-4):
    a = float("nan") if a is None else float(a)
    b = float("nan") if b is None else float(b)
    if np.isnan(a) or np.isnan(b):
        return np.isnan(a) and np.isnan(b)
    return abs(a - b) <= tol
