"""Pick the vanishing-mean evidence set (test infra).

    python tests/golden/make_mean_band.py

The fp64 re-score takes segments whose float32 MFCC mean vector has |mean| < kTinyMean
(csrc/ewk_mfcc.hip); round 5 lowered that from 64 to 32 on one recipe's data.  This script
draws segments of four recipes other than the streaming bench's (tests/synth.py
mean_band_segment: loud white noise, pink noise, a tone plus noise, the word in loud noise),
keeps those whose ORACLE MFCC mean has |mean| in [32, 64) and a finite score, 150 per recipe,
and writes their parameters with the oracle's |mean| and score to mean_band_cases.json.
tests/test_gpu_vanishing_mean.py regenerates the segments from the parameters and checks the
GPU's float32 scores against these oracle scores.
"""
from __future__ import annotations

import json
import os
import sys

os.environ.setdefault("OMP_NUM_THREADS", "1")

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import synth  # noqa: E402
from oracle import mfcc_ref  # noqa: E402

# gain ranges (log-uniform) where each recipe's |mean| crosses [32, 64) (scanned at L = 16,000)
RANGES = {"white": (0.22, 0.40), "pink": (0.3, 1.1), "tone_noise": (0.7, 1.5), "word_noise": (0.22, 0.36)}
PER_KIND = 150


def main():
    word = synth.load_word()
    tm, ts = (x.astype(np.float32) for x in mfcc_ref.extract_mfcc(word))
    rng = np.random.Generator(np.random.PCG64(20261018))
    cases = []
    for kind, (lo, hi) in RANGES.items():
        got = tried = 0
        while got < PER_KIND:
            tried += 1
            if tried > 40 * PER_KIND:
                raise SystemExit(f"{kind}: only {got} of {tried} draws in the band")
            seed = int(rng.integers(0, 2**31))
            gain = float(np.exp(rng.uniform(np.log(lo), np.log(hi))))
            length = int(rng.integers(6400, 33601))
            x = synth.mean_band_segment(kind, seed, gain, length)
            cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64))
            mn = float(np.linalg.norm(cm))
            s = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
            if 32.0 <= mn < 64.0 and np.isfinite(s):
                cases.append({"kind": kind, "seed": seed, "gain": gain, "length": length, "mean_norm": mn,
                              "std_norm": float(np.linalg.norm(cs)), "score": s})
                got += 1
        print(f"{kind}: {got} of {tried} draws in the band")
    with open(os.path.join(HERE, "mean_band_cases.json"), "w") as f:
        json.dump({"template": "reference_word.wav (oracle/mfcc_ref.py)", "band": [32.0, 64.0],
                   "generator": "tests/synth.py mean_band_segment", "cases": cases}, f, indent=0)


if __name__ == "__main__":
    main()
