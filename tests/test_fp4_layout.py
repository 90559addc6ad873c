"""CPU checks of the four-lanes-per-frame pass's index algebra (scripts/experiments/fp4/ewk_fp4.h).

scripts/fp4_model.py replays, in float64, what the four lanes of a frame hold at every step
(row transposition, untangle pairs, mel incidences, reduce-scatter) -- these tests pin it:
the power spectrum and the mel band energies through the lane algorithm equal numpy's, and the
generated incidence header the kernel unrolls is the one the model emits.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, ROOT)

import fp4_model  # noqa: E402
from oracle import mfcc_ref  # noqa: E402


def test_layout_closed_and_covering():
    fp4_model.check_layout()


def test_lane_algorithm_power_and_mel():
    W = mfcc_ref.mel_filterbank().astype(np.float64)
    win = mfcc_ref.hann_window()
    rng = np.random.default_rng(3)
    inc = fp4_model.mel_incidence(W)
    for _ in range(3):
        x = rng.standard_normal(512)
        P = fp4_model.stft_frame(x, win)
        ref = np.abs(np.fft.rfft(x * win)) ** 2
        assert max(abs(P[k] - ref[k]) for k in P) <= 1e-9 * ref.max()
        E = np.zeros(128)
        for g in range(4):
            for m in range(128):
                for (q, kp) in inc[m]:
                    b = fp4_model.bin_of(g, q, kp)
                    E[m] += W[m, b] * P.get(b, 0.0)
        np.testing.assert_allclose(E, W @ ref, rtol=1e-9, atol=1e-12 * ref.max())


def test_generated_header_is_current(tmp_path):
    out = tmp_path / "ewk_fp4_mel.h"
    fp4_model.emit_header(str(out))
    cur = open(os.path.join(ROOT, "scripts", "experiments", "fp4", "ewk_fp4_mel.h")).read()
    assert out.read_text() == cur
