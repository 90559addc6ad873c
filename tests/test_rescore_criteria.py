"""The fp64 re-score's vanishing-mean criterion is stated twice: kTinyMean in the scorer
(csrc/ewk_mfcc.hip) and RESCORE_TINY_MEAN in easywakeword_amd/_lib.py, which the GPU tests use
to pick the events that must carry EWK_EV_RESCORED.  They must agree."""
import os
import re

from easywakeword_amd._lib import NAN_MARGIN_A, NAN_MARGIN_B, RESCORE_TINY_MEAN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tiny_mean_matches_the_scorer():
    src = open(os.path.join(ROOT, "easywakeword_amd", "csrc", "ewk_mfcc.hip")).read()
    m = re.search(r"#define EWK_TINY_MEAN ([0-9.]+)", src)
    assert m is not None
    assert float(m.group(1)) == RESCORE_TINY_MEAN


def test_nan_margin_matches_the_scorer():
    src = open(os.path.join(ROOT, "easywakeword_amd", "csrc", "ewk_mfcc.hip")).read()
    a = re.search(r"#define EWK_NAN_MARGIN_A ([0-9.]+)", src)
    b = re.search(r"constexpr double kNanMarginB = ([0-9.]+);", src)
    assert a is not None and b is not None
    assert float(a.group(1)) == NAN_MARGIN_A and float(b.group(1)) == NAN_MARGIN_B
