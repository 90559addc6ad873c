"""The fp64 re-score's FFT buffer swizzle (ewk_rescore.h rs_swz): a permutation of the 256
slots that makes every radix-4 Stockham store and natural-order read of a 16-lane group hit 16
distinct 16-B bank groups (scripts/f64_chunk_model.py swizzle_conflicts)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import f64_chunk_model as m  # noqa: E402


def test_swizzle_is_conflict_free():
    r = m.swizzle_conflicts()
    assert r["plain"]["stores"] == 4            # the unswizzled Ns = 1 / 4 stores
    assert r["swizzled"]["stores"] == 1
    assert r["swizzled"]["reads"] == 1
    assert r["swizzled"]["untangle_reads"] <= 2


def test_swizzle_matches_header():
    src = open(os.path.join(ROOT, "easywakeword_amd", "csrc", "ewk_rescore.h")).read()
    assert "return i ^ (((i >> 4) * 5) & 15);" in src
