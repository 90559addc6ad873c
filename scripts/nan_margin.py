"""How far can the float32 pass's similarity percent be from the float64 path's on loud segments
whose MFCC mean vector nearly vanishes (|mean| < 32, the fp64 re-score's vanishing-mean
criterion)?  Run on the GPU box:

    python scripts/nan_margin.py [n_per_recipe] > gpurun_out/nan_margin.txt

The reference scores p ** 1.5 / 10 with p = 100 (0.7 sm + 0.3 ss) (wakeword.py:611-625): any
p < 0 is NaN.  A segment whose float32 p is negative by more than the float32 pass's possible
error is NaN in the reference too, so its fp64 re-score cannot change its score or decision.
This script measures that error: ~n segments per recipe (the streaming bench's event sources
in a gated cut, loud white / pink noise, a tone plus noise, the word in loud noise, the top_db
fuzz recipe), float32 stats from the batch scorer (ewk_score_segments' mean / std outputs,
written by the float32 pass before any re-score) against the fp64 path's (ewk_score_segments_f64),
p computed from each with the reference's float64 arithmetic.  It prints, for |mean| < 32, the
worst |dp| and |dp| x |mean| by |mean| bucket, and how many segments the exemption rule
(ewk_mfcc.hip kNanMarginA / kNanMarginB: p32 < -(A / |mean| + B)) takes and whether any of
them has p64 >= 0.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import synth  # noqa: E402

A, B = 0.5, 0.05   # the rule under test (percent units)


def percent(tm, ts, m, s):
    """p = 100 (0.7 sm + 0.3 ss), scipy cosine arithmetic in float64, per row."""
    tm = tm.astype(np.float64)
    ts = ts.astype(np.float64)
    uu_m = float(np.float32(np.dot(tm, tm)))
    uu_s = float(np.float32(np.dot(ts, ts)))
    m = m.astype(np.float64)
    s = s.astype(np.float64)
    dm = np.clip(1.0 - (m @ tm) / np.sqrt(uu_m * np.einsum("ij,ij->i", m, m)), 0, 2)
    ds = np.clip(1.0 - (s @ ts) / np.sqrt(uu_s * np.einsum("ij,ij->i", s, s)), 0, 2)
    return ((1 - dm) * 0.7 + (1 - ds) * 0.3) * 100.0


def streaming_events(rng, n, word):
    import bench
    table = bench.event_sources(word, rng)
    out = []
    for _ in range(n):
        src = table[int(bench.event_kind(rng, 1)[0])] * np.float32(rng.uniform(0.3, 2.0))
        pre, post = int(rng.integers(800, 4000)), int(rng.integers(800, 4000))
        x = (rng.standard_normal(pre + len(src) + post) * rng.uniform(1e-4, 3e-3)).astype(np.float32)
        x[pre:pre + len(src)] += src
        out.append(x)
    return out


def main():
    from easywakeword_amd import Engine
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    word = synth.load_word()
    eng = Engine()
    eng.template_from_pcm(word)
    tm, ts = eng.get_template()
    rng = np.random.Generator(np.random.PCG64(606))
    recipes = {"streaming events": streaming_events(rng, n, word)}
    for kind, (lo, hi) in {"white": (0.15, 4.0), "pink": (0.2, 4.0), "tone_noise": (0.5, 4.0),
                           "word_noise": (0.2, 2.0)}.items():
        recipes[kind] = [synth.mean_band_segment(kind, int(rng.integers(0, 2**31)),
                                                 float(np.exp(rng.uniform(np.log(lo), np.log(hi)))),
                                                 int(rng.integers(6400, 33601))) for _ in range(n)]
    recipes["fuzz"] = synth.fuzz_segments(77, n, word)
    tot_exempt = tot_bad = 0
    allrows = []
    for name, segs in recipes.items():
        segs = [s for s in segs if len(s) >= 2560]   # T > 16 (shorter ones are listed for their length anyway)
        m32, s32, _, _ = eng.score(segs, candidate_dtype="float64")
        m64, s64, sc64 = eng.score_f64(segs)
        p32 = percent(tm, ts, m32, s32)
        p64 = percent(tm, ts, m64, s64)
        mn = np.linalg.norm(m64, axis=1)
        sn = np.linalg.norm(s64, axis=1)
        sel = (mn < 32.0) & (sn >= 20.0) & np.isfinite(p32) & np.isfinite(p64)
        dp = np.abs(p32 - p64)[sel]
        m32n = np.linalg.norm(m32, axis=1)[sel]
        exempt = p32[sel] < -(A / np.maximum(m32n, 1e-30) + B)
        bad = exempt & (p64[sel] >= 0)
        tot_exempt += int(exempt.sum())
        tot_bad += int(bad.sum())
        allrows.append(np.stack([mn[sel], dp, p32[sel], p64[sel], exempt], 1))
        print(f"{name:17s} segments {len(segs):6d}  |mean|<32 & |std|>=20: {int(sel.sum()):6d}  "
              f"max |dp| {dp.max() if dp.size else 0:.3e}  max |dp|*|mean| {(dp * mn[sel]).max() if dp.size else 0:.3e}  "
              f"p64<0: {int((p64[sel] < 0).sum())}  exempt: {int(exempt.sum())}  exempt with p64>=0: {int(bad.sum())}")
    rows = np.concatenate(allrows)
    print("\nby |mean| bucket (all recipes): n, max |dp|, max |dp| x |mean|, min (-(p32) - rule) margin over |dp|")
    for lo, hi in ((0, 0.5), (0.5, 1), (1, 2), (2, 4), (4, 8), (8, 16), (16, 32)):
        b = (rows[:, 0] >= lo) & (rows[:, 0] < hi)
        if not b.any():
            continue
        e = b & (rows[:, 4] > 0)
        ratio = ""
        if e.any():
            slack = -rows[e, 2] - 0.0   # how negative p32 is
            ratio = f"{np.min(slack / np.maximum(rows[e, 1], 1e-12)):.3g}"
        print(f"  [{lo:5.1f}, {hi:5.1f}) {int(b.sum()):6d}  {rows[b, 1].max():.3e}  {(rows[b, 1] * rows[b, 0]).max():.3e}  "
              f"exempt {int(e.sum())}  min |p32|/|dp| over exempt {ratio}")
    print(f"\nrule p32 < -({A} / |mean| + {B}): exempt {tot_exempt}, of which p64 >= 0: {tot_bad}")
    eng.close()


if __name__ == "__main__":
    main()
