"""Score one batch three times through the product scorer and count bitwise differences
(a race in the staging / DMA shows as launch-to-launch differences), then compare a sample
with the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402
from oracle import mfcc_ref  # noqa: E402
import easywakeword_amd as ewa  # noqa: E402

eng = ewa.Engine()
word = synth.load_word()
eng.template_from_pcm(word)
tm, ts = eng.get_template()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
segs = synth.ragged_segments(4321, n, 160, 48000)
lens = np.array([len(x) for x in segs])
outs = [eng.score(segs, candidate_dtype="float64") for _ in range(3)]
for k in range(1, 3):
    dm = np.any(outs[k][0] != outs[0][0], axis=1)
    d_sc = np.sum(~((outs[k][2] == outs[0][2]) | (np.isnan(outs[k][2]) & np.isnan(outs[0][2]))))
    mag = np.abs(outs[k][0] - outs[0][0]).max(axis=1)
    print(f"launch {k} vs 0: {dm.sum()} segments with different mean bits, {d_sc} different scores; "
          f"max |dmean| {mag.max():.3e}; differing lengths: min {lens[dm].min() if dm.any() else 0} "
          f"median {np.median(lens[dm]) if dm.any() else 0}; T<=16 differing {np.sum(dm & (lens < 2560))}")
    tiles = 1 + (1 + lens // 160 - 1) // 16
    for t in range(1, 20):
        sel = tiles == t
        if sel.any():
            print(f"   tiles {t:2d}: {sel.sum():4d} segments, {np.sum(dm & sel):4d} differ")
# single segment, alone, 4 times
x = segs[int(np.argmax(lens))]
r = [eng.score([x], candidate_dtype="float64")[0][0] for _ in range(4)]
print("single longest segment repeated: identical" if all(np.array_equal(r[0], q) for q in r) else
      f"single segment differs: {[np.abs(q - r[0]).max() for q in r]}")
cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64))
print("single vs oracle |mean err|", np.abs(r[0] - cm).max())
bad = 0
worst = 0.0
for i in range(0, n, max(1, n // 100)):
    x = segs[i]
    cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64))
    ref = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
    s = outs[0][2][i]
    if not (np.isnan(ref) and np.isnan(s)):
        e = abs(s - ref)
        worst = max(worst, e)
        if e > 1e-4:
            bad += 1
            if bad < 6:
                mm = np.abs(outs[0][0][i] - cm).max()
                print(f"seg {i} len {len(x)}: score {s:.6f} ref {ref:.6f}  |mean err| {mm:.3e}")
print(f"oracle sample: {bad} beyond 1e-4, worst {worst:.3e}")
