"""Find the smallest batch whose per-segment results differ from the same segments scored alone."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402
import easywakeword_amd as ewa  # noqa: E402

eng = ewa.Engine()
eng.template_from_pcm(synth.load_word())
segs = synth.ragged_segments(4321, 600, 160, 48000)
alone = np.stack([eng.score([x], candidate_dtype="float64")[0][0] for x in segs[:64]])
for n in (2, 4, 8, 16, 64):
    m = eng.score(segs[:n], candidate_dtype="float64")[0]
    d = np.any(m != alone[:n], axis=1)
    print(f"batch {n:3d}: {d.sum()} differ from alone; max {np.abs(m - alone[:n]).max():.3e}; idx {np.nonzero(d)[0][:10]}")
# 600 segments: compare the first 64 with alone
m = eng.score(segs, candidate_dtype="float64")[0][:64]
d = np.any(m != alone, axis=1)
print(f"batch 600: first 64: {d.sum()} differ")
# the same segment repeated 2048 times
x = segs[5]
m = eng.score([x] * 2048, candidate_dtype="float64")[0]
u = np.unique(m, axis=0)
print(f"segment 5 x 2048: {len(u)} distinct mean vectors; alone equal to row 0: {np.array_equal(m[0], alone[5])}")
# zeros then the segment: does a preceding segment matter?
for pre_len in (200, 16000, 47000):
    pre = np.random.default_rng(1).standard_normal(pre_len).astype(np.float32)
    mm = eng.score([pre] * 2048 + [x] * 2048, candidate_dtype="float64")[0][2048:]
    print(f"after {pre_len}-sample segments: {len(np.unique(mm, axis=0))} distinct, max err {np.abs(mm - alone[5]).max():.3e}")
