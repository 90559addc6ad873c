"""Precision of the fp32 scorer against the device fp64 path (itself within 1e-9 of the
oracle, tests/test_gpu_scorer.py) on the bench's ragged batch: |score32 - score64| over
segments the fp32 score decides alone (outside rescore_margin, > 16 frames), and the
MFCC mean/std deviations.  Usage: python scripts/score_err.py [n_segments]  (EWK_LIB
selects a libewk.so variant)."""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import easywakeword_amd as ewa
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda", 0)
word = bench.load_word()
pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, dev, n, 1234, word)
host = pcm.cpu().numpy()
e = ewa.Engine()
e.template_from_pcm(word)
m32, s32, sc32, _ = e.score_packed(host, offsets, lengths, True, False)
m64, s64, sc64 = e.score_f64([host[o:o + l] for o, l in zip(offsets, lengths)])
T = 1 + lengths // 160
solo = (np.abs(sc32 - 75.0) > 1e-3) & (T > 16) & np.isfinite(sc64)
d = np.abs(sc32 - sc64)[solo]
dm = np.abs(m32 - m64)[solo] / np.maximum(1.0, np.abs(m64[solo]))
ds = np.abs(s32 - s64)[solo] / np.maximum(1.0, np.abs(s64[solo]))
lib = os.path.basename(os.environ.get("EWK_LIB", "libewk.so"))
print(f"{lib}: {int(solo.sum())} of {n} segments decided by the fp32 score: |dscore| max {d.max():.3e} "
      f"p99.9 {np.quantile(d, 0.999):.3e} median {np.median(d):.3e}; mean rel/abs max {dm.max():.3e}, "
      f"std rel/abs max {ds.max():.3e}; decisions differ {int(np.sum((sc32 >= 75.0) != (sc64 >= 75.0)))}")
