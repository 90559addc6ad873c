"""fp32 score error against the device fp64 path by |mean| (the MFCC mean vector's norm) on
streaming events of the bench's recipe, for choosing kTinyMean (csrc/ewk_mfcc.hip): run with a
build that does not list vanishing-mean segments (-DEWK_TINY_MEAN=0) so the scores below the
current criterion are the float32 pipeline's own.

    EWK_LIB=variants/tiny0.so python scripts/mean_err.py [n_events] [ticks]
"""
import os
import sys

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import easywakeword_amd as ewa  # noqa: E402

n_pick = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 800
dev = torch.device("cuda", 0)
word = bench.load_word()
n_streams = 8192
period, spcm = bench.make_streams(torch, dev, n_streams, 1234, word)
se = ewa.StreamEngine(n_streams)
se.template_from_pcm(word)
evs, t = [], 0
while t < ticks:
    k = t % period
    nt = min(32, ticks - t, period - k)
    se.push_device(spcm.data_ptr() + k * 1600 * 4, period * 1600, 1600, nt)
    evs.append(se.poll())
    t += nt
ev = np.concatenate(evs)
ev = ev[(ev["flags"] & 1) == 0]
del se
pick = ev[np.random.Generator(np.random.PCG64(5)).choice(len(ev), size=min(n_pick, len(ev)), replace=False)]
rows = spcm[torch.from_numpy(pick["stream"].astype(np.int64)).to(dev)].cpu().numpy()
lp = period * 1600
segs = []
for r, ev1 in zip(rows, pick):
    n_req = (int(ev1["tick"]) * 1600 - int(ev1["ring_start"])) % 160000
    s0 = int(ev1["tick"]) * 1600 - n_req
    segs.append(r[np.arange(s0, s0 + int(ev1["length"])) % lp])
e = ewa.Engine()
e.template_from_pcm(word)
m32, s32, sc32, _ = e.score(segs, candidate_dtype="float64")
m64, s64, sc64 = e.score_f64(segs)
mn = np.linalg.norm(m64, axis=1)
T = 1 + np.array([len(x) for x in segs]) // 160
ok = np.isfinite(sc32) & np.isfinite(sc64) & (np.abs(sc32 - 75.0) > 1e-3) & (T > 16)
d = np.abs(sc32 - sc64)
print(f"{len(segs)} streaming events of {len(ev)}; fp32 (EWK_TINY_MEAN build) vs fp64, decided by fp32 alone otherwise")
edges = (0, 4, 8, 12, 16, 20, 24, 32, 40, 48, 56, 64, 80, 100, 150, 200, 400, 1e9)
for lo_, hi_ in zip(edges[:-1], edges[1:]):
    sel = ok & (mn >= lo_) & (mn < hi_)
    if sel.any():
        print(f"|mean| in [{lo_:5g}, {hi_:5g}): {int(sel.sum()):6d} events, |dscore| max {d[sel].max():.3e} "
              f"p99 {np.quantile(d[sel], 0.99):.3e} median {np.median(d[sel]):.3e}; "
              f"max |dscore| x |mean| {np.max(d[sel] * mn[sel]):.3e}")
print("NaN agreement:", bool(np.array_equal(np.isnan(sc32), np.isnan(sc64))))
