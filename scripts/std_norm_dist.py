"""|std| and |mean| (the MFCC std / mean vectors' norms) over the bench's batch and over
streaming events: how many segments a |std| < X or |mean| < Y fp64 re-score criterion would
send to k_score_f64 (DESIGN.md numerics)."""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import easywakeword_amd as ewa
dev = torch.device("cuda", 0)
word = bench.load_word()
TH = (2, 4, 8, 12, 16, 20)


def report(name, s, m=None):
    if m is not None:
        mn = np.linalg.norm(m, axis=1)
        mn = mn[np.isfinite(mn)]
        qm = np.quantile(mn, [0, 0.001, 0.01, 0.1, 0.5, 1.0])
        print(f"{name}: |mean| min {qm[0]:.1f} p0.1 {qm[1]:.1f} p1 {qm[2]:.1f} p10 {qm[3]:.1f} median {qm[4]:.1f} max {qm[5]:.1f}; "
              + ", ".join(f"<{t}: {int(np.sum(mn < t))}" for t in (100, 200, 300, 400, 500)))
    n = np.linalg.norm(s, axis=1)
    n = n[np.isfinite(n)]
    q = np.quantile(n, [0, 0.001, 0.01, 0.1, 0.5])
    print(f"{name}: {len(n)} segments, |std| min {q[0]:.2f} p0.1 {q[1]:.2f} p1 {q[2]:.2f} p10 {q[3]:.2f} median {q[4]:.2f}; "
          + ", ".join(f"<{t}: {int(np.sum(n < t))}" for t in TH))


n = 65536
pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, dev, n, 1234, word)
e = ewa.Engine()
e.template_from_pcm(word)
host = pcm.cpu().numpy()
m, s, sc, mt = e.score_packed(host, offsets, lengths, True, False)
report("bench batch (configs[1])", s, m)
del pcm
n_streams, ticks = 8192, 400
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
pick = ev[np.random.Generator(np.random.PCG64(3)).choice(len(ev), size=min(8192, len(ev)), replace=False)]
rows = spcm[torch.from_numpy(pick["stream"].astype(np.int64)).to(dev)].cpu().numpy()
lp = period * 1600
segs = []
for r, ev1 in zip(rows, pick):
    n_req = (int(ev1["tick"]) * 1600 - int(ev1["ring_start"])) % 160000
    s0 = int(ev1["tick"]) * 1600 - n_req
    segs.append(r[np.arange(s0, s0 + int(ev1["length"])) % lp])
m2, s2, sc2, mt2 = e.score(segs, candidate_dtype="float64")
report("streaming events (configs[2] recipe)", s2, m2)
# fp32 score vs the device fp64 path on the streaming segments, by |mean| bucket
m64, s64, sc64 = e.score_f64(segs)
mn = np.linalg.norm(m2, axis=1)
d = np.abs(sc2 - sc64)
ok = np.isfinite(sc2) & np.isfinite(sc64)
for lo_, hi_ in ((0, 50), (50, 100), (100, 200), (200, 400), (400, 1e9)):
    sel = ok & (mn >= lo_) & (mn < hi_)
    if sel.any():
        print(f"streaming |mean| in [{lo_}, {hi_}): {int(sel.sum())} scored, |dscore| vs fp64 max {d[sel].max():.3e} "
              f"median {np.median(d[sel]):.3e}")
print("NaN agreement:", bool(np.array_equal(np.isnan(sc2), np.isnan(sc64))))
# the ring path's own scores (StreamEngine, cooperative ring scorer + k_rescore_ring) vs the fp64 path
dr = np.abs(pick["score"] - sc64)
okr = np.isfinite(pick["score"]) & np.isfinite(sc64)
for lo_, hi_ in ((0, 50), (50, 64), (64, 100), (100, 200), (200, 400), (400, 1e9)):
    sel = okr & (mn >= lo_) & (mn < hi_)
    if sel.any():
        print(f"ring path |mean| in [{lo_}, {hi_}): {int(sel.sum())} events, |dscore| vs fp64 max {dr[sel].max():.3e} "
              f"median {np.median(dr[sel]):.3e}, re-scored {int(np.sum((pick['flags'][sel] & 2) != 0))}")
print("ring NaN agreement:", bool(np.array_equal(np.isnan(pick["score"]), np.isnan(sc64))))
