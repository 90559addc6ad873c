"""Per-tick fp64 re-score load of the streaming path (the bench's 8,192-stream recipe): events
listed (EWK_EV_RESCORED) per tick, their frames and chunks, and the k_rescore_ring time per tick
(profile kind 1), to tell a slow chunk from a serial drain."""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import easywakeword_amd as ewa

dev = torch.device("cuda", 0)
word = bench.load_word()
n_streams = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 60
period, spcm = bench.make_streams(torch, dev, n_streams, 1234, word)
se = ewa.StreamEngine(n_streams)
se.template_from_pcm(word)
base = spcm.data_ptr()
t = 0
while t < 100:   # prefill
    k = t % period
    n = min(32, 100 - t, period - k)
    se.push_device(base + k * 1600 * 4, period * 1600, 1600, n)
    se.poll()
    t += n
se.sync()
import ctypes
dlib = ctypes.CDLL(os.environ.get("EWK_LIB") or os.path.join(ROOT, "easywakeword_amd", "libewk.so"))
dbg = hasattr(dlib, "ewk_debug_rs")
dbuf = (ctypes.c_ulonglong * 16)()
if dbg:
    dlib.ewk_debug_rs(dbuf)
    if hasattr(dlib, "ewk_debug_rs_ph"):
        dlib.ewk_debug_rs_ph((ctypes.c_ulonglong * 8)())
rows = []
dmax = [0]
for i in range(ticks):
    k = t % period
    se.profile(True)
    se.push_device(base + k * 1600 * 4, period * 1600, 1600, 1)
    ev = se.poll()
    se.sync()
    sc_ms, _ = se.profile_read(0)
    r_ms, _ = se.profile_read(1)
    se.profile(False)
    real = ev[(ev["flags"] & 1) == 0]
    rs = real[(real["flags"] & 2) != 0]
    if dbg:
        dlib.ewk_debug_rs(dbuf)
        if len(rs):
            d = list(dbuf)
            print(f"  tick {i}: drain waves {d[0]} wgs {d[9]} chunks {d[1]} ({d[2] / max(1, d[1]):,.0f} cyc each) "
                  f"finishes {d[3]} ({d[4] / max(1, d[3]):,.0f} cyc each) serial {d[5]} redo_all {d[6]} "
                  f"chunks-in-finished {d[7]} recomputed {d[8]}; drain per wave max {d[10] / 100:.0f} us mean {d[11] / 100 / max(1, d[0]):.0f} us; "
                  f"claim scans {d[12]}; last-WG tail {d[13] / 100:.1f} us; max |theta - theta_s| {d[14] * 1e-9:.2e} dB")
            dmax[0] = max(dmax[0], d[14])
    T = 1 + rs["length"].astype(np.int64) // 160
    rows.append((len(real), len(rs), int(T.sum()), int(((T + 7) // 8).sum()), int(T.max()) if len(T) else 0, sc_ms * 1e3, r_ms * 1e3))
    t += 1
if dbg and hasattr(dlib, "ewk_debug_rs_ph"):
    ph = (ctypes.c_ulonglong * 8)()
    dlib.ewk_debug_rs_ph(ph)   # (accumulated over all timed ticks; the prefill's were reset above)
    ph = list(ph)
    nch, ngr = max(1, ph[6]), max(1, ph[7])
    print(f"chunk sub-phases over {ph[6]} chunks ({ph[7]} frame groups), s_memtime cycles per chunk: "
          f"samples+window {ph[0] / nch:,.0f}  FFT {ph[1] / nch:,.0f}  untangle {ph[2] / nch:,.0f}  "
          f"mel+log10 {ph[3] / nch:,.0f}  DCT {ph[4] / nch:,.0f}  sums+flags {ph[5] / nch:,.0f}  "
          f"(total {sum(ph[:6]) / nch:,.0f})")
a = np.array(rows, dtype=np.float64)
print("tick events listed frames chunks maxT scorer_us rescore_us")
for r in rows[:40]:
    print(" ".join(f"{x:.0f}" if j < 5 else f"{x:.1f}" for j, x in enumerate(r)))
print("mean: events %.1f listed %.2f frames %.1f chunks %.1f scorer %.1f us rescore %.1f us" % tuple(a[:, [0, 1, 2, 3, 5, 6]].mean(0)))
sel = a[:, 1] == 0
if sel.any():
    print("ticks without a listed event: %d, rescore %.1f us" % (sel.sum(), a[sel, 6].mean()))
if (~sel).any():
    print("ticks with listed events: %d, rescore %.1f us, per chunk %.2f us, per max-T frame %.2f us" % (
        (~sel).sum(), a[~sel, 6].mean(), (a[~sel, 6] / a[~sel, 3]).mean(), (a[~sel, 6] / np.maximum(a[~sel, 4], 1)).mean()))
if dbg:
    print(f"max |theta - theta_s| over the listed segments: {dmax[0] * 1e-9:.3e} dB (window {os.environ.get('EWK_RS_WINDOW_NOTE', '')})")
