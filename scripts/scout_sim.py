"""Offline model of k_score_f32's loudest-first tile order (CPU, oracle log-mel).

For segments of the bench's ragged recipe (bench.make_segments on the CPU) it computes each
16-frame tile's exact max / min log-mel (before top_db), orders the tiles by a scout
heuristic, replays the speculative clamp (running max - 80 dB, self-clamp included) and
counts the tiles and 8-frame passes the kernel would recompute.  Usage:
    python scripts/scout_sim.py [n_segments] [fixed_len]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HOP = 160


def log_mel_raw(y):
    from oracle import mfcc_ref
    mel_basis, _ = mfcc_ref._tables()
    S = mfcc_ref.power_spectrogram(y.astype(np.float64))
    mel = np.einsum("ft,mf->mt", S, mel_basis)
    return 10.0 * np.log10(np.maximum(1e-10, mel))          # [128, T]


def sample_rows(y, t, rows, width, stride, first):
    base = t * 16 * HOP
    out = []
    for q in range(rows):
        s0 = base + first + stride * q
        seg = y[max(0, s0):max(0, s0 + width)]
        out.append(seg if len(seg) == width else np.concatenate([seg, np.zeros(width - len(seg))]))
    return np.stack(out)


def heuristics(y, ntile):
    h = {}
    r4 = [sample_rows(y, t, 4, 64, 640, 64) for t in range(ntile)]
    h["H0 sum 4x64 (current)"] = np.array([float((r.astype(np.float32) ** 2).sum()) for r in r4])
    r8 = [sample_rows(y, t, 8, 32, 320, 64) for t in range(ntile)]
    h["H1 max 8x32"] = np.array([float((r ** 2).sum(axis=1).max()) for r in r8])
    h["H1b max 4x64"] = np.array([float((r ** 2).sum(axis=1).max()) for r in r4])
    r16 = [sample_rows(y, t, 16, 16, 160, 64) for t in range(ntile)]
    h["H2 max 16x16"] = np.array([float((r ** 2).sum(axis=1).max()) for r in r16])
    r8b = [sample_rows(y, t, 8, 64, 320, 64) for t in range(ntile)]   # 2x the loads
    h["H3 max 8x64 (2x loads)"] = np.array([float((r ** 2).sum(axis=1).max()) for r in r8b])
    # full coverage: the max over the tile's 16 frames of the frame energy (512-sample
    # windows, Hann-weighted or flat), and of 160-sample hop chunks
    yp = np.concatenate([np.zeros(256), y.astype(np.float64), np.zeros(256 + 16 * HOP * ntile)])
    win = np.hanning(514)[1:-1]
    fe = np.array([[float(((yp[(16 * t + f) * HOP:(16 * t + f) * HOP + 512] * win) ** 2).sum()) for f in range(16)]
                   for t in range(ntile)])
    h["H4 max frame energy (hann)"] = fe.max(axis=1)
    fe2 = np.array([[float((yp[(16 * t + f) * HOP:(16 * t + f) * HOP + 512] ** 2).sum()) for f in range(16)]
                    for t in range(ntile)])
    h["H5 max frame energy (flat)"] = fe2.max(axis=1)
    ch = np.array([[float((yp[256 + (16 * t + f) * HOP:256 + (16 * t + f + 1) * HOP] ** 2).sum()) for f in range(16)]
                   for t in range(ntile)])
    h["H6 max hop-chunk energy"] = ch.max(axis=1)
    w2 = win ** 2
    for fs, ss in ((2, 1), (4, 1), (8, 1), (4, 2), (4, 4), (8, 2), (16, 1)):
        e = np.array([[float((yp[(16 * t + f) * HOP:(16 * t + f) * HOP + 512:ss] ** 2 * w2[::ss]).sum())
                       for f in range(0, 16, fs)] for t in range(ntile)])
        h[f"H7 hann frames/{fs} samples/{ss}"] = e.max(axis=1)
    # chunked: energy of C-sample chunks, frame energy = sum of chunk energies x mean w^2
    for C in (16, 32, 64):
        wc = w2.reshape(512 // C, C).mean(axis=1)
        u = yp[:len(yp) // C * C].reshape(-1, C)
        ce = (u ** 2).sum(axis=1)
        e = np.array([[float((ce[(16 * t + f) * HOP // C:(16 * t + f) * HOP // C + 512 // C] * wc).sum())
                       for f in range(16)] for t in range(ntile)])
        h[f"H8 chunk {C} hann-weighted"] = e.max(axis=1)
    return h


POS = {}
PARK = {}


def simulate(order, tmax, tmin, pmin, name=""):
    run = -np.inf
    stored, stored_p = {}, {}
    for t in order:
        run = max(run, tmax[t] - 80.0)
        stored[t] = max(tmin[t], run)
        stored_p[t] = [max(m, run) for m in pmin[t]]
    theta = tmax.max() - 80.0
    tiles = sum(1 for t in order if stored[t] < theta)
    passes = sum(sum(1 for m in stored_p[t] if m < theta) for t in order)
    pos = POS.setdefault(name, {})
    for k, t in enumerate(order):   # processing position of the recomputed tiles
        if stored[t] < theta:
            pos[k] = pos.get(k, 0) + 1
    return tiles, passes


def main():
    import torch
    import bench
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    fixed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    word = bench.load_word()
    pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, torch.device("cpu"), n, 1234, word,
                                                                   fixed_len=fixed)
    pcm = pcm.numpy()
    tot = {}
    n_tiles = 0
    for i in range(n):
        y = pcm[offsets[i]:offsets[i] + lengths[i]].astype(np.float32)
        L = log_mel_raw(y)
        T = L.shape[1]
        ntile = (T + 15) // 16
        n_tiles += ntile
        tmax = np.array([L[:, 16 * t:min(T, 16 * t + 16)].max() for t in range(ntile)])
        tmin = np.array([L[:, 16 * t:min(T, 16 * t + 16)].min() for t in range(ntile)])
        pmin = [[L[:, p:min(T, p + 8)].min() if p < T else np.inf for p in (16 * t, 16 * t + 8)] for t in range(ntile)]
        hs = heuristics(y, ntile)
        hs["oracle (true tile max)"] = tmax
        hs["time order"] = -np.arange(ntile, dtype=float)
        # hybrid: the current scout's order, its top K re-ranked by the chunked Hann energy
        h0, h8 = hs["H0 sum 4x64 (current)"], hs["H8 chunk 32 hann-weighted"]
        for K in (2, 3, 4, 6):
            o0 = sorted(range(ntile), key=lambda t: (-h0[t], t))
            top = sorted(o0[:K], key=lambda t: (-h8[t], t))
            hs[f"H9 hybrid top {K}"] = {t: -k for k, t in enumerate(top + o0[K:])}
        for name, sc in hs.items():
            order = sorted(range(ntile), key=lambda t: (-sc[t], t))
            a, b = simulate(order, tmax, tmin, pmin, name)
            ta, tb = tot.get(name, (0, 0))
            tot[name] = (ta + a, tb + b)
        # parking policy on the current scout: park tile k if an unprocessed tile's scout energy
        # is within X dB of the best processed so far (a later tile might raise the max)
        sc = hs["H0 sum 4x64 (current)"]
        order = sorted(range(ntile), key=lambda t: (-sc[t], t))
        db = 10 * np.log10(np.maximum(sc, 1e-30))
        run = -np.inf
        stored = {}
        for k, t in enumerate(order):
            run = max(run, tmax[t] - 80.0)
            stored[t] = max(tmin[t], run)
        theta = tmax.max() - 80.0
        for X in (0, 3, 6, 10, 20):
            parked = fixed_parked = fixed_rec = 0
            best = -np.inf
            for k, t in enumerate(order):
                best = max(best, db[t])
                rest = max((db[u] for u in order[k + 1:]), default=-np.inf)
                park = rest > best - X
                need = stored[t] < theta
                parked += park
                fixed_parked += need and park
                fixed_rec += need and not park
            key = f"park X={X:2d} dB"
            pa, fp, fr = PARK.get(key, (0, 0, 0))
            PARK[key] = (pa + parked, fp + fixed_parked, fr + fixed_rec)
    print(f"{n} segments, {n_tiles} tiles (fixed_len={fixed or 'ragged'})")
    for name, (a, b) in tot.items():
        print(f"  {name:28s} recomputed tiles/segment {a / n:6.3f} ({100.0 * a / n_tiles:5.1f} % of tiles)  "
              f"passes/segment {b / n:6.3f}  positions {dict(sorted(POS.get(name, {}).items())[:6])}")
    for key, (pa, fp, fr) in PARK.items():
        print(f"  {key}: parked tiles/segment {pa / n:6.3f}, fixes from parked {fp / n:6.3f}, "
              f"recomputed {fr / n:6.3f}")


if __name__ == "__main__":
    main()
