"""numpy model of the round-5 frame pass ("four lanes per frame") -- index algebra only.

A wave holds 16 frames x 4 rows: lane = p + 16 r (p = frame of the pass, r = row).  This
model replays, for one frame, what the four lanes of a frame hold at every step, in float64,
and checks the power spectrum, the mel band energies and the band -> DCT-slot map against
numpy.  It also prints the tables' sizes and the mel incidence count the kernel unrolls.
The HIP code (scripts/experiments/fp4/ewk_fp4.h) and the host tables (ewk_tables.cpp,
build_tables) follow the same maps; tests/test_fp4_tables.py checks the C++ tables against
the functions below.

Steps (z[n] = x[2n] w[2n] + i x[2n+1] w[2n+1], n < 256):
  1. row r holds z[r + 4 n'], n' < 64                       (staged samples, window)
  2. in-lane DFT64 over n':   Y_r[k'']                      (4 DFT16 + W64 twiddles + DFT4)
  3. transposition T (v_permlane16_swap, v_permlane32_swap): quad q of row g holds
     Y_s[I_g(q)] for s = 0..3 in registers named by item I_s(q)
  4. V_s = Y_s W256^(s k''), Z[k'' + 64 k'] = sum_s V_s W4^(s k')   (k'' = I_g(q))
  5. untangle pairs (q, k') <-> (15 - q, 3 - k'); row 0 slot pair (0, 15) is special
  6. mel partial sums over the row's 64 bins, reduce-scatter over the 4 rows:
     row r ends with bands 32 G + 8 r + i (G = DCT k-step, i < 8)
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

SIGMA = [0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11, 12, 13, 14, 15, 8]   # row 0 slot -> k''/4


def item(g: int, q: int) -> int:
    """k'' held in slot q of row g after the transposition."""
    if g == 0:
        return 4 * SIGMA[q]
    if g == 2:
        return 4 * q + 2
    if g == 1:
        return 4 * q + (1 if q < 8 else 3)
    return 4 * q + (3 if q < 8 else 1)


def bin_of(g: int, q: int, kp: int) -> int:
    return item(g, q) + 64 * kp


def untangle_pairs(g: int):
    """32 pair computations of row g: (u slot, v slot, bin of u, out slot of P[u], out slot of P[v]).

    Slots are (q, k').  Regular pair j = 4 q + k' (q < 8): u = (q, k'), v = (15 - q, 3 - k').
    Row 0, q = 0 is special: bins 64/192, 32/224, 96/160 and 128 (self); bin 0 and 256 carry
    zero mel weight and are not produced."""
    out = []
    for q in range(8):
        for kp in range(4):
            u, v = (q, kp), (15 - q, 3 - kp)
            if g == 0 and q == 0:
                u, v = [((0, 1), (0, 3)), ((15, 0), (15, 3)), ((15, 1), (15, 2)), ((0, 2), (0, 2))][kp]
            out.append((u, v, bin_of(g, *u), u, v))
    return out


def check_layout():
    for g in range(4):
        bins = sorted(bin_of(g, q, kp) for q in range(16) for kp in range(4))
        assert len(set(bins)) == 64
        # every 4-block [4b, 4b+4) holds exactly one bin of each row
        assert all(len([b for b in bins if b // 4 == blk]) == 1 for blk in range(64)), g
        for (u, v, ku, _, _) in untangle_pairs(g):
            bu, bv = bin_of(g, *u), bin_of(g, *v)
            assert bu == ku
            assert bu + bv == 256 or (bu == bv == 128), (g, u, v, bu, bv)
    cover = set()
    for g in range(4):
        for (u, v, *_r) in untangle_pairs(g):
            cover.add(bin_of(g, *u))
            cover.add(bin_of(g, *v))
    assert cover == set(range(1, 256)), sorted(set(range(1, 256)) - cover)


def stft_frame(x: np.ndarray, w: np.ndarray):
    """Power spectrum |X|^2 (257) of one frame through the lane algorithm, in float64."""
    xw = x * w
    z = xw[0::2] + 1j * xw[1::2]                       # 256
    Y = [np.fft.fft(z[r::4]) for r in range(4)]        # row r: DFT64 over n' (z[r + 4 n'])
    P = {}
    for g in range(4):
        Z = {}
        for q in range(16):
            kpp = item(g, q)
            V = [Y[s][kpp] * np.exp(-2j * np.pi * s * kpp / 256) for s in range(4)]
            for kp in range(4):
                Z[(q, kp)] = sum(V[s] * np.exp(-2j * np.pi * s * kp / 4) for s in range(4))
        for (u, v, ku, ou, ov) in untangle_pairs(g):
            zu, zv = Z[u], Z[v]
            A = zu + np.conj(zv)
            B = zu - np.conj(zv)
            C = 1j * np.exp(-2j * np.pi * ku / 512) * B
            P[bin_of(g, *ou)] = abs(A - C) ** 2 / 4
            P[bin_of(g, *ov)] = abs(A + C) ** 2 / 4
    return P


def mel_incidence(W: np.ndarray):
    """R_m = register slots (q, k') some row holds a bin of band m in; per-row weights."""
    inc = []
    for m in range(128):
        nz = np.nonzero(W[m])[0]
        lo, hi = nz[0], nz[-1]
        regs = sorted({(q, kp) for g in range(4) for q in range(16) for kp in range(4)
                       if lo <= bin_of(g, q, kp) <= hi})
        inc.append(regs)
    return inc


def main():
    from oracle import mfcc_ref
    check_layout()
    W = mfcc_ref.mel_filterbank().astype(np.float64)
    win = mfcc_ref.hann_window()
    rng = np.random.default_rng(1)
    x = rng.standard_normal(512)
    P = stft_frame(x, win)
    ref = np.abs(np.fft.rfft(x * win)) ** 2
    err = max(abs(P[k] - ref[k]) / ref.max() for k in P)
    print(f"power spectrum via lanes: {len(P)} bins, max rel err {err:.2e}")
    assert err < 1e-12
    inc = mel_incidence(W)
    n_inc = sum(len(r) for r in inc)
    print(f"mel incidences (uniform register FMAs per lane per frame-pass): {n_inc}")
    # band energies from per-row partial sums, reduce-scatter bookkeeping
    E = np.zeros(128)
    for g in range(4):
        for m in range(128):
            for (q, kp) in inc[m]:
                b = bin_of(g, q, kp)
                E[m] += W[m, b] * P.get(b, 0.0)
    Eref = W @ ref
    print(f"mel energies max rel err {np.max(np.abs(E - Eref) / Eref.max()):.2e}")
    # reduce-scatter: row r, register (G, i) = band 32 G + 8 r + i
    for G in range(4):
        acc = {r: np.arange(32) + 32 * G for r in range(4)}          # band ids per register
        s1 = {r: (acc[r][:16] if r < 2 else acc[r][16:]) for r in range(4)}
        s2 = {r: (s1[r][:8] if r % 2 == 0 else s1[r][8:]) for r in range(4)}
        for r in range(4):
            assert list(s2[r]) == [32 * G + 8 * r + i for i in range(8)]
    print("reduce-scatter map: row r register (G, i) = band 32 G + 8 r + i")


if __name__ == "__main__":
    main()


def emit_header(path: str) -> None:
    """scripts/experiments/fp4/ewk_fp4_mel.h: the mel incidence list the kernel unrolls."""
    from oracle import mfcc_ref
    W = mfcc_ref.mel_filterbank().astype(np.float64)
    inc = mel_incidence(W)
    lines = ["// ewk_fp4_mel.h -- GENERATED by scripts/fp4_model.py (emit_header); do not edit.",
             "// Mel incidence list of the four-lanes-per-frame pass (ewk_fp4.h): band group G (DCT",
             "// k-step, bands 32 G .. 32 G + 31) lists (band - 32 G, power slot 4 q + k') for every slot",
             "// in which some row holds a bin of the band's Slaney support (librosa 0.11.0, n_fft 512,",
             "// 128 mels, 0..8 kHz).  ewk_tables.cpp rebuilds it from the basis and checks it (ok4).",
             "#pragma once", "", "namespace ewk {", ""]
    counts, bands, slots = [], [], []
    for G in range(4):
        n0 = len(bands)
        # round robin over the group's bands (the k-th incidence of every band, then the
        # (k+1)-th): consecutive FMAs accumulate into different bands, no dependency chains
        per = [inc[m] for m in range(32 * G, 32 * G + 32)]
        for k in range(max(len(x) for x in per)):
            for j, regs in enumerate(per):
                if k < len(regs):
                    q, kp = regs[k]
                    bands.append(j)
                    slots.append(4 * q + kp)
        counts.append(len(bands) - n0)
        while (len(bands) - n0) % 4:        # pad each group to whole b128 weight reads
            bands.append(0)
            slots.append(0)
    starts = [0]
    for G in range(4):
        n = counts[G] + (-counts[G]) % 4
        starts.append(starts[-1] + n)
    lines.append(f"constexpr int F4_NINC = {starts[-1]};   // incidences incl. per-group padding (zero weights)")
    lines.append("constexpr int F4_INC_START[5] = {" + ", ".join(map(str, starts)) + "};")
    lines.append("constexpr int F4_INC_COUNT[4] = {" + ", ".join(map(str, counts)) + "};")
    for name, arr in (("F4_INC_BAND", bands), ("F4_INC_SLOT", slots)):
        lines.append(f"constexpr unsigned char {name}[F4_NINC] = {{")
        for i in range(0, len(arr), 24):
            lines.append("    " + ", ".join(map(str, arr[i:i + 24])) + ",")
        lines.append("};")
    lines += ["", "}  // namespace ewk", ""]
    with open(path, "w") as f:
        f.write("\n".join(lines))
    print(f"wrote {path}: {starts[-1]} incidences ({counts})")
