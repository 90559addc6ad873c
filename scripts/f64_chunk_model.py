"""numpy model of the chunked fp64 re-score (csrc/ewk_f64.h) -- a development check of its
index maps and algebra against oracle/mfcc_ref.py, not a test of the GPU code.

Per 8-frame chunk (one wave, 64 lanes, one frame at a time):
  * z[n] = w[2n] x[2n] + i w[2n+1] x[2n+1], lane j holds n = j + 64 r (r < 4)
  * radix-4 Stockham autosort FFT, Ns = 1, 4, 16, 64: lane j reads v[r] = d[j + 64 r],
    twiddles v[r] *= W_{4 Ns}^{r (j % Ns)}, radix-4 DFT, writes V[r] to
    d'[(j // Ns) * 4 Ns + j % Ns + r Ns]; after Ns = 64 lane j holds Z[j + 64 r]
  * untangle + power, Slaney mel over each band's packed support, 10 log10 max(1e-10, .)
  * DCT split by the speculative clamp theta_s: A_k = sum_{x >= theta_s} D x,
    B_k = sum_{x < theta_s} D, so c_k = A_k + theta B_k for the exact theta as long as no
    value lies within W of theta_s (else the chunk is recomputed with the exact theta)
  * shifted sums per chunk (shift = the chunk's first frame), combined in chunk order.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import mfcc_ref  # noqa: E402


def stockham256(z):
    d = z.astype(np.complex128).copy()
    for Ns in (1, 4, 16, 64):
        out = np.zeros(256, np.complex128)
        for j in range(64):
            v = np.array([d[j + 64 * r] for r in range(4)])
            e = j % Ns
            v = v * np.exp(-2j * np.pi * np.arange(4) * e / (4 * Ns))
            V = np.array([v[0] + v[1] + v[2] + v[3],
                          v[0] - 1j * v[1] - v[2] + 1j * v[3],
                          v[0] - v[1] + v[2] - v[3],
                          v[0] + 1j * v[1] - v[2] - 1j * v[3]])
            base = (j // Ns) * 4 * Ns + e
            for r in range(4):
                out[base + r * Ns] = V[r]
        d = out
    return d


def frame_logmel(x, t, win, melw):
    """log-mel (dB, fp64) of frame t of segment x (stft center=True, constant pad)."""
    L = len(x)
    q = t * 160 - 256 + np.arange(512)
    s = np.where((q >= 0) & (q < L), x[np.clip(q, 0, L - 1)], 0.0).astype(np.float64)
    xw = s * win
    z = xw[0::2] + 1j * xw[1::2]
    Z = stockham256(z)
    k = np.arange(257)
    zk, zc = Z[k & 255], np.conj(Z[(256 - k) & 255])
    E, O = 0.5 * (zk + zc), -0.5j * (zk - zc)
    X = E + np.exp(-2j * np.pi * k / 512) * O
    P = X.real ** 2 + X.imag ** 2
    mel = melw.astype(np.float64) @ P
    return 10.0 * np.log10(np.maximum(1e-10, mel))


def chunk_sums(lm, theta_s, W, D, first):
    """lm [n, 128] log-mel of the chunk's valid frames -> (ref A, ref B, sA, sB, sAA, sAB, sBB,
    n, max, ambiguous)."""
    keep = lm >= theta_s
    A = (np.where(keep, lm, 0.0)) @ D.T       # [n, 20]
    B = (np.where(keep, 0.0, 1.0)) @ D.T
    rA, rB = A[0], B[0]
    dA, dB = A - rA, B - rB
    amb = bool(np.any(np.abs(lm - theta_s) <= W))
    return dict(rA=rA, rB=rB, sA=dA.sum(0), sB=dB.sum(0), sAA=(dA * dA).sum(0), sAB=(dA * dB).sum(0),
                sBB=(dB * dB).sum(0), n=len(lm), mx=float(lm.max()), amb=amb)


def model_stats(x, theta_s, W=1e-3, F=8):
    melw, win = mfcc_ref._tables()
    D = np.array([[(np.sqrt(1 / 128) if k == 0 else np.sqrt(2 / 128)) * np.cos(np.pi * k * (2 * m + 1) / 256)
                   for m in range(128)] for k in range(20)])
    T = 1 + len(x) // 160
    lm = np.array([frame_logmel(x, t, win, melw) for t in range(T)])
    parts = [chunk_sums(lm[c:c + F], theta_s, W, D, c) for c in range(0, T, F)]
    theta = max(p["mx"] for p in parts) - 80.0
    recomputed = 0
    for i, p in enumerate(parts):
        if p["amb"] or abs(theta - theta_s) > W:
            parts[i] = chunk_sums(lm[i * F:(i + 1) * F], theta, 0.0, D, i * F)
            recomputed += 1
    ref0 = parts[0]["rA"] + theta * parts[0]["rB"]
    S1 = np.zeros(20)
    S2 = np.zeros(20)
    for p in parts:
        s1 = p["sA"] + theta * p["sB"]
        s2 = p["sAA"] + 2 * theta * p["sAB"] + theta * theta * p["sBB"]
        dl = p["rA"] + theta * p["rB"] - ref0
        S2 += s2 + 2 * dl * s1 + p["n"] * dl * dl
        S1 += s1 + p["n"] * dl
    mean = ref0 + S1 / T
    var = np.maximum((S2 - S1 * S1 / T) / T, 0.0)
    return mean, np.sqrt(var), recomputed


def rs_swz(i):
    """FFT buffer slot of complex element i (ewk_rescore.h rs_swz)."""
    return i ^ (((i >> 4) * 5) & 15)


def swizzle_conflicts():
    """Worst bank-group multiplicity of each 16-lane group's 16-B accesses (1 = conflict free)
    for the Stockham stores, the natural-order reads and the untangle's partner reads, with and
    without rs_swz; also checks that rs_swz permutes 0..255."""
    from collections import Counter
    assert sorted(rs_swz(i) for i in range(256)) == list(range(256))

    def worst(addrs):
        return max(max(Counter(a % 16 for a in addrs[16 * q:16 * q + 16]).values()) for q in range(4))

    out = {}
    for name, f in (("plain", lambda i: i), ("swizzled", rs_swz)):
        st = max(worst([f((((l >> lg) << (lg + 2)) + (l & ((1 << lg) - 1)) if lg < 6 else l) + (r << lg))
                        for l in range(64)]) for lg in (0, 2, 4, 6) for r in range(4))
        rd = max(worst([f(l + 64 * r) for l in range(64)]) for r in range(4))
        un = max(worst([f((256 - (l + 64 * r)) & 255) for l in range(64)]) for r in range(4))
        out[name] = {"stores": st, "reads": rd, "untangle_reads": un}
    return out


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
    import synth
    rng = np.random.default_rng(3)
    word = synth.load_word().astype(np.float64)
    cases = [word, rng.normal(0, 1e-3, 6400), np.concatenate([rng.normal(0, 1e-4, 8000), word * 3.0])]
    for x in cases:
        m_ref, s_ref = mfcc_ref.extract_mfcc(x)
        th32 = float(mfcc_ref.log_mel(x.astype(np.float32)).max()) - 80.0   # an f32-ish estimate
        m, s, rc = model_stats(x, th32)
        print(f"T={1 + len(x) // 160:4d} recomputed={rc} |dmean|={np.abs(m - m_ref).max():.3e} "
              f"|dstd|={np.abs(s - s_ref).max():.3e}")
