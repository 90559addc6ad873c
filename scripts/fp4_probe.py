"""Check / time the four-lanes-per-frame pass alone (scripts/probes/fp4_probe.hip).

    python scripts/fp4_probe.py build          # hipcc, here (no GPU needed)
    python scripts/fp4_probe.py check          # on the GPU box: log-mel vs the oracle
    python scripts/fp4_probe.py time           # on the GPU box: frames/s of the pass

The check compares the probe's per-frame log-mel (dB, before top_db) with oracle/mfcc_ref.py's
float64 path on random segments, loud and quiet ones, and reports the error relative to each
frame's max (the scorer's values feed a top_db clamp at the segment max - 80 dB).
"""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROBE = os.path.join(ROOT, "scripts", "probes", "fp4_probe")
SRC = os.path.join(ROOT, "scripts", "probes", "fp4_probe.hip")


def build():
    for extra, out in (([], PROBE), (["-DFP4_TIMING"], PROBE + "_t"), (["-DFP4_NW=4"], PROBE + "_nw4")):
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", SRC,
               os.path.join(ROOT, "easywakeword_amd", "csrc", "ewk_tables.cpp"), "-o", out] + extra
        subprocess.run(cmd, check=True)


def log_mel_nodb(y: np.ndarray) -> np.ndarray:
    """oracle log-mel [T, 128] in float64 without the top_db clamp."""
    from oracle import mfcc_ref
    mel_basis, _ = mfcc_ref._tables()
    S = mfcc_ref.power_spectrogram(y.astype(np.float64))
    melspec = np.einsum("...ft,mf->...mt", S, mel_basis.astype(np.float64))
    return (10.0 * np.log10(np.maximum(1e-10, melspec))).T


def check():
    rng = np.random.default_rng(7)
    n_seg, L = 24, 16000 + 37
    segs = []
    for i in range(n_seg):
        kind = i % 4
        t = np.arange(L) / 16000.0
        if kind == 0:
            y = rng.standard_normal(L) * 0.1
        elif kind == 1:
            y = 0.5 * np.sin(2 * np.pi * (300 + 40 * i) * t) * np.exp(-3 * t) + 1e-4 * rng.standard_normal(L)
        elif kind == 2:
            y = np.convolve(rng.standard_normal(L + 64), np.ones(64) / 8, mode="valid")[:L] * 0.05
        else:
            y = rng.standard_normal(L) * np.linspace(0, 1, L) ** 3 * 0.8
        segs.append(y.astype(np.float32))
    pcm = np.stack(segs)
    tmp = "/tmp/fp4_in.f32" if os.access("/tmp", os.W_OK) else os.path.join(ROOT, "gpurun_out", "fp4_in.f32")
    out = tmp.replace("_in", "_out")
    pcm.tofile(tmp)
    subprocess.run([PROBE, "check", tmp, str(n_seg), str(L), out], check=True)
    T = 1 + L // 160
    got = np.fromfile(out, dtype=np.float32).reshape(n_seg, T, 128)
    worst = 0.0
    for i in range(n_seg):
        ref = log_mel_nodb(pcm[i])
        # error in dB, for values within 80 dB of the segment max (the rest is clamped)
        mask = ref >= ref.max() - 80.0
        err = np.abs(got[i].astype(np.float64) - ref)[mask].max()
        worst = max(worst, err)
        print(f"seg {i:2d} kind {i % 4}: max |dB err| (unclamped region) {err:.3e}   max {ref.max():7.2f} dB")
    print(f"WORST {worst:.3e} dB")
    return 0 if worst < 2e-3 else 1


def determinism():
    """4096 segments through the check kernel twice: the log-mel must be identical bit for bit."""
    rng = np.random.default_rng(11)
    n_seg, L = 4096, 16000
    pcm = (rng.standard_normal((n_seg, L)) * 0.1).astype(np.float32)
    tmp = os.path.join(ROOT, "gpurun_out", "fp4_det_in.f32")
    pcm.tofile(tmp)
    outs = []
    for k in range(2):
        out = tmp.replace("_in", f"_out{k}")
        subprocess.run([PROBE, "check", tmp, str(n_seg), str(L), out], check=True)
        outs.append(np.fromfile(out, dtype=np.float32))
        os.remove(out)
    os.remove(tmp)
    T = 1 + L // 160
    a, b = outs[0].reshape(n_seg, T, 128), outs[1].reshape(n_seg, T, 128)
    diff = np.argwhere(a != b)
    print(f"determinism: {len(diff)} differing values, {len(np.unique(diff[:, 0])) if len(diff) else 0} segments")
    if len(diff):
        segs = np.unique(diff[:, 0])[:5]
        for sg in segs:
            d = diff[diff[:, 0] == sg]
            print(f"  seg {sg}: frames {np.unique(d[:, 1])[:20]} bands {np.unique(d[:, 2])[:10]}")
    return 1 if len(diff) else 0


def mfcc_check():
    """pass + DCT (no top_db clamp) for 4096 segments, twice: bitwise identical, and a sample
    of segments against the oracle's unclamped MFCCs."""
    import scipy.fft
    rng = np.random.default_rng(12)
    n_seg, L = 4096, 16000
    pcm = (rng.standard_normal((n_seg, L)) * 0.1).astype(np.float32)
    tmp = os.path.join(ROOT, "gpurun_out", "fp4_mf_in.f32")
    pcm.tofile(tmp)
    outs = []
    for k in range(2):
        out = tmp.replace("_in", f"_out{k}")
        subprocess.run([PROBE, "mfcc", tmp, str(n_seg), str(L), out], check=True)
        outs.append(np.fromfile(out, dtype=np.float32))
        os.remove(out)
    os.remove(tmp)
    T = 1 + L // 160
    nm = n_seg * T * 20
    a, b = outs[0][:nm].reshape(n_seg, T, 20), outs[1][:nm].reshape(n_seg, T, 20)
    la, lb = outs[0][nm:].reshape(n_seg, T, 128), outs[1][nm:].reshape(n_seg, T, 128)
    nd = np.sum(a != b)
    print(f"mfcc determinism: {nd} differing values in {np.sum(np.any(a != b, axis=(1, 2)))} segments; "
          f"log-mel: {np.sum(la != lb)} differing values in {np.sum(np.any(la != lb, axis=(1, 2)))} segments")
    dl = np.argwhere(la != lb)
    if len(dl):
        dv = np.abs(la - lb)[la != lb]
        print(f"  log-mel diffs: max {dv.max():.3e} median {np.median(dv):.3e}; segs {np.unique(dl[:, 0])[:12].tolist()}")
        print(f"  frames {np.unique(dl[:, 1]).tolist()[:40]}  bands {np.unique(dl[:, 2]).tolist()[:40]}")
        for sg in np.unique(dl[:, 0])[:12]:
            d = dl[dl[:, 0] == sg]
            b = d[:, 2]
            gi = sorted({(int(x) // 32, int(x) % 8) for x in b})
            rows = sorted({(int(x) % 32) // 8 for x in b})
            ref = log_mel_nodb(pcm[sg])
            ea = np.abs(la[sg] - ref)[la[sg] != lb[sg]].max()
            eb = np.abs(lb[sg] - ref)[la[sg] != lb[sg]].max()
            print(f"  seg {sg}: pass {np.unique(d[:, 1] // 16).tolist()} n={len(d)} (G,i)={gi} rows={rows} "
                  f"err run0 {ea:.2e} run1 {eb:.2e}")
    # MFCC recomputed on the host from the probe's own log-mel (float64 DCT)
    own = scipy.fft.dct(la.astype(np.float64), axis=2, type=2, norm="ortho")[:, :, :20]
    print(f"mfcc vs host DCT of the kernel's own log-mel: worst {np.abs(a - own).max():.3e}")
    bad = np.argwhere(np.abs(a - own) > 1e-2)
    if len(bad):
        print("  first bad (seg, t, coef):", bad[:8].tolist(), " frames mod 16:", np.unique(bad[:, 1] % 16)[:16])
    worst = 0.0
    for i in range(0, n_seg, 97):
        lm = log_mel_nodb(pcm[i])                      # [T, 128] unclamped
        ref = scipy.fft.dct(lm, axis=1, type=2, norm="ortho")[:, :20]
        worst = max(worst, np.abs(a[i] - ref).max())
    print(f"mfcc vs oracle (unclamped): worst abs err {worst:.3e}")
    return 1 if nd else 0


def occupancy():
    """The pass at one wave per SIMD (4 waves per CU) against two (8 per CU), same grid."""
    for exe in (PROBE + "_nw4", PROBE):
        subprocess.run([exe, "time", "65536", "16000", "10"], check=True)


def time_(quick=False):
    for L, n in ((16000, 65536),) if quick else ((16000, 65536), (6400, 65536), (32000, 32768)):
        subprocess.run([PROBE, "time", str(n), str(L), "10"], check=True)
        subprocess.run([PROBE, "time", str(n), str(L), "10", "dct"], check=True)
    subprocess.run([PROBE + "_t", "time", "65536", "16000", "3"], check=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "check"
    if what == "build":
        build()
    elif what == "check":
        sys.exit(check())
    elif what == "mfcc":
        sys.exit(mfcc_check())
    elif what == "det":
        sys.exit(determinism())
    elif what == "occ":
        occupancy()
    else:
        time_(what == "quick")
