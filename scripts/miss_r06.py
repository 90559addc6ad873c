"""Round-6 recurrence of the ring-path score miss: model search on the CPU (oracle).

The round-6 session `r06_v10` failed tests/test_gpu_gate.py::test_many_streams_vs_oracle with
two events, full precision kept by tests/evidence.py:
    stream 1 tick 164 L 14400 ring_start 82400: 97.77742062925678, oracle 98.04756856169448
    stream 0 tick 196 L 17600 ring_start 128800: 99.25763811033005, oracle 99.22792074878643
(round 5: stream 1 tick 164 at 98.3817).  The ring read back after the run and scored by the
linear batch scorer gives the oracle's value (98.0475693, 99.2282756): the ring memory held
the right samples.  This scores, with the oracle, what the ring scorer would return under each
corruption model and prints the nearest ones:
  A. log-mel level (the cooperative scorer: wave w owns tile w of a <= 8-tile segment): a tile
     dropped, zeroed, duplicated from another, left unclamped, clamped at its own max - 80, or
     the segment threshold taken without one tile's max;
  B. sample level, 32-sample (128 B) granularity: every run of lines replaced by the samples one
     ring wrap earlier (stale), zeros, the neighbouring stream's samples, or the samples one tick
     earlier / later.
Usage: python scripts/miss_r06.py [--samples]
"""
import os
import sys

import numpy as np
import scipy.fft

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)

from golden_io import matcher_fixture, template_arrays  # noqa: E402
from oracle import mfcc_ref  # noqa: E402
import miss_r05  # noqa: E402

R = 160000
CASES = [(1, 164, 14400, 82400, 97.77742062925678, 98.04756856169448),
         (0, 196, 17600, 128800, 99.25763811033005, 99.22792074878643)]


def raw_log_mel(y):
    mel_basis, _ = mfcc_ref._tables()
    S = mfcc_ref.power_spectrogram(np.asarray(y, np.float64))
    return 10.0 * np.log10(np.maximum(mfcc_ref.AMIN, np.einsum("ft,mf->mt", S, mel_basis)))


def score_from_logmel(lm, tm, ts, theta=None):
    if theta is None:
        theta = lm.max() - 80.0
    c = scipy.fft.dct(np.maximum(lm, theta), axis=0, type=2, norm="ortho")[:20]
    return float(mfcc_ref.similarity_from_stats(tm, ts, c.mean(1), c.std(1)))


def main():
    fx, _ = matcher_fixture()
    tm, ts = template_arrays(fx)
    data = miss_r05.scenario()
    for st, tick, ln, rs, target, oracle in CASES:
        p = (tick - 1) // 16
        end = (16 * p + 16) * 1600
        j0 = end - 1 - ((end - 1 - rs) % R)          # stream index of ring position rs now
        if j0 + ln > end:
            j0 -= R
        seg = data[st][j0:j0 + ln].astype(np.float64)
        lm = raw_log_mel(seg)
        base = score_from_logmel(lm, tm, ts)
        print(f"stream {st} tick {tick}: oracle {oracle:.8f} (recomputed {base:.8f}), engine {target:.8f}; "
              f"segment = stream samples [{j0}, {j0 + ln}), push {p} ends at sample {end}")
        T = lm.shape[1]
        nt = (T + 15) // 16
        res = []
        for k in range(nt):
            cols = slice(16 * k, min(T, 16 * k + 16))
            keep = np.ones(T, bool)
            keep[cols] = False
            res.append((f"tile {k} dropped", score_from_logmel(lm[:, keep], tm, ts)))
            z = lm.copy(); z[:, cols] = -100.0
            res.append((f"tile {k} at the -100 dB floor", score_from_logmel(z, tm, ts)))
            others = np.delete(lm, np.r_[cols], axis=1)
            res.append((f"theta without tile {k}'s max", score_from_logmel(lm, tm, ts, theta=others.max() - 80.0)))
            u = np.maximum(lm, lm.max() - 80.0)
            u[:, cols] = lm[:, cols]                    # this tile unclamped
            c = scipy.fft.dct(u, axis=0, type=2, norm="ortho")[:20]
            res.append((f"tile {k} unclamped", float(mfcc_ref.similarity_from_stats(tm, ts, c.mean(1), c.std(1)))))
            u = np.maximum(lm, lm.max() - 80.0)
            u[:, cols] = np.maximum(lm[:, cols], lm[:, cols].max() - 80.0)
            c = scipy.fft.dct(u, axis=0, type=2, norm="ortho")[:20]
            res.append((f"tile {k} clamped at its own max", float(mfcc_ref.similarity_from_stats(tm, ts, c.mean(1), c.std(1)))))
            for k2 in range(nt):
                if k2 == k:
                    continue
                d = lm.copy()
                w = min(T, 16 * k + 16) - 16 * k
                w2 = min(T, 16 * k2 + 16) - 16 * k2
                ww = min(w, w2)
                d[:, 16 * k:16 * k + ww] = lm[:, 16 * k2:16 * k2 + ww]
                res.append((f"tile {k} := tile {k2}", score_from_logmel(d, tm, ts)))
        if "--samples" in sys.argv:
            srcs = {"stale (one wrap earlier)": data[st][j0 - R:j0 - R + ln] if j0 >= R else None,
                    "zeros": np.zeros(ln),
                    "stream+1": data[st + 1][j0:j0 + ln], "stream-1": data[st - 1][j0:j0 + ln] if st else None,
                    "one tick earlier": data[st][j0 - 1600:j0 - 1600 + ln],
                    "one tick later": data[st][j0 + 1600:j0 + 1600 + ln]}
            nl = ln // 32
            for name, alt in srcs.items():
                if alt is None:
                    continue
                alt = np.asarray(alt, np.float64)
                for a in range(nl):
                    for b in (1, 2, 4, 8, 16, 25, 50, 100):
                        if a + b > nl:
                            break
                        y = seg.copy()
                        y[32 * a:32 * (a + b)] = alt[32 * a:32 * (a + b)]
                        cm, cs = mfcc_ref.extract_mfcc(y)
                        res.append((f"samples [{32 * a}, {32 * (a + b)}) from {name}",
                                    float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))))
        res.sort(key=lambda r: abs(r[1] - target))
        for name, s in res[:8]:
            print(f"   {s:.8f}  d {s - target:+.2e}  {name}")


if __name__ == "__main__":
    main()
