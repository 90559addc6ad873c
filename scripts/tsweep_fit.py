"""Fit kernel time per wave-segment = a + b*T from scripts/tsweep.sh output.
Usage: python scripts/tsweep_fit.py tsweep.log [waves]   (waves = 256 CUs x 8 = 2048 resident)"""
import re, sys
import numpy as np
waves = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
rows = []
for line in open(sys.argv[1]):
    m = re.search(r"L=(\d+)\s+([\d.]+) ms\s+([\d.]+) Gframes", line)
    if m:
        L, ms = int(m.group(1)), float(m.group(2))
        rows.append((L, 1 + L // 160, ms))
n = 65536
T = np.array([r[1] for r in rows], float)
us = np.array([r[2] for r in rows]) * 1e3 * waves / n      # wave-us per segment
A = np.vstack([np.ones_like(T), T]).T
(a, b), *_ = np.linalg.lstsq(A, us, rcond=None)
for (L, t, ms), u in zip(rows, us):
    print(f"L={L:6d} T={t:4d} {ms:7.3f} ms/launch  {u:7.2f} us/segment/wave  fit {a + b * t:7.2f}  "
          f"{n * t / ms / 1e6:6.3f} Gframes/s")
print(f"fit: {a:.2f} us fixed per segment per wave + {b:.4f} us per frame  (waves={waves})")
