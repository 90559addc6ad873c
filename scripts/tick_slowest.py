"""Slowest streaming ticks of one leg from a rocprofv3 --kernel-trace csv: each tick = a gate
launch and the kernels up to the next gate; kept when its scorer's name contains SCORER
(default "k_score_f32<2, 1>": the int16 one-segment-per-wave ring scorer of streaming_max).
Prints the slowest ticks (gate start -> last kernel end) with each launch's duration, and the
gate / scorer / re-score distributions.
The bench's leg runs 100 prefill ticks in launches of 32, then its timed ticks one per launch,
then an instrumented pass: FIRST / COUNT select the timed ticks by their order in the trace.
Usage: python scripts/tick_slowest.py <dir with *_kernel_trace.csv> [SCORER] [n shown] [FIRST] [COUNT]"""
import csv
import glob
import os
import sys

import numpy as np

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "k_score_f32<2, 1>"
show = int(sys.argv[3]) if len(sys.argv) > 3 else 15
first = int(sys.argv[4]) if len(sys.argv) > 4 else 0
count = int(sys.argv[5]) if len(sys.argv) > 5 else 1 << 30
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "ewk::" in r["Kernel_Name"]]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
gi = [i for i, r in enumerate(rows) if "k_gate_ticks" in r["Kernel_Name"]]
ticks = []
for a, b in zip(gi, gi[1:] + [len(rows)]):
    ks = rows[a:b]
    if not any(want in r["Kernel_Name"] for r in ks):
        continue
    t0 = int(ks[0]["Start_Timestamp"])
    te = max(int(r["End_Timestamp"]) for r in ks)
    p = {"gate": dur(ks[0])}
    for r in ks[1:]:
        n = r["Kernel_Name"]
        k = "scorer" if "k_score_f32" in n else ("rescore" if "k_rescore" in n else n.split("(")[0][-24:])
        p[k] = p.get(k, 0.0) + dur(r)
    ticks.append(((te - t0) / 1e3, a, p))
print(f"{len(ticks)} ticks with a '{want}' scorer; gate durations in trace order (ms):")
print("  " + " ".join(f"{p['gate'] / 1e3:.1f}" for _, _, p in ticks))
ticks = ticks[first:first + count]
print(f"ticks {first} .. {first + len(ticks) - 1} analysed")
for name in ("gate", "scorer", "rescore"):
    v = np.array([p.get(name, 0.0) for _, _, p in ticks])
    if v.size:
        print(f"  {name:8s} mean {v.mean():9.1f} us  p50 {np.median(v):9.1f}  p99 {np.percentile(v, 99):9.1f}  max {v.max():9.1f}")
tot = np.array([t for t, _, _ in ticks])
if tot.size:
    print(f"  tick     mean {tot.mean():9.1f} us  p50 {np.median(tot):9.1f}  p99 {np.percentile(tot, 99):9.1f}  max {tot.max():9.1f}")
order = sorted(ticks, key=lambda x: -x[0])
print("slowest ticks (index in the trace, duration, parts):")
for t, a, p in order[:show]:
    print(f"  #{a:6d} {t:9.1f} us: " + ", ".join(f"{k} {v:.1f}" for k, v in p.items()))
