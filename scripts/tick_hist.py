"""Distribution of the 8,192-stream streaming tick's kernel times from a rocprofv3
--kernel-trace csv: ring scorer (k_score_f32<1, *>) and gate durations, tick period.
Usage: python scripts/tick_hist.py <dir with *_kernel_trace.csv>"""
import csv, glob, os, sys
import numpy as np
f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
sc = np.array([dur(r) for r in rows if "k_score_f32<1," in r["Kernel_Name"]])
ga = np.array([dur(r) for r in rows if "k_gate_ticks" in r["Kernel_Name"]])
gs = [int(r["Start_Timestamp"]) for r in rows if "k_gate_ticks" in r["Kernel_Name"]]
per = np.diff(gs) / 1e3
print(f"scorer launches {sc.size}: mean {sc.mean():.1f} us, sum {sc.sum()/1e3:.2f} ms")
for lo, hi in ((0, 5), (5, 10), (10, 20), (20, 40), (40, 80), (80, 160), (160, 1e9)):
    m = (sc >= lo) & (sc < hi)
    print(f"  [{lo:>4},{hi if hi < 1e9 else 'inf':>4}) us: {m.sum():5d} launches, {sc[m].sum()/1e3:7.3f} ms ({100*sc[m].sum()/sc.sum():5.1f} %)")
print(f"gate launches {ga.size}: mean {ga.mean():.1f} us, median {np.median(ga):.1f}")
print(f"gate-to-gate period: median {np.median(per):.1f} us, mean {per[per < 1000].mean():.1f} us (periods < 1 ms)")
# the slowest 8,192-stream ticks (the cooperative ring scorer, k_score_f32<1, *>): gate start ->
# the tick's last kernel end, with the three launches' durations
ticks = []
gi = [i for i, r in enumerate(rows) if "k_gate_ticks" in r["Kernel_Name"]]
for a, b in zip(gi, gi[1:] + [len(rows)]):
    ks = rows[a:b]
    if not any("k_score_f32<1," in r["Kernel_Name"] for r in ks):
        continue
    t0 = int(ks[0]["Start_Timestamp"])
    te = max(int(r["End_Timestamp"]) for r in ks if "ewk::" in r["Kernel_Name"])
    part = {"gate": dur(ks[0])}
    for r in ks[1:]:
        if "k_score_f32" in r["Kernel_Name"]:
            part["scorer"] = dur(r)
        elif "k_rescore_ring" in r["Kernel_Name"]:
            part["rescore"] = dur(r)
    ticks.append(((te - t0) / 1e3, part))
ticks.sort(key=lambda x: -x[0])
print(f"slowest of {len(ticks)} cooperative-scorer ticks (gate start -> last kernel end):")
for t, p in ticks[:12]:
    print(f"  {t:7.1f} us: " + ", ".join(f"{k} {v:.1f}" for k, v in p.items()))
rs = np.array([p.get("rescore", 0.0) for _, p in ticks])
sc2 = np.array([p.get("scorer", 0.0) for _, p in ticks])
print(f"rescore: mean {rs.mean():.1f} us, p99 {np.percentile(rs, 99):.1f}, max {rs.max():.1f}; "
      f"scorer: mean {sc2.mean():.1f}, p99 {np.percentile(sc2, 99):.1f}, max {sc2.max():.1f}")
