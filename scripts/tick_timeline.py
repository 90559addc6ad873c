"""Per-tick GPU timeline of the streaming loop from a rocprofv3 --kernel-trace csv:
kernel durations and the idle gaps between consecutive dispatches (all queues).
Usage: python scripts/tick_timeline.py <dir with *_kernel_trace.csv> [ticks shown] [last tick index, default -1]"""
import csv, glob, os, sys
d = sys.argv[1]
show = int(sys.argv[2]) if len(sys.argv) > 2 else 6
end = int(sys.argv[3]) if len(sys.argv) > 3 else -1   # e.g. 420: inside the un-instrumented timed ticks
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "ewk::" in r["Kernel_Name"] or "rocclr" in r["Kernel_Name"]]
def short(n):
    for k in ("k_gate_ticks", "k_score_f32<1, 0>", "k_score_f64<1>", "k_advance", "copyBuffer", "fillBuffer", "k_snapshot", "k_normalize", "k_bank_mirror"):
        if k in n:
            return k
    return n[:30]
gates = [i for i, r in enumerate(rows) if "k_gate_ticks" in r["Kernel_Name"]]
per_tick = []
sel = gates[:end + 1] if end >= 0 else gates
for a, b in zip(sel[-show - 1:-1], sel[-show:]):
    t0 = int(rows[a]["Start_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    parts, prev_end = [], t0
    busy = 0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        parts.append(f"{short(r['Kernel_Name'])} {(e - s) / 1e3:.1f}us (gap {(s - prev_end) / 1e3:.1f})")
        prev_end = max(prev_end, e)
    print(f"tick {(t1 - t0) / 1e3:.1f} us: " + ", ".join(parts))
