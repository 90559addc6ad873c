"""Print the streaming lines of one bench.py JSON line (stdin): us/tick, gate/scorer us, events."""
import json, sys
src = open(sys.argv[1]) if len(sys.argv) > 1 else sys.stdin
d = json.loads([l for l in src.read().splitlines() if l.startswith("{")][-1])
for k in ("streaming", "streaming_f32_max", "streaming_max"):
    s = d.get(k)
    if s:
        print(k, s["streams"], "%.1f us/tick" % (s["ms_per_tick"] * 1e3), "gate %.1f" % (s["gate_kernel_ms_per_tick"] * 1e3),
              "scorer %.1f" % (s["scorer_kernel_ms_per_tick"] * 1e3),
              "rescore %.1f" % (s.get("rescore_kernel_ms_per_tick", 0.0) * 1e3), "max %.1f us" % ((s.get("tick_ms_max") or 0.0) * 1e3), "p999 %.1f" % ((s.get("tick_ms_p999") or 0.0) * 1e3),
              "events", s["events"], "matches", s["matches"])
