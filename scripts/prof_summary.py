"""Summarise a rocprofv3 --kernel-trace --stats csv run (scripts/gpu_round.sh prof) into text.

Usage: python scripts/prof_summary.py gpurun_out/prof <warmup launches> > profiles/rNN_<tag>_kernel_stats.txt
Lists the per-kernel stats table and, for the bench-shaped k_score_f32<0> dispatches (full grid),
the per-dispatch durations and their mean after the warmup launches (what bench.py's HIP-event
timing of the same kernel reports as roofline.kernel_ms).
"""
import csv
import os
import sys


def short(name, n=70):
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    d, warm = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0   # > 0: only the bench's timed launches
    stats = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))
    print(f"rocprofv3 --kernel-trace --stats: {d}")
    print(f"{'kernel':72s} {'calls':>6s} {'total ms':>10s} {'avg us':>10s} {'pct':>6s}")
    for r in stats[:15]:
        print(f"{short(r['Name']):72s} {int(r['Calls']):6d} {int(r['TotalDurationNs']) / 1e6:10.3f} "
              f"{float(r['AverageNs']) / 1e3:10.1f} {float(r['Percentage']):6.2f}")
    tr = [r for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))
          if "k_score_f32<0," in r["Kernel_Name"]]
    full = max(int(r["Grid_Size_X"]) for r in tr) if tr else 0
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr if int(r["Grid_Size_X"]) == full]
    print(f"\nk_score_f32<0> bench-shaped dispatches (grid {full}): " + ", ".join(f"{x:.3f}" for x in durs) + " ms")
    if len(durs) > warm:
        # (the launches after the timed ones -- short_length / fixed_length legs on the same grid --
        # are left out when `steps` is given)
        t = durs[warm:warm + steps] if steps else durs[warm:]
        print(f"mean after {warm} warmup launch(es): {sum(t) / len(t):.3f} ms over {len(t)} launches")


if __name__ == "__main__":
    main()
