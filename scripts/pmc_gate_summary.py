"""Summarise scripts/pmc_gate.sh passes: the streaming kernels' counters per tick.

Usage: python scripts/pmc_gate_summary.py <dir with p*/run_counter_collection.csv> [streams] > profiles/rNN_gate_pmc.txt
Medians over the last 150 dispatches of each kernel (steady-state ticks).  SQ_* wave
counters are quad-cycles; FETCH_SIZE / WRITE_SIZE are KB (FETCH_SIZE x2 on gfx950).
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    n_streams = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    print(f"streaming-kernel PMC summary ({d}), {n_streams} streams, one tick per launch")
    # the gate grid: one wave per stream up to 131,072 workgroups of 4 waves (kGateGridMax)
    for kern, grid in (("k_gate_ticks", min(n_streams, 4 * 131072) * 64), ("k_score_f32<", None)):
        agg = collections.defaultdict(list)
        durs = []
        for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            dd = {}
            for r in csv.DictReader(open(f)):
                if kern not in r["Kernel_Name"]:
                    continue
                if grid and int(r["Grid_Size"]) != grid:
                    continue
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                dd[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            for i in sorted(per, key=int)[-150:]:
                for n, v in per[i].items():
                    agg[n].append(v)
                durs.append(dd[i])
        if not durs:
            continue
        med = {n: statistics.median(v) for n, v in agg.items()}
        print(f"\n{kern}: median dispatch {statistics.median(durs):.1f} us under counters")
        for n in sorted(med):
            print(f"  {n:22s} {med[n]:.4g}")
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if n in med:
                    print(f"  {n} / SQ_WAVE_CYCLES = {med[n] / wc:.3f}")
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            fetch = med["FETCH_SIZE"] * 2 * 1024
            write = med["WRITE_SIZE"] * 1024
            print(f"  HBM traffic per tick: fetch {fetch / 1e6:.1f} MB (FETCH_SIZE x2), write {write / 1e6:.1f} MB; "
                  f"per stream {(fetch + write) / n_streams / 1e3:.2f} KB")


if __name__ == "__main__":
    main()
