"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh) for k_score_f32 into one text report.

Usage: python scripts/pmc_summary.py gpurun_out/pmc_<tag> <n_segments> [traffic.json] > profiles/rNN_<tag>_pmc.txt
(traffic.json: HBM bytes per launch / per frame for bench.py's roofline.traffic)

Units (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units" and the HBM section):
SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* count quad-cycles; FETCH_SIZE / WRITE_SIZE are KB,
FETCH_SIZE reports half the bytes of a wide coalesced read on gfx950 (doubled below).
"""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np

HOP = 160


def bench_frames(n_seg, seed=1234):
    # bench.make_segments' length draw, without building the PCM
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = rng.integers(6400, 33600 + 1, n_seg).astype(np.int64)
    return int((1 + lengths // HOP).sum()), int(lengths.sum())


def main():
    d, n = sys.argv[1], int(sys.argv[2])
    frames, samples = bench_frames(n)
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if "k_score_f32" not in r["Kernel_Name"] or int(r["Grid_Size"]) < 1024:
                continue
            per[f][(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
            meta.setdefault(f, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    c = {}
    for f, vals in per.items():
        by = defaultdict(list)
        for (name, _), v in vals.items():
            by[name].append(v)
        for name, v in by.items():
            c[name] = float(np.median(v))
    ms = float(np.median([t for ts in meta.values() for t in ts]))
    waves = c.get("SQ_WAVES", 0)
    print(f"k_score_f32 PMC summary: {n} segments, {frames} frames, {samples} samples per launch")
    print(f"median dispatch duration under counters: {ms:.3f} ms")
    for k in sorted(c):
        print(f"  {k:28s} {c[k]:.4g}")
    if waves:
        wc = c["SQ_WAVE_CYCLES"] * 4 / waves
        print("\nper wave (cycles; quad-cycle counters x4):")
        print(f"  lifetime                 {wc:,.0f}")
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY",
                  "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY"):
            if k in c:
                v = c[k] * 4 / waves
                print(f"  {k:24s} {v:,.0f}  ({100 * v / wc:.1f}% of lifetime)")
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_MFMA"):
            if k in c:
                print(f"  {k:24s} {c[k] / waves:,.0f} instr  ({c[k] / frames:.1f} per frame)")
        if "SQ_INSTS_VALU" in c:
            # wave64 VALU occupies the SIMD's vector pipe 2 cycles; 2 waves share a SIMD here
            simd_busy = c["SQ_INSTS_VALU"] * 2 / (waves / 2) / wc
            print(f"  VALU pipe utilisation (2 cyc/instr, waves/SIMD = {waves / 1024:.0f}): {100 * simd_busy:.1f}%")
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_ACTIVE_INST_LDS" in c:
            print(f"  LDS bank-conflict cycles / LDS active cycles: "
                  f"{c['SQ_LDS_BANK_CONFLICT'] / (4 * c['SQ_ACTIVE_INST_LDS']):.3f}")
    if "FETCH_SIZE" in c:
        fetch = c["FETCH_SIZE"] * 1024 * 2
        write = c.get("WRITE_SIZE", 0) * 1024
        alg = frames * 640
        print(f"\nHBM traffic per launch: fetch {fetch / 1e9:.3f} GB (FETCH_SIZE x2, gfx950), "
              f"write {write / 1e9:.3f} GB, total {(fetch + write) / 1e9:.3f} GB")
        print(f"algorithmic bytes per launch (640 B/frame): {alg / 1e9:.3f} GB; "
              f"traffic/algorithmic = {(fetch + write) / alg:.2f}")
        print(f"  (fetch = segment samples, incl. the re-read of the tiles the top_db pass recomputes; write = results)")
        if len(sys.argv) > 3:
            import json
            with open(sys.argv[3], "w") as fh:
                import datetime
                json.dump({"kernel": "k_score_f32", "segments": n, "frames": frames,
                           "head": os.environ.get("EWK_HEAD", "unknown"),
                           "date_utc": datetime.datetime.utcnow().strftime("%Y-%m-%dT%H:%M:%SZ"),
                           "valu_active_frac": (c["SQ_ACTIVE_INST_VALU"] * 4 / waves) / (c["SQ_WAVE_CYCLES"] * 4 / waves)
                           if waves and "SQ_ACTIVE_INST_VALU" in c else None,
                           "fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
                           "traffic_bytes_per_frame": (fetch + write) / frames,
                           # wave-instructions per MFCC frame (bench.py's VALU-issue roofline)
                           "valu_instr_per_frame": c.get("SQ_INSTS_VALU", 0.0) / frames,
                           "lds_instr_per_frame": c.get("SQ_INSTS_LDS", 0.0) / frames,
                           "mfma_instr_per_frame": c.get("SQ_INSTS_MFMA", 0.0) / frames,
                           "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE, SQ_INSTS_* "
                                     "in separate passes, median over dispatches of scripts/mb_score.py"}, fh, indent=1)


if __name__ == "__main__":
    main()
