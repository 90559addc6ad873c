"""Static instruction counts of k_score_f32 by phase, from the gfx950 ISA.

    python scripts/isa_phase_count.py [--kernel k_score_f32ILi0ELi0E] [--json out.json]

Compiles csrc/ewk_mfcc.hip to gfx950 assembly with line tables, attributes every instruction
of the kernel to the source line its .loc names, groups the lines into phases (the frame
pass's stages, the tile work, the segment work) and counts VALU (v_*, MFMA apart), LDS (ds_*),
VMEM (buffer_/global_), SALU (s_*) instructions per phase and per inlined instance.

Per-frame figures: a frame-pass instance runs once per 8 frames, the tile phases once per 16
frames, the segment phases once per segment (the bench's ragged batch: 125.5 frames on
average).  The main-loop instance of the frame pass is the largest; the top_db recompute runs a
second instance (fix_tile) on ~5 % of tiles.  Shared helpers (dft4,
dft16_stage2, cmul, wave_min/max, row_sum_d...) are attributed to the phase of the caller by
the surrounding run of instructions.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "easywakeword_amd", "csrc", "ewk_mfcc.hip")


def func_ranges(src_lines):
    """{function name: (first line, last line)} of the device functions in ewk_mfcc.hip."""
    out = {}
    pat = re.compile(r"^(?:template <[^>]*>\s*)?__(?:device|global)__.*?\b(\w+)\s*\(")
    starts = []
    for i, l in enumerate(src_lines, 1):
        m = pat.match(l)
        if m:
            starts.append((i, m.group(1)))
    for k, (i, name) in enumerate(starts):
        end = starts[k + 1][0] - 1 if k + 1 < len(starts) else len(src_lines)
        out.setdefault(name, []).append((i, end))
    return out


def markers(src_lines):
    """Line numbers of the frame pass's phase comments (frame_pass body)."""
    keys = {"window": "---- window the staged samples", "twiddle": "next pass's samples: issued before the mel",
            "transpose": "---- transpose through LDS", "dft16b": "---- DFT16 over n2",
            "untangle": "---- untangle + power", "mel": "---- mel + log", "tilewrite": "Rows of frames past T keep"}
    pos = {}
    for i, l in enumerate(src_lines, 1):
        for k, s in keys.items():
            if s in l and k not in pos:
                pos[k] = i
    return pos


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="k_score_f32ILi0ELi0E")
    ap.add_argument("--json", default="")
    ap.add_argument("--frames-per-segment", type=float, default=125.5)
    args = ap.parse_args()
    out_s = "/tmp/ewk_isa_phase.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                    "--cuda-device-only", "-S", "-gline-tables-only", SRC, "-o", out_s], check=True,
                   capture_output=True)
    s = open(out_s).read()
    src = open(SRC).read().split("\n")
    fr = func_ranges(src)
    mk = markers(src)
    fp_lo, fp_hi = fr["frame_pass"][0]
    # frame-pass sub-phases by the marker comments
    cuts = sorted(mk.items(), key=lambda kv: kv[1])

    own = {int(m.group(1)) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]*)"', s, re.M)
           if m.group(2).endswith("ewk_mfcc.hip")}
    rescore = {int(m.group(1)) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]*)"', s, re.M)
               if m.group(2).endswith(("ewk_rescore.h", "ewk_db64.h"))}
    last = ["kernel: setup / loop"]

    def phase_of(file_no, line):
        if file_no in rescore:
            return "segment: epilogue (fp64 listing)"
        if file_no not in own:   # HIP / math headers: the caller's phase
            return last[0]
        last[0] = own_phase(line)
        return last[0]

    def own_phase(line):
        if fp_lo <= line <= fp_hi:
            name = "pass: setup"
            for k, l0 in cuts:
                if line >= l0:
                    name = "pass: " + k
            return name
        for f in ("stage_load", "stage_store"):
            for lo, hi in fr.get(f, []):
                if lo <= line <= hi:
                    return "pass: staging"
        for f, ph in (("dft4", "pass: fft helper"), ("dft16_stage2", "pass: fft helper"), ("dft16_perm", "pass: fft helper"),
                      ("dft16_perm_win", "pass: fft helper"), ("cmul", "pass: fft helper"), ("xpose_write", "pass: transpose"),
                      ("split2", "pass: tilewrite"), ("split8", "pass: tilewrite"), ("f16_trunc", "tile: clamp"),
                      ("clamp_load", "tile: clamp"), ("clamp_store", "tile: clamp"), ("tile_dct", "tile: dct"),
                      ("stats_add", "tile: stats"), ("stats_replace", "recompute: stats"), ("wave_min", "tile: wave min/max"),
                      ("wave_max", "tile: wave min/max"), ("zero_rows", "tile: zero rows"),
                      ("finish_stats", "segment: finish_stats"), ("row_sum_d", "segment: finish_stats"),
                      ("wave_sum_d", "segment: epilogue"), ("score_epilogue", "segment: epilogue"),
                      ("score_f64_finish", "segment: epilogue"), ("score_f32_finish", "segment: epilogue"),
                      ("tile_passes", "recompute: tile_passes"), ("fix_tile", "recompute: fix_tile"),
                      ("segment_stats", "segment: segment_stats body"), ("work_claim", "segment: work claim"),
                      ("work_order", "segment: work claim"), ("work_describe", "segment: work claim"),
                      ("make_src", "segment: work claim"), ("k_score_f32", "kernel: setup / loop")):
            for lo, hi in fr.get(f, []):
                if lo <= line <= hi:
                    return ph
        return f"line {line}"

    names = [m for m in re.findall(r"^\s*\.type\s+(\S+),@function", s, re.M) if args.kernel in m]
    if not names:
        sys.exit(f"kernel {args.kernel} not found")
    i = s.index(names[0] + ":")
    j = s.index(".Lfunc_end", i)
    cur = (0, 0)
    counts = defaultdict(lambda: defaultdict(int))
    runs = []   # contiguous runs of frame-pass phases: the inlined instances
    in_pass = False
    for raw in s[i:j].split("\n"):
        l = raw.strip()
        if l.startswith(".loc"):
            p = l.split()
            cur = (int(p[1]), int(p[2]))
            continue
        if not l or l.startswith((";", ".")) or l.endswith(":"):
            continue
        ph = phase_of(*cur)
        c = classify(l)
        counts[ph][c] += 1
        if ph.startswith("pass:"):
            if not in_pass:
                runs.append(defaultdict(int))
                in_pass = True
            runs[-1][c] += 1
        elif ph.startswith(("tile:", "segment:", "kernel:", "recompute:")) and c in ("valu", "lds"):
            in_pass = False
    rows = []
    for ph in sorted(counts):
        r = counts[ph]
        rows.append((ph, r["valu"], r["lds"], r["mfma"], r["vmem"], r["salu"]))
    print(f"{args.kernel}: static instructions by phase (all inlined instances)")
    print(f"{'phase':42s} {'VALU':>6s} {'LDS':>5s} {'MFMA':>5s} {'VMEM':>5s} {'SALU':>5s}")
    for r in rows:
        print(f"{r[0]:42s} {r[1]:6d} {r[2]:5d} {r[3]:5d} {r[4]:5d} {r[5]:5d}")
    big = sorted(runs, key=lambda r: -r["valu"])[:4]
    print("largest frame-pass runs (VALU, LDS):", [(r["valu"], r["lds"]) for r in big])
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"kernel": args.kernel, "phases": rows, "pass_runs": [dict(r) for r in big]}, f, indent=1)


if __name__ == "__main__":
    main()
