"""Median gap (us) from a k_fill end to the next kernel's start, per following kernel + LDS size."""
import csv, glob, sys, collections
import numpy as np
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
gaps = collections.defaultdict(list)
for a, b in zip(rows, rows[1:]):
    if "k_fill" in a["Kernel_Name"] and "k_fill" not in b["Kernel_Name"]:
        key = b["Kernel_Name"].split("(")[0] + " lds=" + b.get("LDS_Block_Size", b.get("Lds_Size", "?")) + \
              " scratch=" + b.get("Scratch_Size", b.get("Private_Segment_Size", "?"))
        gaps[key].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for k, v in gaps.items():
    print(f"{k}: median gap {np.median(v[5:]):.2f} us over {len(v) - 5}")
fills = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_fill" in r["Kernel_Name"]]
print(f"k_fill median {np.median(fills):.1f} us")
