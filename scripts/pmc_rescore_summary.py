"""Summarise scripts/pmc_rescore.sh: k_rescore_ring counters summed over its burst-tick
dispatches (> 50 us), per wave and per chunk-frame.  SQ_* wave counters are quad-cycles."""
import collections, csv, glob, os, sys

d = sys.argv[1]
tot = collections.defaultdict(float)
n_disp = collections.Counter()
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(f)):
        if "k_rescore_ring" not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for i, cs in per.items():
        if dur[i] < 50:
            continue
        n_disp[f] += 1
        tot["dur_us@" + f[-40:]] += dur[i]
        for n, v in cs.items():
            tot[n] += v
print(f"k_rescore_ring burst dispatches per pass: {dict((os.path.basename(os.path.dirname(k)), v) for k, v in n_disp.items())}")
for n in sorted(tot):
    print(f"  {n:40s} {tot[n]:.6g}")
g = tot.get
if g("SQ_WAVE_CYCLES"):
    wc = g("SQ_WAVE_CYCLES")
    for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
        if g(n):
            print(f"  {n} / SQ_WAVE_CYCLES = {g(n) / wc:.3f}")
if g("SQ_INSTS_VALU") and g("SQ_INSTS_LDS"):
    print(f"  LDS instructions per VALU instruction: {g('SQ_INSTS_LDS') / g('SQ_INSTS_VALU'):.3f}")
if g("SQ_LDS_IDX_ACTIVE"):
    print(f"  LDS bank conflict cycles / LDS active cycles = {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
if g("GRBM_GUI_ACTIVE") and g("SQ_LDS_IDX_ACTIVE"):
    # SQ_LDS_IDX_ACTIVE summed over the CUs (per-SE/XCD sums); GRBM_GUI_ACTIVE: GPU busy cycles per XCD
    print(f"  SQ_LDS_IDX_ACTIVE / GRBM_GUI_ACTIVE = {g('SQ_LDS_IDX_ACTIVE') / g('GRBM_GUI_ACTIVE'):.2f}  (divide by CUs per unit of GRBM for a per-CU duty)")
