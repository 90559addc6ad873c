"""Max |score - oracle| over test_top_db_order_fuzz's segments (same generator; default seed
2024 and 120 segments, the test's) for one libewk.so variant (EWK_LIB): how close a scorer
change runs to the 1e-4 bar.  Usage: python scripts/fuzz_err.py [seed] [n_segments] [gain]
(gain scales every segment: un-normalised float audio, e.g. int16-range samples)"""
import math, os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth
from oracle import mfcc_ref
import easywakeword_amd as ewa

e = ewa.Engine()
e.template_from_pcm(synth.load_word())
tm, ts = e.get_template()
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 2024
n_seg = int(sys.argv[2]) if len(sys.argv) > 2 else 120
gain = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
segs = [(x * np.float32(gain)).astype(np.float32) for x in synth.fuzz_segments(seed, n_seg, synth.load_word())]
_, _, score, match = e.score(segs, candidate_dtype="float64")
errs = []
for i, x in enumerate(segs):
    if np.ptp(mfcc_ref.log_mel(x.astype(np.float64))) == 0.0:
        continue
    cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64))
    ref = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
    if math.isnan(ref) and math.isnan(score[i]):
        continue
    errs.append((abs(score[i] - ref), i, len(x), ref))
    if bool(match[i]) != (ref >= 75.0):
        print(f"DECISION DIFFERS: seed {seed} case {i} L={len(x)} score {score[i]!r} ref {ref!r}")
errs.sort(reverse=True)
lib = os.path.basename(os.environ.get("EWK_LIB", "libewk.so"))
print(f"{lib} seed {seed} n {n_seg} gain {gain:g}: fuzz max |dscore| {errs[0][0]:.3e} (case {errs[0][1]}, L={errs[0][2]}, ref {errs[0][3]:.4f}); "
      f"next {errs[1][0]:.3e} {errs[2][0]:.3e}; median {np.median([e[0] for e in errs]):.3e}")
