"""Max |score - oracle| over test_top_db_order_fuzz's 120 segments (same generator, seed
2024) for one libewk.so variant (EWK_LIB): how close a scorer change runs to the 1e-4 bar."""
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
rng = np.random.Generator(np.random.PCG64(2024))
word = synth.load_word()
segs = []
for k in range(120):
    L = int(rng.integers(1, 60001))
    x = (rng.normal(0, 1, L) * 10 ** rng.uniform(-7, -2)).astype(np.float32)
    for _ in range(int(rng.integers(0, 5))):
        n = int(rng.integers(200, 12000))
        s0 = int(rng.integers(0, max(1, L - n)))
        amp = np.float32(10 ** rng.uniform(-5, 0))
        kind = int(rng.integers(0, 3))
        if kind == 0:
            src = word[:n] if n <= len(word) else np.resize(word, n)
        elif kind == 1:
            src = np.sin(2 * np.pi * rng.uniform(100, 7000) * np.arange(n) / 16000).astype(np.float32)
        else:
            src = rng.normal(0, 1, n).astype(np.float32)
        m = min(n, L - s0)
        x[s0:s0 + m] += amp * src[:m]
    if k % 7 == 0 and L > 4000:
        a = int(rng.integers(0, L - 3000))
        x[a:a + 3000] = 0.0
    if k % 11 == 0 and L > 5120:
        x[2560:5120] = x[0:2560]
    segs.append(x)
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
errs.sort(reverse=True)
lib = os.path.basename(os.environ.get("EWK_LIB", "libewk.so"))
print(f"{lib}: fuzz max |dscore| {errs[0][0]:.3e} (case {errs[0][1]}, L={errs[0][2]}, ref {errs[0][3]:.4f}); "
      f"next {errs[1][0]:.3e} {errs[2][0]:.3e}; median {np.median([e[0] for e in errs]):.3e}")
