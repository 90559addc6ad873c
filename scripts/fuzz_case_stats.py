"""Features of the worst fuzz_err.py cases: T, |mean|, |std|, clamped fraction, the fp32
mean/std errors against the oracle -- what the fp64 re-score criterion should catch.
Usage: python scripts/fuzz_case_stats.py seed:case[:gain] ... (n = 200 segments per seed)"""
import math, os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth
from oracle import mfcc_ref
import easywakeword_amd as ewa


word = synth.load_word()
e = ewa.Engine()
e.template_from_pcm(word)
tm, ts = e.get_template()
cache = {}
for arg in sys.argv[1:]:
    parts = arg.split(":")
    seed, case = int(parts[0]), int(parts[1])
    gain = float(parts[2]) if len(parts) > 2 else 1.0
    if seed not in cache:
        cache[seed] = synth.fuzz_segments(seed, 200, word)
    x = (cache[seed][case] * np.float32(gain)).astype(np.float32)
    m32, s32, sc, _ = e.score([x], candidate_dtype="float64")
    lm = mfcc_ref.log_mel(x.astype(np.float64))
    cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64))
    ref = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
    T = lm.shape[1]
    thr = lm.max() - 80.0
    clamped = float(np.mean(lm <= thr + 1e-9))
    print(f"seed {seed} case {case} gain {gain:g}: score {sc[0]:.6f} ref {ref:.6f} L={len(x)} T={T} d={abs(sc[0]-ref):.2e} |mean|={np.linalg.norm(cm):.1f} "
          f"|std|={np.linalg.norm(cs):.2f} min|std_k|={np.min(np.abs(cs)):.3f} clamped={clamped:.3f} "
          f"dmean={np.max(np.abs(m32[0]-cm)):.2e} dstd={np.max(np.abs(s32[0]-cs)):.2e} "
          f"dstd_rel={np.max(np.abs(s32[0]-cs)/np.maximum(1e-3,np.abs(cs))):.2e}")
