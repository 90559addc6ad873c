"""Re-create tests/test_gpu_scorer.py::test_top_db_order_fuzz segments and print the scorer vs
the oracle for the first N (debug helper; EWK_LIB selects a libewk variant)."""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth
from oracle import mfcc_ref


def segments(n_take):
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
    return segs[:n_take]


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    segs = segments(120)[:n]
    if os.environ.get("CPU_ONLY"):
        for i, x in enumerate(segs):
            S = mfcc_ref.log_mel(x.astype(np.float64))
            print(i, len(x), "max %.2f min %.2f" % (S.max(), S.min()))
        sys.exit(0)
    import easywakeword_amd as ewa
    e = ewa.Engine()
    e.template_from_pcm(synth.load_word())
    tm, ts = e.get_template()
    dt = os.environ.get("FUZZ_DTYPE", "float64")
    mean, std, score, match = e.score(segs, candidate_dtype=dt)
    for i, x in enumerate(segs):
        cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64) if dt == "float64" else x.astype(np.float32))
        ref = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
        bad = not (abs(score[i] - ref) < 1e-4 or (np.isnan(score[i]) and np.isnan(ref)))
        print(i, len(x), "gpu %.6f ref %.6f %s" % (score[i], ref, "BAD" if bad else ""),
              "mean0 %.4f/%.4f std0 %.4f/%.4f" % (mean[i][0], cm[0], std[i][0], cs[0]))
