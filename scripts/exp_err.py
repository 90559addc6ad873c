import sys, os, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import synth, easywakeword_amd as ewa
e = ewa.Engine()
e.template_from_pcm(synth.load_word())
rng = np.random.default_rng(0)
rows = []
segs = []; meta = []
for L in [160, 320, 480, 800, 1600, 3200, 6400, 16000, 48000]:
    for f in [50, 300, 1000, 2546, 4000, 7000, 7900]:
        for amp in [0.01, 0.5]:
            t = np.arange(L)/16000
            segs.append((amp*np.sin(2*np.pi*f*t)).astype(np.float32)); meta.append(("tone", L, f, amp))
    for sig in [0, 1e-5, 1e-4]:
        w = synth.load_word()[:L] * 1.0
        segs.append((w + rng.normal(0, sig, len(w))).astype(np.float32) if sig else w.astype(np.float32)); meta.append(("word", L, sig, 0))
_, _, s32, _ = e.score(segs, candidate_dtype="float64")
_, _, s64 = e.score_f64(segs)
d = np.abs(s32 - s64)
order = np.argsort(-np.nan_to_num(d))
for i in order[:25]:
    print(meta[i], round(float(s32[i]),6), round(float(s64[i]),6), d[i])
print("n>1e-4:", int(np.sum(d > 1e-4)), "of", len(d), "n>3e-5:", int(np.sum(d>3e-5)))
