"""Debug: the claim-ahead patch's part-record headers against the slot / event they copy
(libewk built with -DEWK_RS_TIMING -DEWK_RS_CHECK, via EWK_LIB)."""
import ctypes, os, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import synth
from oracle import mfcc_ref
from easywakeword_amd import Engine
lib = ctypes.CDLL(os.environ["EWK_LIB"])
buf = (ctypes.c_ulonglong * 16)()
e = Engine()
word = synth.load_word()
e.template_from_pcm(word)
tm, ts = e.get_template()
lib.ewk_debug_rs(buf)
segs = synth.ragged_segments(4321, 200, 160, 48000)
_, _, score, match = e.score(segs, candidate_dtype="float64")
lib.ewk_debug_rs(buf)
d = list(buf)
print("chunks", d[1], "finishes", d[3], "serial", d[5], "checked", d[14], "bad", d[15], "bad bits", bin(d[13]), "claims", d[12])
bad = []
for i, x in enumerate(segs):
    cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64))
    ref = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
    if not (abs(score[i] - ref) <= 1e-4 or (np.isnan(ref) and np.isnan(score[i]))):
        bad.append((i, len(x), 1 + len(x) // 160, score[i], ref))
print("wrong scores:", bad)
