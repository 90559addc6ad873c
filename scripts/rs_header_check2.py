"""Debug: tests/test_gpu_scorer.py's first tests in order on one engine, then the ragged batch,
with the header check library (EWK_LIB, -DEWK_RS_TIMING -DEWK_RS_CHECK)."""
import ctypes, os, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import synth
import test_gpu_scorer as T
from golden_io import matcher_fixture
from easywakeword_amd import Engine
lib = ctypes.CDLL(os.environ["EWK_LIB"])
buf = (ctypes.c_ulonglong * 16)()
e = Engine()
fx = matcher_fixture()
def dbg(tag):
    lib.ewk_debug_rs(buf); d = list(buf)
    print(tag, "chunks", d[1], "finishes", d[3], "serial", d[5], "checked", d[14], "bad", d[15], "claims", d[12], flush=True)
for name, f in [("template", lambda: T.test_template_from_wav_matches_reference(e, fx)),
                ("golden64", lambda: T.test_golden_scores_and_decisions(e, fx, "float64")),
                ("golden32", lambda: T.test_golden_scores_and_decisions(e, fx, "float32")),
                ("fp64api", lambda: T.test_fp64_path_matches_float64_reference_tightly(e, fx)),
                ("ragged", lambda: T.test_random_ragged_batch_vs_oracle(e))]:
    try:
        f(); print(name, "ok")
    except AssertionError as ex:
        print(name, "FAIL", str(ex)[:300])
    dbg(name)
