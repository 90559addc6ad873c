"""Timing variants of the fp64 re-score (-DEWK_RS_TIMING counters plus phase switches that
skip work: wrong scores, timing only) built in parallel into easywakeword_amd/_var/."""
import os, sys
from concurrent.futures import ThreadPoolExecutor
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easywakeword_amd import build

VARIANTS = {
    "t12": ["EWK_RS_TIMING"],
    "t8": ["EWK_RS_TIMING", "EWK_RS_NW=8"],
    "t12_nodct": ["EWK_RS_TIMING", "EWK_RS_SKIP_DCT"],
    "t12_nomel": ["EWK_RS_TIMING", "EWK_RS_SKIP_MEL"],
    "t12_nolog": ["EWK_RS_TIMING", "EWK_RS_SKIP_LOG"],
    "t12_nofft": ["EWK_RS_TIMING", "EWK_RS_SKIP_FFT"],
}
sel = sys.argv[1:] or list(VARIANTS)
out = os.path.join(build.HERE, "_var")
os.makedirs(out, exist_ok=True)
with ThreadPoolExecutor(4) as ex:
    for r in ex.map(lambda k: build.build(out=os.path.join(out, f"libewk_{k}.so"), defines=VARIANTS[k]), sel):
        print(r)
