"""One-off wide sweep of tests/test_gpu_stream_fuzz.py's random configurations (seeds a..b)."""
import os, sys, traceback
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_stream_fuzz as t
from golden_io import matcher_fixture, template_arrays
a, b = int(sys.argv[1]), int(sys.argv[2])
tmpl = template_arrays(matcher_fixture()[0])
bad = 0
for seed in range(a, b):
    try:
        t.test_random_stream_configs_vs_oracle(seed, tmpl)
        print(seed, "ok", t._case(seed), flush=True)
    except AssertionError as e:
        bad += 1
        print(seed, "FAIL", t._case(seed), str(e)[:400], flush=True)
print("failures", bad)
