# fp64 re-score window: theta gap / recompute counters (timing build) and the new test
set -o pipefail
V=$PWD/variants
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rescore_window.py > gpurun_out/rsw_test.log 2>&1
