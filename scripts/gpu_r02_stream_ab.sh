#!/bin/bash
# GPU tests (optional subset), streaming tick A/B over variants/*.so, and the per-tick timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${1:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 scripts/ab_stream.sh 8192 ${2:-3} > gpurun_out/ab_stream.log 2>&1 || { cat gpurun_out/ab_stream.log; exit 1; }
cat gpurun_out/ab_stream.log
timeout -k 10 400 bash scripts/tl.sh > gpurun_out/tl.txt 2>&1 || { tail gpurun_out/tl.txt; exit 1; }
cat gpurun_out/tl.txt
