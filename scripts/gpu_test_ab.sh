#!/bin/bash
# GPU tests on the in-tree build, then the streaming A/B of abv/*.so (2 rounds, 8,192 / 131,072 / 2 M streams)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu3.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu3.log; [ $rc -eq 0 ] || exit $rc
VDIR=abv bash scripts/ab_bench_stream.sh 2 131072 2097152
