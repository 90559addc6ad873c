#!/bin/bash
# Round-6 GPU session: the certain-NaN evidence, the GPU suite, smoke, bench.  Stops at the
# first GPU fault / timeout (each step under its own limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok_or_testfail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 400 python -u scripts/nan_margin.py ${NAN_N:-3000} > gpurun_out/nan_margin.txt 2>&1
rc=$?; echo "nan_margin rc=$rc"; tail -14 gpurun_out/nan_margin.txt
ok_or_testfail $rc || exit $rc
bash scripts/gpu_round.sh ${1:-test} && bash scripts/gpu_round.sh bench
