#!/bin/bash
# Round-3 GPU session: full GPU tests, then the interleaved scorer A/B of variants/*.so
# (mb_score on the bench's ragged batch and on L = 16000), then the phase timing build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  timeout -k 10 900 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = ab ] || [ "$MODE" = abt ]; then
  for r in 1 2; do
    for L in 0 16000; do
      for f in variants/*.so; do
        EWK_FIXED_LEN=$L EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py 65536 10 2>&1 | grep Gframes
        rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "variant $f rc=$rc"; exit $rc; }
      done
    done
  done
fi
if [ "$MODE" = all ] || [ "$MODE" = timing ] || [ "$MODE" = abt ]; then
  bash scripts/gpu_timing.sh
fi
