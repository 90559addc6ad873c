#!/bin/bash
# Round-3 (second session): GPU tests on the in-tree build, fp32-vs-fp64 precision of
# variants/b_all.so and a_base.so, then the interleaved scorer A/B of variants/*.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = prec ]; then
  for f in variants/a_base.so variants/b_all.so; do
    EWK_LIB=$PWD/$f timeout -k 10 180 python scripts/score_err.py 8192 2>&1 | grep segments
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "score_err $f rc=$rc"; exit $rc; }
  done
fi
if [ "$MODE" = all ] || [ "$MODE" = ab ]; then
  for r in 1 2 3; do
    for L in 0 16000; do
      for f in variants/*.so; do
        EWK_FIXED_LEN=$L EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py 65536 10 2>&1 | grep Gframes
        rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "variant $f rc=$rc"; exit $rc; }
      done
    done
  done
fi
