#!/bin/bash
# Per variants/*.so: fp32-vs-fp64 score error of streaming segments by |mean|, then the
# streaming bench A/B and the batch scorer timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in variants/*.so; do
  echo "== $(basename $f)"
  EWK_LIB=$PWD/$f timeout -k 10 300 python scripts/std_norm_dist.py 2>&1 | grep -E "^streaming \||NaN"
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
done
bash scripts/ab_bench_stream.sh 2 || exit $?
for r in 1 2; do
  for f in variants/*.so; do
    EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py 65536 20 2>&1 | grep Gframes
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
  done
done
