#!/bin/bash
# Scorer A/B of variants/*.so (ragged + L = 16000, 3 rounds); score_err guards each variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in variants/*.so; do
  EWK_LIB=$PWD/$f timeout -k 10 180 python scripts/score_err.py 2048 2>&1 | grep segments
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "score_err $f rc=$rc"; exit $rc; }
done
for r in 1 2 3; do
  for L in 0 16000; do
    for f in variants/*.so; do
      EWK_FIXED_LEN=$L EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py 65536 20 2>&1 | grep Gframes
      rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "variant $f rc=$rc"; exit $rc; }
    done
  done
done
