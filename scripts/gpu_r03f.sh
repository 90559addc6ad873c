#!/bin/bash
# Per variants/*.so: worst fuzz cases' mean/std errors, fuzz sweeps at gains 1 and 1000, timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in variants/*.so; do
  EWK_LIB=$PWD/$f timeout -k 10 300 python scripts/fuzz_case_stats.py 33:187:1000 31:113:1000 31:113:1 33:187:1 2>&1 | grep seed | sed "s|^|$(basename $f) |"
  for g in 1 1000; do for s in 31 33; do
    EWK_LIB=$PWD/$f timeout -k 10 300 python scripts/fuzz_err.py $s 200 $g 2>&1 | grep -E "fuzz|DIFFERS"
  done; done
  EWK_LIB=$PWD/$f timeout -k 10 180 python scripts/score_err.py 8192 2>&1 | grep segments
done
for r in 1 2 3; do
  for L in 0 16000; do
    for f in variants/*.so; do
      EWK_FIXED_LEN=$L EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py 65536 20 2>&1 | grep Gframes
      rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "variant $f rc=$rc"; exit $rc; }
    done
  done
done
