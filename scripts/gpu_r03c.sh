#!/bin/bash
# Per variants/*.so: max error over the top_db fuzz segments, and score_err on the bench batch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in variants/*.so; do
  EWK_LIB=$PWD/$f timeout -k 10 240 python scripts/fuzz_err.py 2>&1 | grep fuzz
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "fuzz_err $f rc=$rc"; exit $rc; }
  EWK_LIB=$PWD/$f timeout -k 10 180 python scripts/score_err.py 8192 2>&1 | grep segments
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "score_err $f rc=$rc"; exit $rc; }
done
