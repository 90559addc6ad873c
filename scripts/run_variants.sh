#!/bin/bash
# time every variants/*.so on the scorer microbenchmark (one process each, bounded)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-16384}
for f in variants/*.so; do
  EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py $N 5 2>&1 | grep -v amdgpu.ids | tail -2
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "variant $f rc=$rc"; exit $rc; fi
done
