#!/bin/bash
# A/B: time each variants/*.so on the scorer microbenchmark, interleaved over R rounds (box noise)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-65536}; R=${2:-2}
for r in $(seq 1 $R); do
  for f in variants/*.so; do
    EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py $N 10 2>&1 | grep -v amdgpu.ids | grep Gframes
    rc=${PIPESTATUS[0]}
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "variant $f rc=$rc"; exit $rc; fi
  done
done
