#!/bin/bash
# A/B: time each variants/*.so on the gate microbenchmark, interleaved over R rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-8192}; R=${2:-2}
for r in $(seq 1 $R); do
  for f in variants/*.so; do
    echo -n "$(basename $f) "
    EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_gate.py $N 200 2>&1 | grep -v amdgpu.ids | tail -2 | tr '\n' ' '
    rc=${PIPESTATUS[0]}; echo
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "variant $f rc=$rc"; exit $rc; fi
  done
done
