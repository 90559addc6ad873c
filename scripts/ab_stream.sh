#!/bin/bash
# A/B: the streaming tick (config 3) of each variants/*.so, interleaved over R rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-8192}; R=${2:-2}
for r in $(seq 1 $R); do
  for f in variants/*.so; do
    echo -n "$(basename $f) "
    MB_PROFILE=0 EWK_LIB=$PWD/$f timeout -k 10 200 python scripts/mb_stream.py 400 $N 2>&1 | grep -v amdgpu.ids | tail -1
    rc=${PIPESTATUS[0]}
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "variant $f rc=$rc"; exit $rc; fi
  done
done
