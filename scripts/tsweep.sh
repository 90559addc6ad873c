#!/bin/bash
# T-sweep of the batch scorer: 65,536 fixed-length segments per launch for several L,
# kernel ms per launch (HIP events) -> per-segment fixed cost a + b*T fit (tsweep_fit.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${N:-65536}
for L in ${LENS:-3200 6400 12800 16000 33600 48000}; do
  EWK_FIXED_LEN=$L timeout -k 10 180 python scripts/mb_score.py $N 10 2>&1 | grep -v amdgpu.ids | grep Gframes
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "L=$L rc=$rc"; exit $rc; }
done
timeout -k 10 180 python scripts/mb_score.py $N 10 2>&1 | grep -v amdgpu.ids | grep Gframes
