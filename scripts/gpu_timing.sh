#!/bin/bash
# Per-phase cycle split of the batch scorer (debug build easywakeword_amd/libewk_timing.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in ${LENS:-0 16000 3200}; do
  EWK_FIXED_LEN=$L EWK_LIB=$PWD/easywakeword_amd/libewk_timing.so timeout -k 10 180 python scripts/mb_score.py 65536 10 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "L=$L rc=$rc"; exit $rc; }
done
