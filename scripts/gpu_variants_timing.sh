#!/bin/bash
# Timing-build variants (variants/*.so built with -DEWK_TIMING=1): kernel time and the
# per-phase / frame-pass sub-phase cycles of each, on the bench's ragged batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for f in variants/*.so; do
    EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py 65536 10 2>&1 | grep -v amdgpu.ids
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "variant $f rc=$rc"; exit $rc; }
  done
done
