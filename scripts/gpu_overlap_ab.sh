#!/bin/bash
# A/B of the 8,192-stream tick with the scorer on the engine stream vs overlapped with the next gate
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for ov in 0 1; do
    echo -n "overlap=$ov: "
    EWK_SCORE_OVERLAP=$ov timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fixed-len 0 --confirm-batch 0 \
        --big-streams 0 --max-streams 0 2>/dev/null | grep "^{" | python scripts/stream_line.py
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
  done
done
