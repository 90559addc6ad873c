#!/bin/bash
# Scorer precision sweep: fuzz_err.py (the top_db fuzz generator) over seeds 1..N, 200 segments each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-12}
for s in $(seq 1 $N); do
  timeout -k 10 400 python scripts/fuzz_err.py $s 200 2>&1 | grep -E "fuzz|DIFFERS"
  rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "seed $s rc=$rc"; exit $rc; }
done
