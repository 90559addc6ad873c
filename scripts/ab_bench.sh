#!/bin/bash
# A/B: the bench's batch-scorer step (wall clock, value) for each variants/*.so, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-2}
for r in $(seq 1 $R); do
  for f in variants/*.so; do
    echo -n "$(basename $f) "
    EWK_LIB=$PWD/$f timeout -k 10 300 python bench.py --no-streaming --no-cpu-baseline --fixed-len 0 --confirm-batch 0 2>/dev/null | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g G frames/s, ms/step %.4f, kernel %.4f' % (d['value']/1e9, d['ms_per_step'], d['roofline']['kernel_ms']))"
    rc=${PIPESTATUS[0]}
    [ $rc -eq 0 ] || exit $rc
  done
done
