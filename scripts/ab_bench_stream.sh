#!/bin/bash
# A/B: bench.py's config-3 streaming line (8,192 streams, 600 timed ticks) and the 131,072-stream
# line for each variants/*.so, interleaved over R rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-2}; BIG=${2:-0}; MAX=${3:-0}
for r in $(seq 1 $R); do
  for f in ${VDIR:-variants}/*.so; do
    echo -n "$(basename $f) "
    EWK_LIB=$PWD/$f timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fixed-len 0 --confirm-batch 0 \
        --big-streams $BIG --max-streams $MAX 2>/dev/null | \
      python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['streaming']
line='8192: %.4f ms/tick (gate %.4f, scorer %.4f, rescore %.4f)' % (s['ms_per_tick'], s['gate_kernel_ms_per_tick'], s['scorer_kernel_ms_per_tick'], s['rescore_kernel_ms_per_tick'])
b=d.get('streaming_f32_max') or d.get('streaming_100k')
if b: line += '; %d: %.4f ms/tick (gate %.4f)' % (b['streams'], b['ms_per_tick'], b['gate_kernel_ms_per_tick'])
m=d.get('streaming_max')
if m: line += '; %d: %.3f ms/tick (gate %.3f)' % (m['streams'], m['ms_per_tick'], m['gate_kernel_ms_per_tick'])
print(line)"
    rc=${PIPESTATUS[0]}
    [ $rc -eq 0 ] || exit $rc
  done
done
