#!/bin/bash
# The streaming legs' re-score cost for every variants/*.so, interleaved (timing bounds only:
# the -DEWK_RS_SKIP_* builds compute wrong fp64 scores).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do for L in variants/*.so; do
  EWK_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --fixed-len 0 --short-len 0 \
      --confirm-batch 0 --no-host-ingest --max-streams 0 --big-streams 131072 --big-ticks 100 > gpurun_out/abv_$i.log 2>&1 || exit 1
  echo "$(basename $L) $i: $(python scripts/stream_line.py gpurun_out/abv_$i.log | tr '\n' ' ')"
done; done
