#!/bin/bash
# Interleaved A/B of the streaming legs' re-score cost: variants/rs_base.so (HEAD) vs the
# working tree's libewk.so, twice each, on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do for v in old new; do
  if [ $v = old ]; then L=$PWD/variants/rs_base.so; else L=$PWD/easywakeword_amd/libewk.so; fi
  EWK_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --fixed-len 0 --short-len 0 \
      --confirm-batch 0 --no-host-ingest --max-streams 0 --big-streams 131072 --big-ticks 100 > gpurun_out/abrs_${v}_$i.log 2>&1 || exit 1
  echo "$v $i: $(python scripts/stream_line.py gpurun_out/abrs_${v}_$i.log | tr '\n' ' ')"
done; done
