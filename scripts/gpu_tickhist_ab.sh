#!/bin/bash
# Scorer-launch histograms of the 8,192-stream streaming leg for each variants/*.so
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for f in $R/variants/*.so; do
  n=$(basename $f .so)
  EWK_LIB=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tprof_$n -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
     --no-cpu-baseline --fixed-len 0 --confirm-batch 0 --big-streams 0 --max-streams 0 > $R/gpurun_out/tprof_$n.log 2>&1 || exit $?
  echo "== $n"; python $R/scripts/tick_hist.py $R/gpurun_out/tprof_$n || exit $?
  find $R/gpurun_out/tprof_$n -name "*kernel_trace.csv" -delete
done
