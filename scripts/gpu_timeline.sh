#!/bin/bash
# rocprofv3 kernel trace of the 8,192-stream streaming leg: per-tick kernel/gap timeline + scorer histogram
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tprof -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
   --no-cpu-baseline --fixed-len 0 --confirm-batch 0 --big-streams 0 --max-streams 0 > $R/gpurun_out/tprof.log 2>&1 || exit $?
python $R/scripts/tick_hist.py $R/gpurun_out/tprof > $R/gpurun_out/tick_hist.txt && echo '-- timed ticks (no event records):' >> $R/gpurun_out/tick_hist.txt && python $R/scripts/tick_timeline.py $R/gpurun_out/tprof 12 420 >> $R/gpurun_out/tick_hist.txt && echo '-- instrumented ticks (event records around each kernel):' >> $R/gpurun_out/tick_hist.txt && python $R/scripts/tick_timeline.py $R/gpurun_out/tprof 6 >> $R/gpurun_out/tick_hist.txt
rc=$?
find $R/gpurun_out/tprof -name "*kernel_trace.csv" -delete
cat $R/gpurun_out/tick_hist.txt
exit $rc
