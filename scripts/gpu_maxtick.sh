#!/bin/bash
# rocprofv3 kernel trace of the bench's streaming_max leg (2.69 M int16 streams): which launch
# makes the slowest ticks (scripts/tick_slowest.py).
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/mprof -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
   --no-cpu-baseline --fixed-len 0 --short-len 0 --confirm-batch 0 --big-streams 0 --no-host-ingest > $R/gpurun_out/mprof.log 2>&1
rc=$?
[ $rc -eq 0 ] && python $R/scripts/tick_slowest.py $R/gpurun_out/mprof "k_score_f32<2, 1>" 20 4 300 > $R/gpurun_out/maxtick.txt 2>&1
cat $R/gpurun_out/maxtick.txt
exit $rc
