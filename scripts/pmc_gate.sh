#!/bin/bash
# PMC passes over the streaming bench (k_gate_ticks / ring-mode scorer), kernel-trace only.
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
RAW="${EWK_RAW:-$R/gpurun_out}"   # raw rocprofv3 output (large); summaries go to gpurun_out
TAG=${1:-gate}
shift
EXTRA=${EWK_PMC_BENCH_ARGS:---big-streams 0 --max-streams 0}   # default: the 8,192-stream config only
mkdir -p "$RAW/pmc_$TAG"
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$RAW/pmc_$TAG/p$i" -o run -- \
     python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --confirm-batch 0 --fixed-len 0 --stream-ticks 200 $EXTRA \
     > "$RAW/pmc_$TAG/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$RAW/pmc_$TAG/p$i.log"; exit $rc; }
done
