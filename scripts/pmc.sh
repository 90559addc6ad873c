#!/bin/bash
# PMC passes over the scorer microbenchmark (kernel-trace only; no sys/runtime trace).
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
RAW="${EWK_RAW:-$R/gpurun_out}"   # raw rocprofv3 output (large); summaries go to gpurun_out
LIB=${1:-$R/easywakeword_amd/libewk.so}
N=${2:-16384}
TAG=${3:-base}
mkdir -p "$RAW/pmc_$TAG"
i=0
shift 3
for set in "$@"; do
  i=$((i+1))
  EWK_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$RAW/pmc_$TAG/p$i" -o run -- python3 "$R/scripts/mb_score.py" $N 2 > "$RAW/pmc_$TAG/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$RAW/pmc_$TAG/p$i.log"; exit $rc; }
done
