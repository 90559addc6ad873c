#!/bin/bash
# Wave-cycle breakdown (parked / issue-stalled / active) of each variants/*.so at one size:
#   scripts/pmc_stall.sh [n_segments] [counter ...]   (one kernel-trace + pmc pass per variant)
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
N=${1:-65536}; shift
CTRS=${*:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE}
for f in "$R"/variants/*.so; do
  b=$(basename $f .so)
  EWK_LIB=$f timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS \
     --output-format csv -d "$R/gpurun_out/stall_$b" -o run -- python3 "$R/scripts/mb_score.py" $N 2 > "$R/gpurun_out/stall_$b.log" 2>&1
  rc=$?; echo "$b rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
