#!/bin/bash
# LDS-array utilisation of each variants/*.so (one kernel-trace + pmc pass each).
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
N=${1:-16384}
for f in "$R"/variants/*.so; do
  b=$(basename $f .so)
  EWK_LIB=$f timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
     --output-format csv -d "$R/gpurun_out/lds_$b" -o run -- python3 "$R/scripts/mb_score.py" $N 2 > "$R/gpurun_out/lds_$b.log" 2>&1
  rc=$?; echo "$b rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
