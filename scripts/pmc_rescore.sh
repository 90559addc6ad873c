#!/bin/bash
# PMC passes over the re-score probe (scripts/rescore_ring_probe.py, the 8,192-stream recipe):
# k_rescore_ring's counters on its burst ticks.  One kernel-trace + pmc pass per counter set.
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-rs}
mkdir -p "$R/gpurun_out/pmc_$TAG"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/pmc_$TAG/p$i" -o run -- \
     python3 "$R/scripts/rescore_ring_probe.py" 8192 60 > "$R/gpurun_out/pmc_$TAG/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/pmc_$TAG/p$i.log"; exit $rc; }
done
python3 "$R/scripts/pmc_rescore_summary.py" "$R/gpurun_out/pmc_$TAG" > "$R/gpurun_out/pmc_${TAG}_summary.txt" 2>&1
cat "$R/gpurun_out/pmc_${TAG}_summary.txt"
rm -f "$R"/gpurun_out/pmc_$TAG/p*/run_kernel_trace.csv
