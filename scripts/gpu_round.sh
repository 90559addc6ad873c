#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof.  Stops at the first GPU fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MODE=${1:-all}
export EWK_RAW=${EWK_RAW:-/tmp/ewk_raw_$$}   # raw PMC csvs stay on the box (gpurun_out is capped at 64 MiB)
ok_or_testfail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
  ok_or_testfail $rc || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
  ok_or_testfail $rc || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 10 > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  cd /tmp && export TMPDIR=/tmp
  R="${GRAFT_REPO_ROOT:-/root/repo}"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 10 --no-cpu-baseline --fixed-len 0 > "$R/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -5 "$R/gpurun_out/prof.log"
  python "$R/scripts/prof_summary.py" "$R/gpurun_out/prof" 10 20 > "$R/gpurun_out/kernel_stats.txt" 2>&1
  rm -f "$R/gpurun_out/prof/run_kernel_trace.csv"   # large; the stats csv and the summary stay
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
  R="${GRAFT_REPO_ROOT:-/root/repo}"
  bash "$R/scripts/pmc.sh" "$R/easywakeword_amd/libewk.so" 65536 bench "FETCH_SIZE" "WRITE_SIZE" \
     "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
     "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
     "SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python "$R/scripts/pmc_summary.py" "${EWK_RAW:-$R/gpurun_out}/pmc_bench" 65536 "$R/gpurun_out/traffic_k_score_f32.json" \
     > "$R/gpurun_out/pmc_summary.txt" 2>&1
fi
if [ "$MODE" = all ] || [ "$MODE" = pmcgate ]; then
  R="${GRAFT_REPO_ROOT:-/root/repo}"
  bash "$R/scripts/pmc_gate.sh" gate "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
     "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"
  rc=$?; echo "pmc gate rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python "$R/scripts/pmc_gate_summary.py" "${EWK_RAW:-$R/gpurun_out}/pmc_gate" 8192 > "$R/gpurun_out/pmc_gate_summary.txt" 2>&1
fi
if [ "$MODE" = pmcgatemax ]; then   # the 2,097,152-stream int16 config (the bench's streaming_max)
  R="${GRAFT_REPO_ROOT:-/root/repo}"
  EWK_PMC_BENCH_ARGS="--big-streams 0 --stream-count 64" bash "$R/scripts/pmc_gate.sh" gatemax \
     "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
     "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"
  rc=$?; echo "pmc gate max rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python "$R/scripts/pmc_gate_summary.py" "${EWK_RAW:-$R/gpurun_out}/pmc_gatemax" 2097152 > "$R/gpurun_out/pmc_gatemax_summary.txt" 2>&1
fi
