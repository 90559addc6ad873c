#!/bin/bash
# Round-6 GPU session: the certain-NaN evidence, the GPU suite, smoke, bench.  Stops at the
# first GPU fault / timeout (each step under its own limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok_or_testfail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ "${1:-}" = n2 ]; then   # the bench's N > 1 path rehearsed with 2 gloo ranks on the one GPU
  EWK_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
     --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 5 --warmup 2 --big-streams 0 --big-ticks 100 \
     --max-streams 262144 --no-host-ingest --confirm-batch 0 --fixed-len 0 --short-len 0 > gpurun_out/bench_n2_gloo.log 2>&1
  rc=$?; echo "n2 rc=$rc"; grep "^{" gpurun_out/bench_n2_gloo.log | tail -1 | head -c 1500; echo
  exit $rc
fi
timeout -k 10 400 python -u scripts/nan_margin.py ${NAN_N:-3000} > gpurun_out/nan_margin.txt 2>&1
rc=$?; echo "nan_margin rc=$rc"; tail -14 gpurun_out/nan_margin.txt
ok_or_testfail $rc || exit $rc
bash scripts/gpu_round.sh ${1:-test} && bash scripts/gpu_round.sh bench
