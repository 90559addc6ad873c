#!/bin/bash
# Round 4, ring re-score sessions.  Every step under its own time limit; a heartbeat line
# every 30 s keeps a long test from reading as silent.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04b}
( while true; do sleep 30; echo "[hb $(date +%T)] $(tail -c 200 gpurun_out/${TAG}_cur.log 2>/dev/null | tail -1)"; done ) &
HB=$!
trap "kill $HB" EXIT
MODE=${1:-stream}
if [ "$MODE" = stream ]; then   # the streaming legs only (8,192 and 131,072 streams), kernel times per tick
  timeout -k 10 400 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --fixed-len 0 --short-len 0 \
     --confirm-batch 0 --no-host-ingest --max-streams 0 --big-ticks 100 > gpurun_out/${TAG}_cur.log 2>&1
  rc=$?; cp gpurun_out/${TAG}_cur.log gpurun_out/${TAG}_stream.log; echo "stream bench rc=$rc"
  python scripts/stream_line.py gpurun_out/${TAG}_stream.log 2>/dev/null || tail -c 2000 gpurun_out/${TAG}_stream.log
  exit $rc
fi
if [ "$MODE" = test ]; then   # GPU tests (-k K optional)
  K=${2:-}
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --durations=15 --timeout 400 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${TAG}_cur.log 2>&1
  rc=$?; cp gpurun_out/${TAG}_cur.log gpurun_out/${TAG}_pytest_gpu.log; echo "pytest rc=$rc"; tail -25 gpurun_out/${TAG}_pytest_gpu.log
  exit $rc
fi
if [ "$MODE" = rsprobe ]; then   # per-tick re-score load and time (scripts/rescore_ring_probe.py)
  timeout -k 10 300 python -u scripts/rescore_ring_probe.py ${2:-8192} ${3:-60} > gpurun_out/${TAG}_cur.log 2>&1
  rc=$?; cp gpurun_out/${TAG}_cur.log gpurun_out/${TAG}_rsprobe.log; echo "rsprobe rc=$rc"; tail -50 gpurun_out/${TAG}_rsprobe.log
  exit $rc
fi
if [ "$MODE" = rsvar ]; then   # the re-score probe over the timing variants (scripts/build_rs_variants.py)
  : > gpurun_out/${TAG}_rsvar.log
  for v in ${2:-t12 t8 t12_nodct t12_nomel t12_nolog t12_nofft}; do
    echo "== $v" >> gpurun_out/${TAG}_rsvar.log
    EWK_LIB=$PWD/easywakeword_amd/_var/libewk_$v.so timeout -k 10 300 python -u scripts/rescore_ring_probe.py 8192 60 > gpurun_out/${TAG}_cur.log 2>&1 || exit $?
    grep -E "^  tick|mean:|ticks with" gpurun_out/${TAG}_cur.log >> gpurun_out/${TAG}_rsvar.log
  done
  cat gpurun_out/${TAG}_rsvar.log
  exit 0
fi
if [ "$MODE" = std ]; then   # |mean| / |std| distributions and the fp32-vs-fp64 score error by |mean|, ring path too
  timeout -k 10 600 python -u scripts/std_norm_dist.py > gpurun_out/${TAG}_cur.log 2>&1
  rc=$?; cp gpurun_out/${TAG}_cur.log gpurun_out/${TAG}_std_norm_dist.txt; echo "std rc=$rc"; tail -25 gpurun_out/${TAG}_std_norm_dist.txt
  exit $rc
fi
if [ "$MODE" = bench ]; then   # the default bench line, then its rocprofv3 kernel trace
  timeout -k 10 900 python bench.py --steps 20 --warmup 10 > gpurun_out/${TAG}_cur.log 2>&1
  rc=$?; cp gpurun_out/${TAG}_cur.log gpurun_out/${TAG}_bench.log; echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.log; echo
  [ $rc -eq 0 ] || exit $rc
  python scripts/stream_line.py gpurun_out/${TAG}_bench.log
  R="$PWD"; cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 10 --no-cpu-baseline --fixed-len 0 --short-len 0 > "$R/gpurun_out/${TAG}_cur.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"
  python "$R/scripts/prof_summary.py" "$R/gpurun_out/${TAG}_prof" 10 > "$R/gpurun_out/${TAG}_kernel_stats.txt" 2>&1
  rm -f "$R/gpurun_out/${TAG}_prof/run_kernel_trace.csv"
  head -12 "$R/gpurun_out/${TAG}_kernel_stats.txt"; tail -3 "$R/gpurun_out/${TAG}_kernel_stats.txt"
  exit $rc
fi
if [ "$MODE" = maxstreams ]; then   # the streaming_max leg alone at the default request (HBM-capped)
  timeout -k 10 600 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --fixed-len 0 --short-len 0 \
     --confirm-batch 0 --no-host-ingest --big-streams 0 --stream-ticks 100 > gpurun_out/${TAG}_cur.log 2>&1
  rc=$?; cp gpurun_out/${TAG}_cur.log gpurun_out/${TAG}_maxstreams.log; echo "maxstreams rc=$rc"
  python scripts/stream_line.py gpurun_out/${TAG}_maxstreams.log || tail -c 3000 gpurun_out/${TAG}_maxstreams.log
  exit $rc
fi
if [ "$MODE" = n2 ]; then   # the bench's N > 1 path rehearsed with 2 gloo ranks on the one GPU
  EWK_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
     --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 5 --warmup 2 --big-streams 0 --big-ticks 100 \
     --max-streams 262144 --no-host-ingest --confirm-batch 0 --fixed-len 0 --short-len 0 > gpurun_out/${TAG}_cur.log 2>&1
  rc=$?; cp gpurun_out/${TAG}_cur.log gpurun_out/${TAG}_n2.log; echo "n2 rc=$rc"; grep "^{" gpurun_out/${TAG}_n2.log | tail -1 | head -c 1500
  exit $rc
fi
