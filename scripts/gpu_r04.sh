#!/bin/bash
# Round 4 GPU sessions.  Stops at the first GPU fault/timeout.
#   test [K]   : GPU tests (-k K optional) + smoke
#   bench      : default bench line
#   stream     : the 8,192-stream tick (mb_stream.py) and the tick histogram
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MODE=${1:-test}
TAG=${TAG:-r04}
ok_or_testfail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ "$MODE" = test ]; then
  K=${2:+-k $2}
  timeout -k 10 1100 python -u -m pytest tests -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread $K > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/${TAG}_pytest_gpu.log
  ok_or_testfail $rc || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${TAG}_smoke.log
  exit $rc
fi
if [ "$MODE" = bench ]; then
  timeout -k 10 900 python bench.py --steps 20 --warmup 10 > gpurun_out/${TAG}_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/${TAG}_bench.log
  exit $rc
fi
if [ "$MODE" = ab ]; then   # interleaved A/B of variants/*.so: ragged, L = 16000, L = 6400
  R=${2:-2}
  for L in 0 16000 6400; do
    for r in $(seq 1 $R); do
      for f in variants/*.so; do
        EWK_FIXED_LEN=$L EWK_LIB=$PWD/$f timeout -k 10 120 python scripts/mb_score.py 65536 10 2>&1 | grep Gframes
        rc=${PIPESTATUS[0]}
        if [ $rc -ne 0 ]; then echo "variant $f rc=$rc"; exit $rc; fi
      done
    done
  done | tee gpurun_out/${TAG}_ab.txt
  exit ${PIPESTATUS[0]}
fi
if [ "$MODE" = probe ]; then
  timeout -k 5 60 ./scripts/probes/buffer_lds_probe 2>&1 | tee gpurun_out/${TAG}_buffer_lds_probe.txt
  exit ${PIPESTATUS[0]}
fi
if [ "$MODE" = varcheck ]; then   # parity subset on a variant: EWK_LIB=variants/<v>.so
  V=${2:-variants/b_prefetch_dma.so}
  EWK_LIB=$PWD/$V timeout -k 10 900 python -u -m pytest tests/test_gpu_scorer.py tests/test_gpu_many_streams.py tests/test_gpu_vanishing_mean.py -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_varcheck.log 2>&1
  rc=$?; echo "varcheck $V rc=$rc"; tail -5 gpurun_out/${TAG}_varcheck.log
  exit $rc
fi
