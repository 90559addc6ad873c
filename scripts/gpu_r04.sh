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
