# the session's earlier GPU tests, then scripts/diag_many_streams_loop.py in the same pytest process
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-x}
shift
PRE="$*"
[ -n "$PRE" ] || PRE="tests/test_gpu_c_host.py tests/test_gpu_compact_ring.py tests/test_gpu_config4_shards.py tests/test_gpu_confirm.py tests/test_gpu_fullsize.py tests/test_gpu_gate.py"
EWK_DIAG_TAG=$TAG timeout -k 10 600 python -u -m pytest -q -s -p no:cacheprovider --timeout 500 --timeout-method thread \
  $PRE scripts/diag_many_streams_loop.py > gpurun_out/diag_$TAG.log 2>&1
rc=$?
echo "diag $TAG rc=$rc: $(grep '\[diag\]' gpurun_out/diag_$TAG.log | cut -c1-300) $(tail -1 gpurun_out/diag_$TAG.log)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
