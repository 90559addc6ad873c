# GPU tests ending in test_gpu_gate.py::test_many_streams_vs_oracle, N times (a wrong score is rc 1 and
# recorded by tests/evidence.py; any other failure code ends the script).
#   bash scripts/gpu_miss_prefix.sh N [test files ...]   (default: the files that precede it in a session)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-4}
shift
FILES="$*"
[ -n "$FILES" ] || FILES="tests/test_gpu_c_host.py tests/test_gpu_compact_ring.py tests/test_gpu_config4_shards.py tests/test_gpu_confirm.py tests/test_gpu_fullsize.py tests/test_gpu_gate.py"
for i in $(seq 1 $N); do
  timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread $FILES > gpurun_out/prefix_$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc: $(tail -1 gpurun_out/prefix_$i.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
