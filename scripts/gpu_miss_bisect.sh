# Which earlier test sets up the ring-path miss?  Each group of test files runs N times in its own
# pytest process, followed by test_many_streams_vs_oracle (rc 1 = the miss, recorded by evidence.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-5}
T=tests/test_gpu_gate.py::test_many_streams_vs_oracle
run_group() {
  local tag=$1; shift
  for i in $(seq 1 $N); do
    timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 250 --timeout-method thread "$@" $T > gpurun_out/bisect_${tag}_$i.log 2>&1
    rc=$?
    echo "$tag $i rc=$rc: $(tail -1 gpurun_out/bisect_${tag}_$i.log)"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || return $rc
  done
}
run_group fullsize tests/test_gpu_fullsize.py || exit $?
run_group config4 tests/test_gpu_config4_shards.py || exit $?
run_group small tests/test_gpu_c_host.py tests/test_gpu_compact_ring.py tests/test_gpu_confirm.py || exit $?
