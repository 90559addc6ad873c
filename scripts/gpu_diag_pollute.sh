cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for k in 0 1 2 3; do
  EWK_DIAG_K=8 EWK_DIAG_POLLUTE=$k EWK_DIAG_TAG=pol$k timeout -k 10 300 python -u -m pytest -q -s -p no:cacheprovider --timeout 250 --timeout-method thread scripts/diag_many_streams_loop.py > gpurun_out/diag_pol$k.log 2>&1
  rc=$?
  echo "pollute $k rc=$rc: $(grep '\[diag\]' gpurun_out/diag_pol$k.log | cut -c1-400)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
