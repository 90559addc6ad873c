set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 scripts/ab.sh 65536 3 > gpurun_out/ab2.log 2>&1 || exit 1
cat gpurun_out/ab2.log
export EWK_RAW=/tmp/ewk_raw_$$
bash scripts/pmc.sh "$PWD/easywakeword_amd/libewk.so" 65536 new "FETCH_SIZE" "WRITE_SIZE" || exit 1
python scripts/pmc_summary.py $EWK_RAW/pmc_new 65536 gpurun_out/traffic_new.json > gpurun_out/pmc_new.txt 2>&1
cat gpurun_out/pmc_new.txt | head -30
