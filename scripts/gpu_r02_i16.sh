# int16 rings: parity tests, then the streaming sections of the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_int16_ring.py tests/test_gpu_level3.py tests/test_gpu_compact_ring.py -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_i16.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --fixed-len 0 --confirm-batch 0 > gpurun_out/bench_i16.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_i16.log; exit $rc
