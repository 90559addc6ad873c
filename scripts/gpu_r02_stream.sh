# streaming scale check: many-stream parity test + the big streaming runs of the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_many_streams.py tests/test_gpu_gate.py -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_stream.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --fixed-len 0 --confirm-batch 0 > gpurun_out/bench_stream.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_stream.log; exit $rc
