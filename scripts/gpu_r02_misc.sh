set -o pipefail
mkdir -p gpurun_out
( nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>&1; cat /proc/self/status | grep -i cpus_allowed_list ) > gpurun_out/cores_probe.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_gate.py -v -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_runtime.log 2>&1 && \
EWK_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --big-streams 65536 --max-streams 0 --big-ticks 100 --stream-ticks 200 --confirm-batch 0 > gpurun_out/bench_n2_gloo.log 2>&1
