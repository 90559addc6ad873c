# GPU timeline of the bench's streaming ticks (config 3) under rocprofv3 --kernel-trace
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT}"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tl" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --confirm-batch 0 --fixed-len 0 --stream-ticks 300 --big-streams 0 --max-streams 0 > "$R/gpurun_out/tl.log" 2>&1 && python3 "$R/scripts/tick_timeline.py" "$R/gpurun_out/tl" 12
