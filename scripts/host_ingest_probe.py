"""Where do the host-ingest leg's slow ticks come from?  (GPU box; diagnostic.)

    python scripts/host_ingest_probe.py [streams] [ticks]

Runs bench.streaming_host_bench's loop (1,048,576 int16 streams by default: 3.36 GB of PCM per
tick from pinned host memory, double-buffered copy stream, then push) and prints every timed
tick's own H2D copy time and kernel time, the slowest ticks, and the copy engine the runtime
used (run it under `rocprofv3 --kernel-trace --memory-copy-trace` to see blit kernels vs DMA).
"""
import os
import sys

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import easywakeword_amd as ewa
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda", 0)
    word = bench.load_word()
    prefill = 100
    sig = bench.make_shifted_signal(torch, dev, n, prefill + ticks + 1, 47, word, pcm16=True)
    host = torch.empty(sig.numel(), dtype=sig.dtype, pin_memory=True)
    host.copy_(sig)
    del sig
    torch.cuda.empty_cache()
    se = ewa.StreamEngine(n, ring_samples=48000, ring_format=1)
    se.template_from_pcm(word)
    per = n * 1600
    stage = [torch.empty(per, dtype=host.dtype, device=dev) for _ in range(2)]
    cs = torch.cuda.Stream(dev)
    es_ = torch.cuda.ExternalStream(se.stream_handle(), device=dev)
    free = [torch.cuda.Event() for _ in range(2)]
    used = [False, False]
    cev, comp = {}, {}

    def copy(t):
        b = t % 2
        with torch.cuda.stream(cs):
            if used[b]:
                cs.wait_event(free[b])
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c0.record(cs)
            stage[b].copy_(host[t * 1600: t * 1600 + per], non_blocking=True)
            c1.record(cs)
            cev[t] = (c0, c1)

    def run(t0, nt, timed):
        copy(t0)
        for t in range(t0, t0 + nt):
            b = t % 2
            if t + 1 < t0 + nt:
                copy(t + 1)
            es_.wait_event(cev[t][1])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(es_)
            se.push_device_pcm16(stage[b].data_ptr(), 1600, 0, 1)
            e1.record(es_)
            comp[t] = (e0, e1)
            free[b].record(es_)
            used[b] = True
            se.poll(lagged=True)
        se.poll()

    run(0, prefill, False)
    torch.cuda.synchronize()
    run(prefill, ticks, True)
    torch.cuda.synchronize()
    rows = []
    for t in range(prefill, prefill + ticks):
        c = cev[t][0].elapsed_time(cev[t][1])
        k = comp[t][0].elapsed_time(comp[t][1])
        # the copy's start relative to the previous tick's kernels' end: overlap with compute
        ov = comp[t - 1][1].elapsed_time(cev[t][0]) if t - 1 in comp else float("nan")
        rows.append((t, c, k, c + k, ov))
    a = np.array(rows)
    print(f"{n} streams, {ticks} ticks: copy ms p50 {np.median(a[:, 1]):.2f} max {a[:, 1].max():.2f}; "
          f"kernels ms p50 {np.median(a[:, 2]):.2f} max {a[:, 2].max():.2f}; copy+kernels max {a[:, 3].max():.2f}")
    print("slowest ticks (tick, copy ms, kernels ms, sum, copy start - previous tick's kernel end ms):")
    for r in sorted(rows, key=lambda r: -r[3])[:12]:
        print("  %d  %.2f  %.2f  %.2f  %.2f" % r)
    print("every 10th tick:", " ".join(f"{r[1]:.1f}/{r[2]:.1f}" for r in rows[::10]))
    se.close()


if __name__ == "__main__":
    main()
