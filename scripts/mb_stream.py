"""Streaming tick loop microbenchmark: push_device + lagged poll per tick (the bench's
config-3 cadence) at several stream counts, to separate host/API cost from GPU time.
Usage: python scripts/mb_stream.py [ticks] [streams ...]"""
import os, sys, time
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import easywakeword_amd as ewa
ticks = int(sys.argv[1]) if len(sys.argv) > 1 else 400
counts = [int(x) for x in sys.argv[2:]] or [64, 1024, 8192]
dev = torch.device("cuda", 0)
word = bench.load_word()
P = 160 * 1600
for n in counts:
    rng = np.random.Generator(np.random.PCG64(3))
    g = torch.Generator(device=dev); g.manual_seed(5)
    pcm = torch.randn((n, P), generator=g, device=dev) * 1e-3
    table = torch.from_numpy(bench.event_sources(word, rng)).to(dev)
    for e in range(5):
        pos = (e * P // 5 + rng.integers(0, 8000, n)).astype(np.int64)
        kind = bench.event_kind(rng, n)
        idx = torch.from_numpy(pos).to(dev)[:, None] + torch.arange(len(word), device=dev)[None, :]
        pcm.scatter_add_(1, idx, table[torch.from_numpy(kind).to(dev)])
    se = ewa.StreamEngine(n)
    se.template_from_pcm(word)
    base = pcm.data_ptr()
    for t in range(110):
        se.push_device(base + (t % 160) * 1600 * 4, P, 1600, 1)
        se.poll(lagged=True)
    se.poll()
    se.sync()
    prof = os.environ.get("MB_PROFILE", "1") == "1"
    se.profile(prof)
    t_push = t_poll = 0.0
    w0 = time.perf_counter()
    for t in range(110, 110 + ticks):
        a = time.perf_counter()
        se.push_device(base + (t % 160) * 1600 * 4, P, 1600, 1)
        b = time.perf_counter()
        se.poll(lagged=True)
        c = time.perf_counter()
        t_push += b - a
        t_poll += c - b
    se.poll()
    se.sync()
    wall = time.perf_counter() - w0
    ms = [se.profile_read(k) for k in (2, 0, 1)] if prof else [(0.0, 0)] * 3
    print(f"{n:6d} streams: {wall / ticks * 1e3:.4f} ms/tick (push {t_push / ticks * 1e3:.4f}, poll {t_poll / ticks * 1e3:.4f}); "
          f"gate {ms[0][0] / max(1, ms[0][1]) * 1e3:.1f} us, f32 {ms[1][0] / max(1, ms[1][1]) * 1e3:.1f} us, "
          f"f64 {ms[2][0] / max(1, ms[2][1]) * 1e3:.1f} us per tick")
    se.close()
    del pcm
