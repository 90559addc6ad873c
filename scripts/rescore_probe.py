"""How many segments of a batch fall inside the fp64 re-score margin (and what it costs).
Usage: python scripts/rescore_probe.py [n_segments] [fixed_len]"""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import easywakeword_amd as ewa
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
fl = int(sys.argv[2]) if len(sys.argv) > 2 else 16000
dev = torch.device("cuda", 0)
word = bench.load_word()
e = ewa.Engine()
e.template_from_pcm(word)
for fixed in (0, fl):
    pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, dev, n, 1234 + 17 * (fixed > 0), word, fixed_len=fixed)
    mean = torch.empty((n, 20), device=dev); std = torch.empty((n, 20), device=dev)
    score = torch.empty(n, device=dev, dtype=torch.float64); match = torch.empty(n, device=dev, dtype=torch.uint8)
    s = torch.cuda.current_stream(dev).cuda_stream
    e.score_device(pcm.data_ptr(), off.data_ptr(), ln.data_ptr(), n, mean.data_ptr(), std.data_ptr(),
                   score.data_ptr(), match.data_ptr(), s)
    torch.cuda.synchronize()
    e.profile(True)
    e.score_device(pcm.data_ptr(), off.data_ptr(), ln.data_ptr(), n, mean.data_ptr(), std.data_ptr(),
                   score.data_ptr(), match.data_ptr(), s)
    torch.cuda.synchronize()
    k0, _ = e.profile_read(0); k1, _ = e.profile_read(1)
    e.profile(False)
    sc = score.cpu().numpy()
    near = np.abs(sc - 75.0) < 1e-3
    short = (1 + lengths // 160) <= 16
    print(f"fixed={fixed}: f32 {k0:.3f} ms, f64 rescore {k1:.3f} ms, near={int(near.sum())}, short={int(short.sum())}, "
          f"nan={int(np.isnan(sc).sum())}, matches={int(match.sum())}, score quantiles={np.nanpercentile(sc, [1, 25, 50, 75, 99]).round(2)}")
    vals, cnt = np.unique(sc.round(6), return_counts=True)
    top = np.argsort(-cnt)[:5]
    print("   most repeated scores:", list(zip(vals[top].tolist(), cnt[top].tolist())))
    del pcm
