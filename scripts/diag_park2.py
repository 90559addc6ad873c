"""Diagnostic: is the batch-vs-alone score difference of a segment (parking on) run-to-run
stable, and does it follow the segment's offset (alignment) in the packed buffer?"""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import easywakeword_amd as ewa
dev = torch.device("cuda", 0)
word = bench.load_word()
n = 65536
pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, dev, n, 1234, word)
eng = ewa.Engine()
eng.template_from_pcm(word)
mean = torch.empty((n, 20), device=dev); std = torch.empty((n, 20), device=dev)
score = torch.empty(n, device=dev, dtype=torch.float64); match = torch.empty(n, device=dev, dtype=torch.uint8)
s = torch.cuda.current_stream(dev)
runs = []
for r in range(3):
    eng.score_device(pcm.data_ptr(), off.data_ptr(), ln.data_ptr(), n, mean.data_ptr(), std.data_ptr(),
                     score.data_ptr(), match.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    runs.append(score.cpu().numpy().copy())
for r in range(1, 3):
    d = np.nonzero(runs[r] != runs[0])[0]
    print(f"run {r} vs run 0: {len(d)} differing segments {d[:10].tolist()}")
seg = int(os.environ.get("EWK_DIAG_SEG", "55320"))
x = pcm[int(offsets[seg]):int(offsets[seg]) + int(lengths[seg])].cpu().numpy()
print(f"seg {seg} offset {int(offsets[seg])} (mod 64: {int(offsets[seg]) % 64}) batch {runs[0][seg]!r}")
for pad in (0, 1, 4, int(offsets[seg]) % 64, int(offsets[seg]) % 1024):
    buf = np.concatenate([np.zeros(pad, np.float32), x])
    _, _, sc, _ = eng.score_packed(buf, np.array([pad], np.int64), np.array([len(x)], np.int32))
    print(f"  alone at offset {pad}: {sc[0]!r}")
# the segment within its neighbours: a 9-segment window of the batch
w = np.arange(max(0, seg - 4), min(n, seg + 5))
segs = [pcm[int(offsets[i]):int(offsets[i]) + int(lengths[i])].cpu().numpy() for i in w]
_, _, sc, _ = eng.score(segs, candidate_dtype="float64")
print(f"  in a window of {len(w)}: {sc[list(w).index(seg)]!r}")
