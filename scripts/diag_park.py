"""Diagnostic: the fullsize test's batch-vs-subset score comparison, per segment, with the
scores printed in full; run twice (EWK_NO_PARK=0/1) to see whether top_db tile parking is
involved."""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import bench
import easywakeword_amd as ewa
from oracle import mfcc_ref
dev = torch.device("cuda", 0)
word = bench.load_word()
n = 65536
pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, dev, n, 1234, word)
eng = ewa.Engine()
eng.template_from_pcm(word)
tm, ts = eng.get_template()
mean = torch.empty((n, 20), device=dev); std = torch.empty((n, 20), device=dev)
score = torch.empty(n, device=dev, dtype=torch.float64); match = torch.empty(n, device=dev, dtype=torch.uint8)
s = torch.cuda.current_stream(dev)
eng.score_device(pcm.data_ptr(), off.data_ptr(), ln.data_ptr(), n, mean.data_ptr(), std.data_ptr(),
                 score.data_ptr(), match.data_ptr(), s.cuda_stream)
torch.cuda.synchronize()
sc = score.cpu().numpy()
rng = np.random.default_rng(5)
idx = np.unique(np.concatenate([rng.choice(n, 40, replace=False),
                                [int(np.argmax(lengths)), int(np.argmin(lengths)), 0, n - 1]]))
segs = [pcm[int(offsets[i]):int(offsets[i]) + int(lengths[i])].cpu().numpy() for i in idx]
_, _, sc2, _ = eng.score(segs, candidate_dtype="float64")
bad = np.nonzero(sc2 != sc[idx])[0]
watch = [int(i) for i in os.environ.get("EWK_DIAG_SEGS", "").split(",") if i]
for i in watch:
    b = int(np.nonzero(idx == i)[0][0]) if i in idx else None
    print(f"watch seg {i}: batch {sc[i]!r}" + (f" subset {sc2[b]!r}" if b is not None else ""))
print("EWK_NO_PARK", os.environ.get("EWK_NO_PARK"), "mismatches", len(bad))
for b in bad:
    i = int(idx[b]); x = segs[b]
    _, _, one, _ = eng.score([x], candidate_dtype="float64")
    cm, cs = mfcc_ref.extract_mfcc(x.astype(np.float64))
    ref = float(mfcc_ref.similarity_from_stats(tm, ts, cm, cs))
    print(f"seg {i} len {len(x)} T {1 + len(x) // 160}: batch {sc[i]!r} subset {sc2[b]!r} alone {one[0]!r} oracle {ref!r}")
