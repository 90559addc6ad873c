"""Scorer microbenchmark: time k_score_f32 over the bench's ragged batch distribution.
Usage: python scripts/mb_score.py [n_segments] [reps]   (EWK_LIB selects the .so variant)"""
import os, sys, time
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import easywakeword_amd as ewa
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
word = bench.load_word()
fixed = int(os.environ.get("EWK_FIXED_LEN", "0"))   # > 0: every segment that many samples (T-sweep)
pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, dev, n, 1234, word, fixed_len=fixed)
if os.environ.get("EWK_SORT"):   # experiment: hand the kernel its work longest-first (LPT)
    order = torch.argsort(ln, descending=True)
    off, ln = off[order].contiguous(), ln[order].contiguous()
mean = torch.empty((n, 20), device=dev); std = torch.empty((n, 20), device=dev)
score = torch.empty(n, device=dev, dtype=torch.float64); match = torch.empty(n, device=dev, dtype=torch.uint8)
e = ewa.Engine()
e.template_from_pcm(word)
s = torch.cuda.Stream(dev); torch.cuda.set_stream(s)
def step():
    e.score_device(pcm.data_ptr(), off.data_ptr(), ln.data_ptr(), n, mean.data_ptr(), std.data_ptr(),
                   score.data_ptr(), match.data_ptr(), s.cuda_stream)
step(); torch.cuda.synchronize()
e.profile(True)
for _ in range(reps): step()
torch.cuda.synchronize()
ms, k = e.profile_read(0)
ms /= k
lib = os.path.basename(os.environ.get("EWK_LIB", "libewk.so"))
print(f"{lib:28s} L={fixed or 'ragged'} {ms:8.3f} ms  {frames/ms/1e6:7.3f} Gframes/s  frac={frames*640/(ms/1e3)/8e12:.4f}  "
      f"matches={int(match.sum())} nan={int(torch.isnan(score).sum())} s0={float(score[0]):.4f}")
import ctypes
lib = ctypes.CDLL(os.environ.get("EWK_LIB") or os.path.join(ROOT, "easywakeword_amd", "libewk.so"))
if hasattr(lib, "ewk_debug_timing"):   # -DEWK_TIMING builds (easywakeword_amd/libewk_timing.so)
    buf = (ctypes.c_ulonglong * 20)()
    lib.ewk_debug_timing(buf)      # reset
    e.profile(False)
    step(); torch.cuda.synchronize()
    lib.ewk_debug_timing(buf)
    names = ["fetch+setup", "scout+rank", "first stage", "frame passes", "tile clamp/dct/stats", "recompute",
             "finish_stats", "epilogue"]
    waves, segs = max(1, buf[8]), max(1, buf[9])
    tot = sum(buf[i] for i in range(8))
    print(f"  waves={waves} segments={segs}; s_memtime cycles per segment: " +
          ", ".join(f"{n}={buf[i] / segs:,.0f} ({100.0 * buf[i] / max(1, tot):.1f}%)" for i, n in enumerate(names)) +
          f"; recomputed tiles/segment={(buf[10] & 0xffff) / segs:.3f} passes/segment={buf[11] / segs:.3f} "
          f"parked fixes/segment={(buf[10] >> 16) / segs:.3f}")
    if buf[19]:   # frame-pass sub-phases (first-pass passes only)
        sub = ["window+DFT16a", "twiddle", "transposes", "DFT16b", "untangle+power", "mel+log", "tile write+stage"]
        print(f"  per frame pass ({buf[19] / waves:,.0f} per wave): " +
              ", ".join(f"{n}={buf[12 + i] / buf[19]:,.0f}" for i, n in enumerate(sub)) +
              f"; total {sum(buf[12 + i] for i in range(7)) / buf[19]:,.0f} cycles")
