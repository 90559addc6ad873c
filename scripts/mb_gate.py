"""Gate microbenchmark: k_gate_ticks alone on the streaming recipe (one tick per launch).
Usage: python scripts/mb_gate.py [streams] [ticks]   (EWK_LIB selects the .so variant, e.g. one
built by scripts/build_variant.sh from another revision)."""
import os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import easywakeword_amd as ewa
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 200
pad = int(sys.argv[3]) if len(sys.argv) > 3 else 0     # extra floats per input row (stride experiments)
dev = torch.device("cuda", 0)
word = bench.load_word()
g = torch.Generator(device=dev); g.manual_seed(5)
P = 160 * 1600
pcm = torch.randn((n, P + pad), generator=g, device=dev) * 1e-3
pcm[:, 50000:50000 + len(word)] += torch.from_numpy(word).to(dev)
se = ewa.StreamEngine(n)
se.template_from_pcm(word)
base = pcm.data_ptr()
for t in range(120):                       # prefill + detection start
    se.push_device(base + (t % 160) * 1600 * 4, P + pad, 1600, 1)
    se.poll()
se.sync()
libname = os.environ.get("EWK_LIB") or os.path.join(ROOT, "easywakeword_amd", "libewk.so")
se.profile(True)
for t in range(120, 120 + ticks):
    se.push_device(base + (t % 160) * 1600 * 4, P + pad, 1600, 1)
    se.poll(lagged=True)
se.poll()
se.sync()
ms, k = se.profile_read(2)
print(f"{os.path.basename(libname):24s} pad {pad:4d} gate {ms / max(1, k) * 1e3:7.1f} us/tick over {k} ticks, {n} streams")
