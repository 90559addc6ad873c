"""Why streaming events go to the fp64 re-score: the bench's streaming recipe (scripts/
rescore_ring_probe.py's setup) through a -DEWK_LIST_STATS build (EWK_LIB), counting per listing
criterion of score_epilogue (csrc/ewk_mfcc.hip) the segments and their frames.

    EWK_LIB=variants/list_stats.so python scripts/list_reasons.py [streams] [ticks]
"""
import ctypes
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import easywakeword_amd as ewa  # noqa: E402

dev = torch.device("cuda", 0)
word = bench.load_word()
n_streams = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 300
period, spcm = bench.make_streams(torch, dev, n_streams, 1234, word)
se = ewa.StreamEngine(n_streams)
se.template_from_pcm(word)
base = spcm.data_ptr()
dlib = ctypes.CDLL(os.environ["EWK_LIB"])
buf = (ctypes.c_ulonglong * 10)()
dlib.ewk_debug_list(buf)
events = 0
t = 0
while t < 100 + ticks:
    k = t % period
    n = min(32, 100 + ticks - t, period - k)
    se.push_device(base + k * 1600 * 4, period * 1600, 1600, n)
    ev = se.poll()
    events += int(((ev["flags"] & 1) == 0).sum())
    t += n
se.sync()
dlib.ewk_debug_list(buf)
d = list(buf)
print(f"{n_streams} streams, {100 + ticks} ticks: {events} events scored, {d[0]} listed ({d[5]} frames)")
for k, name in enumerate(["within rescore_margin of the threshold", "T <= 16 frames", "0 < |std| < 20",
                          "|mean| < 64"]):
    print(f"  {name:40s} {d[1 + k]:8d} segments  {d[6 + k]:10d} frames")
