"""How far is the float32 pass's top_db threshold from the fp64 one?  (GPU box; diagnostic.)

    EWK_LIB=variants/rs_timing.so python scripts/rs_window_probe.py [n_segments]

The fp64 re-score classifies each log-mel value against the float32 pass's threshold theta_s
(max - 80 dB) and is exact for the fp64 threshold theta as long as |theta - theta_s| <= kRsWindow
and no value lies within kRsWindow of theta_s (ewk_rescore.h); a chunk holding such a value is
recomputed by the slot's finishing wave.  With every segment listed (rescore_margin = 1e9) over
the bench's ragged batch, the streaming recipe's segments and a few quiet / loud / stationary
recipes, this reads the -DEWK_RS_TIMING build's counters: max |theta - theta_s|, slots that had
to redo every chunk, chunks recomputed.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import bench
    import easywakeword_amd as ewa
    import synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    dev = torch.device("cuda", 0)
    word = bench.load_word()
    lib = ctypes.CDLL(os.environ["EWK_LIB"])
    d = (ctypes.c_ulonglong * 16)()
    e = ewa.Engine(rescore_margin=1e9)
    e.template_from_pcm(word)

    def report(name, nseg):
        lib.ewk_debug_rs(d)
        v = list(d)
        print(f"{name}: {nseg} segments, finishes {v[3]} serial {v[5]}, chunks {v[1]} (in finished slots {v[7]}), "
              f"redo_all {v[6]}, chunks recomputed {v[8]}, max |theta - theta_s| {v[14] * 1e-9:.3e} dB", flush=True)

    lib.ewk_debug_rs(d)   # reset
    for fixed in (0, 16000, 6400):
        pcm, off, ln, frames, lengths, offsets = bench.make_segments(torch, dev, n, 1234 + fixed, word, fixed_len=fixed)
        mean = torch.empty((n, 20), device=dev)
        std = torch.empty((n, 20), device=dev)
        score = torch.empty(n, device=dev, dtype=torch.float64)
        match = torch.empty(n, device=dev, dtype=torch.uint8)
        s = torch.cuda.current_stream(dev).cuda_stream
        e.score_device(pcm.data_ptr(), off.data_ptr(), ln.data_ptr(), n, mean.data_ptr(), std.data_ptr(),
                       score.data_ptr(), match.data_ptr(), s)
        torch.cuda.synchronize()
        report(f"bench batch fixed_len={fixed}", n)
        del pcm
    rng = np.random.default_rng(11)
    for kind in ("quiet", "loud", "stationary", "streams"):
        segs = []
        for i in range(2048):
            L = int(rng.integers(6400, 33600))
            if kind == "quiet":
                y = rng.standard_normal(L) * 10 ** rng.uniform(-6, -3)
            elif kind == "loud":
                y = np.clip(rng.standard_normal(L) * rng.uniform(0.5, 4.0), -1, 1)
            elif kind == "stationary":
                t = np.arange(L) / 16000.0
                y = 0.3 * np.sin(2 * np.pi * rng.uniform(100, 4000) * t) + 1e-4 * rng.standard_normal(L)
            else:
                p, _ = synth.make_stream(seed=int(rng.integers(1 << 30)), n_words=1, sigma=float(rng.uniform(1e-4, 5e-3)),
                                         gain=float(rng.uniform(0.2, 3.0)), distractors=bool(i % 2))
                y = p[-L:]
            segs.append(y.astype(np.float32))
        e.score(segs, candidate_dtype="float64")
        report(kind, len(segs))
    # tests/test_gpu_rescore_window.py's segments: a value placed at the threshold on purpose
    import test_gpu_rescore_window as tw
    segs = tw._segments()
    e.score(segs, candidate_dtype="float64")
    report("values at the threshold (chunked slots)", len(segs))
    e.score_f64(segs)
    report("values at the threshold (serial slots)", len(segs))
    e.close()


if __name__ == "__main__":
    main()
