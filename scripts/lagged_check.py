"""Are all events of a streaming_max-shaped run scored?  (GPU box; diagnostic.)

    python scripts/lagged_check.py [streams] [ticks] [lagged 0|1]

The rocprofv3 trace of the bench's streaming_max leg (2.8 M int16 streams, one tick per push,
lagged polls; scripts/tick_slowest.py) shows the ring scorer doing nothing on some ticks and
twice the work on the next.  This replays that leg's input (bench.make_shifted_signal, int16,
compact 3 s rings) and, per push, records the events delivered, how many carry a NaN score,
and the scorer's kernel time; then every NaN-scored event's segment is cut from the signal and
scored by the linear batch scorer: a finite score there means the ring path delivered an
event it never scored.
"""
import os
import sys
import time

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from easywakeword_amd import Engine, StreamEngine
    from easywakeword_amd._lib import EWK_RING_I16
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 160
    lagged = bool(int(sys.argv[3])) if len(sys.argv) > 3 else True
    dev = torch.device("cuda", 0)
    word = bench.load_word()
    sig = bench.make_shifted_signal(torch, dev, n, ticks + 1, 2718, word, pcm16=True)
    se = StreamEngine(n, ring_samples=48000, ring_format=EWK_RING_I16)
    se.template_from_pcm(word)
    got, per = [], []
    for t in range(ticks):
        se.profile(True)
        se.push_device_pcm16(sig.data_ptr() + t * 1600 * 2, 1600, 1600, 1)
        ev = se.poll(lagged=lagged)
        ms, k = se.profile_read(0)
        se.profile(False)
        real = ev[(ev["flags"] & 1) == 0]
        ticks_in = np.unique(ev["tick"]) if len(ev) else []
        per.append((t + 1, len(ev), int(np.isnan(real["score"]).sum()), ms, list(map(int, ticks_in))[:4]))
        got.append(ev)
    got.append(se.poll())
    se.close()
    ev = np.concatenate(got)
    print(f"{n} streams, {ticks} ticks, lagged={lagged}: {len(ev)} events")
    print("push tick: events delivered, NaN scores, scorer ms, event ticks in the poll")
    for row in per[95:140]:
        print("  ", row)
    real = ev[(ev["flags"] & 1) == 0]
    nan = real[np.isnan(real["score"])]
    print(f"scored events {len(real)}, NaN {len(nan)}")
    if len(nan):
        host = sig.cpu().numpy()
        pick = nan[:: max(1, len(nan) // 4000)]
        segs = []
        for m in pick:
            n_req = (int(m["tick"]) * 1600 - int(m["ring_start"])) % 48000
            p0 = int(m["stream"]) * 1600 + int(m["tick"]) * 1600 - n_req
            segs.append(host[p0:p0 + int(m["length"])].astype(np.float32) / np.float32(32768.0))
        eng = Engine()
        eng.template_from_pcm(word)
        _, _, sc, _ = eng.score(segs, candidate_dtype="float64")
        fin = np.isfinite(sc)
        print(f"NaN events re-scored by the linear scorer: {len(pick)}, finite there: {int(fin.sum())}")
        if fin.any():
            bad = pick[fin]
            print("  first unscored events (stream, tick, length):",
                  [(int(b["stream"]), int(b["tick"]), int(b["length"])) for b in bad[:10]])
            print("  their ticks:", np.unique(bad["tick"])[:40].tolist())
        eng.close()


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"({time.time() - t0:.1f} s)")
