"""Decode the per-wave log-mel tiles a -DEWK_COOP_DEBUG scorer recorded for a wrong ring-path
score (tests/test_gpu_gate.py evidence, "coop" -> "tile") and compare them with the oracle's
raw log-mel of the same frames (CPU).

    python scripts/miss_tile_decode.py evidence.json

Tile layout (ewk_mfcc.hip tile_chunk): frame row r of a wave's 16-frame tile holds 16 hi chunks
then 16 lo chunks of 8 f16; lane j's chunk (bands j, j + 16, ..., j + 112) sits at slot j ^ r;
a value is float(hi) + float(lo).  Rows past the segment's last frame are ignored.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)
EVIDENCE = sys.argv.pop(1) if len(sys.argv) > 1 else ""   # (miss_r05 reads sys.argv at import)

import miss_r05  # noqa: E402
import miss_r06  # noqa: E402
from oracle.gate_ref import GateConfig, run_stream  # noqa: E402


def decode(tile_u32):
    """[512, 4] uint32 (8 KB) -> [16 rows, 128 bands] float32."""
    raw = np.asarray(tile_u32, np.uint32).reshape(16, 2, 16, 4).view(np.float16).reshape(16, 2, 16, 8)
    out = np.zeros((16, 128), np.float32)
    for r in range(16):
        for j in range(16):
            slot = j ^ r
            hi = raw[r, 0, slot].astype(np.float32)
            lo = raw[r, 1, slot].astype(np.float32)
            out[r, j + 16 * np.arange(8)] = hi + lo
    return out


def main():
    d = json.load(open(EVIDENCE))
    data = miss_r05.scenario()
    cfg = GateConfig(pre_speech_silence=0.8, speech_duration_min=0.3, speech_duration_max=2.0, post_speech_silence=0.4)
    for b in d["bad"]:
        c = b.get("coop")
        if not c or "tile" not in c:
            continue
        st, ln, tick = int(b["mine"][0]), int(b["mine"][1]), int(b["mine"][2])
        e = [e for e in run_stream(data[st], cfg).events if e.tick == tick][0]
        lm = miss_r06.raw_log_mel(np.asarray(e.audio, np.float64)).T        # [T, 128]
        T = lm.shape[0]
        tiles = np.asarray(c["tile"], dtype=np.uint64).astype(np.uint32)
        print(f"stream {st} tick {tick} L {ln} T {T}: engine {b['mine'][5]} oracle {b['oracle']}")
        for w in range((T + 15) // 16):
            g = decode(tiles[w])
            rows = min(16, T - 16 * w)
            ref = lm[16 * w:16 * w + rows]
            err = np.abs(g[:rows] - ref)
            bad = err > 1e-2
            if not bad.any():
                print(f"  wave {w} (frames {16 * w}..{16 * w + rows - 1}): all {rows * 128} values within {err.max():.1e}")
                continue
            fr = np.nonzero(bad.any(1))[0]
            print(f"  wave {w}: {int(bad.sum())} wrong values, frames {(16 * w + fr).tolist()}")
            for r in fr[:8]:
                bands = np.nonzero(bad[r])[0]
                lanes = sorted(set((bands % 16).tolist()))
                print(f"    frame {16 * w + r}: {len(bands)} bands wrong, lanes {lanes}, max err {err[r].max():.3f}")
                # is the wrong row another frame's true row (a misplaced frame)?
                dist = np.abs(lm - g[r][None, :]).max(1)
                k = int(np.argmin(dist))
                print(f"      nearest true frame {k} (max diff {dist[k]:.3e})")


if __name__ == "__main__":
    main()
