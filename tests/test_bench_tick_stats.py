"""bench.tick_stats: the per-tick latency summary every streaming leg reports, and the
real-time verdict built on its max (every tick within 100 ms, not the mean)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_tick_stats_max_and_tail():
    ms = [10.0] * 998 + [99.0, 101.0]
    st = bench.tick_stats(ms)
    assert st["tick_ms_max"] == 101.0
    assert st["ticks_over_100ms"] == 1
    assert st["ticks_timed"] == 1000
    assert 10.0 <= st["tick_ms_p999"] <= 101.0
    assert st["tick_ms_p50"] == 10.0


def test_tick_stats_empty():
    st = bench.tick_stats([])
    assert st["tick_ms_max"] is None and st["ticks_over_100ms"] is None
