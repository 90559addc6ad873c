"""PositiveCollector.add when some polled positives' samples are already gone from their
ring (a poll more than (ring - request) / block ticks behind the cut, e.g. a
32-tick push on a compact ring): ewk_normalize_events refuses those events with
EWK_EOVERWRITTEN (RingOverwrittenError, a ValueError); the collector must keep them as records without PCM and keep the PCM of the
others, not lose the poll."""
import numpy as np
import pytest
import torch

from easywakeword_amd._lib import EVENT_DTYPE, RingOverwrittenError
from easywakeword_amd.shard import PositiveCollector


def _events(ticks):
    ev = np.zeros(len(ticks), dtype=EVENT_DTYPE)
    ev["stream"] = np.arange(len(ticks))
    ev["tick"] = ticks
    ev["length"] = 100 + np.arange(len(ticks))
    ev["score"] = 80.0
    ev["match"] = 1
    return ev


def test_add_keeps_records_of_overwritten_events():
    now, intact_ticks = 40, 8   # a ring that keeps a segment for 8 ticks after its cut

    def audio_fn(ev):   # the engine's rule: all or nothing per call
        if np.any(now - ev["tick"] > intact_ticks):
            raise RingOverwrittenError("the ring has overwritten its samples since")
        return [torch.full((int(e["length"]),), float(e["stream"])) for e in ev]

    col = PositiveCollector(0, torch.device("cpu"), every=10, audio_cap=64, audio_fn=audio_fn)
    ev = _events([39, 10, 35, 2, 33])   # ticks 10 and 2: overwritten
    col.add(ev)
    assert len(col.captured) == 1
    cap_ev, pcm = col.captured[0]
    assert sorted(cap_ev["tick"].tolist()) == [33, 35, 39]
    for e, x in zip(cap_ev, pcm):   # PCM still paired with its own record
        assert len(x) == int(e["length"]) and float(x[0]) == float(e["stream"])
    lost = np.concatenate(col.pending)
    assert sorted(lost["tick"].tolist()) == [2, 10]


def test_add_all_overwritten_goes_pending():
    def audio_fn(ev):
        raise RingOverwrittenError("the ring has overwritten its samples since")

    col = PositiveCollector(0, torch.device("cpu"), every=10, audio_cap=64, audio_fn=audio_fn)
    col.add(_events([1, 2, 3]))
    assert col.captured == []
    assert sorted(np.concatenate(col.pending)["tick"].tolist()) == [1, 2, 3]


def test_other_errors_propagate():
    def audio_fn(ev):
        raise ValueError("bad dtype")   # a bug in the capture, not a lost ring

    col = PositiveCollector(0, torch.device("cpu"), every=10, audio_cap=8, audio_fn=audio_fn)
    with pytest.raises(ValueError, match="bad dtype"):
        col.add(_events([39, 35, 33]))


def test_overwritten_is_a_value_error():
    assert issubclass(RingOverwrittenError, ValueError)
