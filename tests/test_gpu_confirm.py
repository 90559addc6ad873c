"""configs[4] on the GPU: 8,192 gated streams + the batched Whisper-tiny confirm.

Gated positives of a full 8,192-stream run (bench.make_streams) are normalised on the
device straight from the rings (ewk_normalize_events, bit-identical to
wakeword.py:1019-1025 -- checked here against the oracle's numpy expression on the
host copy of the same segments) and handed, still on cuda:0, to WhisperConfirm:
batch shapes, device residency, and the offline contract that a model without a
tokenizer never confirms (random init: parity unpinned, no weights offline).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_config5_gated_positives_to_whisper_on_gpu():
    import torch
    import bench
    from easywakeword_amd import StreamEngine
    from easywakeword_amd.confirm import WhisperConfirm
    from oracle.gate_ref import normalize_level3
    dev = torch.device("cuda", 0)
    word = bench.load_word()
    n_streams = 8192
    period, pcm = bench.make_streams(torch, dev, n_streams, 1234, word)
    se = StreamEngine(n_streams)
    se.template_from_pcm(word)
    evs = []
    for t in range(0, 160, 32):
        se.push_device(pcm.data_ptr() + t * 1600 * 4, period * 1600, 1600, 32)
        evs.append(se.poll())
    ev = np.concatenate(evs)
    pos = ev[(ev["match"] != 0) & ((ev["flags"] & 1) == 0)]
    assert len(pos) > 1000
    batch = pos[np.argsort(-pos["tick"], kind="stable")][:32]        # the newest: still in the rings
    audio = se.normalize_events_device(batch)
    assert len(audio) == 32
    for a, e in zip(audio, batch):
        assert a.device == dev and a.dtype == torch.float64 and a.numel() == int(e["length"])
    for a, e in list(zip(audio, batch))[:8]:
        host = se.read_segment(int(e["stream"]), int(e["ring_start"]), int(e["length"]))
        np.testing.assert_array_equal(a.cpu().numpy(), normalize_level3(host))
    wc = WhisperConfirm(device=dev, max_new_tokens=4)
    assert wc.random_init and wc.dtype == torch.bfloat16
    feats = wc.log_mel(audio)
    assert tuple(feats.shape) == (32, 80, 3000) and feats.device == dev
    assert torch.isfinite(feats).all()
    out = wc.transcribe(audio)
    assert out == [""] * 32                                           # no tokenizer offline: never confirms
    assert wc(audio[0]) is None
    se.close()
