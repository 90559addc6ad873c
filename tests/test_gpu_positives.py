"""Positive detections on their way to the level-3 confirm (the
reference confirms each detection, wakeword.py:1120-1130):

* ewk_compact_positives (the C-ABI compaction a C/C++ host hands to its own RCCL
  gather) equals easywakeword_amd.shard.MatchGather's device compaction, one step and
  K steps appended;
* ewk_normalize_events refuses an event whose samples a compact ring has overwritten
  since its tick, and the PositiveCollector captures each positive's level-3 PCM at
  its poll, so a compact ring with a 10-tick gather still delivers intact audio
  (ADVICE r2);
* the batch gather over RCCL itself (world size 1 on the box's one GPU).
"""
import os
import socket

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(n, seed):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    score = torch.rand(n, generator=g, device="cuda", dtype=torch.float64) * 100.0
    score[::7] = float("nan")
    match = (score >= 75.0).to(torch.uint8)
    return score, match


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 100003])
def test_compact_positives_equals_matchgather(n):
    import torch
    from easywakeword_amd import Engine, _lib
    from easywakeword_amd.shard import MatchGather
    eng = Engine()
    score, match = _batch(n, 11 + n)
    out = torch.empty((max(n, 1), 3), dtype=torch.int64, device="cuda")
    cnt = torch.full((1,), -5, dtype=torch.int32, device="cuda")
    eng.compact_positives_device(score.data_ptr(), match.data_ptr(), n, 1000, out.data_ptr(), cnt.data_ptr(), step=0)
    torch.cuda.synchronize()
    g = MatchGather(n, 1000, torch.device("cuda"))
    rec, c = g.compact(score, match)
    k = int(c.item())
    assert int(cnt.item()) == k == int(match.sum().item())
    # ewk_positive {id, score, step} vs MatchGather rows {id, score bits, step}
    np.testing.assert_array_equal(out[:k].cpu().numpy(), rec[:k].cpu().numpy())
    assert _lib.POSITIVE_DTYPE.itemsize == 24


def test_compact_positives_append_k_steps():
    import torch
    from easywakeword_amd import Engine
    from easywakeword_amd.shard import MatchGather
    n, K = 50001, 4
    eng = Engine()
    g = MatchGather(n, 7, torch.device("cuda"), steps=K)
    out = torch.empty((n * K, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    for k in range(K):
        score, match = _batch(n, 100 + k)
        eng.compact_positives_device(score.data_ptr(), match.data_ptr(), n, 7, out.data_ptr(), cnt.data_ptr(),
                                     step=k, append=k > 0)
        g.add(score, match)
    torch.cuda.synchronize()
    total = int(cnt.item())
    assert total == int(g.count.item()) > 0
    np.testing.assert_array_equal(out[:total].cpu().numpy(), g.buf[:total].cpu().numpy())


def _hum_stream(seed, start_s, total_s=24.0, dur=1.8, block=1600):
    """Noise with one 1.8 s harmonic hum starting at start_s (a long utterance: its
    segment request nearly fills a compact ring)."""
    rng = np.random.default_rng(seed)
    sr = 16000
    x = rng.normal(0.0, 1e-3, int(total_s * sr)).astype(np.float32)
    t = np.arange(int(dur * sr)) / sr
    env = np.minimum(1.0, np.minimum(t, t[-1] - t) / 0.05)
    hum = (0.3 * np.sin(2 * np.pi * 150 * t) + 0.2 * np.sin(2 * np.pi * 500 * t)) * env
    i0 = int(start_s * sr)
    x[i0:i0 + len(hum)] += hum.astype(np.float32)
    return x[: len(x) // block * block]


def _numpy_normalize(x):   # wakeword.py:1019-1025
    a = np.asarray(x, dtype=np.float64)
    a = a - np.mean(a)
    m = np.max(np.abs(a))
    if m > 0:
        a = a / m
    return np.clip(a * 1.5, -1.0, 1.0)


def test_compact_ring_positives_pcm_captured_at_poll():
    import torch
    import torch.distributed as dist
    from easywakeword_amd import StreamEngine
    from easywakeword_amd.shard import PositiveCollector
    pcm = np.stack([_hum_stream(1, 12.3), _hum_stream(2, 14.1), _hum_stream(3, 16.0)])
    # the smallest compact ring the engine accepts for this config (43,200 samples)
    eng = StreamEngine(3, ring_samples=43200, similarity_threshold=1.0)
    eng.template_from_pcm(synth.load_word())
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        col = PositiveCollector(0, torch.device("cpu"), every=10, audio_cap=64,
                                audio_fn=eng.normalize_events_device)
        seen, got_rec, got_aud, late = {}, [], [], []
        for t in range(pcm.shape[1] // 1600):
            eng.push(pcm[:, t * 1600:(t + 1) * 1600])
            ev = eng.poll()
            for e in ev[(ev["match"] != 0) & ((ev["flags"] & 1) == 0)]:
                key = (int(e["stream"]), int(e["tick"]))
                seen[key] = _numpy_normalize(eng.read_segment(key[0], int(e["ring_start"]), int(e["length"])))
                late.append(e.copy())
            col.add(ev)
            rec, aud = col.tick()
            if rec is not None:
                got_rec.append(rec.numpy())
                got_aud.extend(a.cpu().numpy() for a in aud)
        rec, aud = col.flush()
        got_rec.append(rec.numpy())
        got_aud.extend(a.cpu().numpy() for a in aud)
    finally:
        dist.destroy_process_group()
    rec = np.concatenate(got_rec)
    assert len(seen) == 3 and len(rec) == 3 and len(got_aud) == 3
    for r, a in zip(rec.tolist(), got_aud):
        assert r[2] == len(a)
        np.testing.assert_array_equal(a, seen[(r[0], r[1])])
    # ten ticks after its cut the ring has overwritten a 1.8 s utterance's first samples:
    # reading it then is refused instead of returning corrupted level-3 input
    ev = np.array(late, dtype=late[0].dtype)
    with pytest.raises(ValueError, match="overwritten"):
        eng.normalize_events(ev[:1])


def test_match_gather_over_rccl_world_1():
    """MatchGather's K-step flush with CUDA tensors over RCCL ("nccl"), world size 1."""
    import torch
    import torch.distributed as dist
    from easywakeword_amd.shard import MatchGather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = 20000
        g = MatchGather(n, 0, torch.device("cuda"), steps=3)
        want = []
        for k in range(3):
            score, match = _batch(n, 300 + k)
            g.add(score, match)
            idx = torch.nonzero(match).reshape(-1)
            want.append(torch.stack([idx, score[idx].view(torch.int64), torch.full_like(idx, k)], 1))
        rec = g.flush()
        assert dist.get_backend() == "nccl"
        np.testing.assert_array_equal(rec.cpu().numpy(), torch.cat(want).cpu().numpy())
    finally:
        dist.destroy_process_group()
