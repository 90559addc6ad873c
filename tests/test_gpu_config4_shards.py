"""configs[3] -- 65,536 streams sharded over ranks, positive detections gathered to rank 0 --
rehearsed end to end on the one MI355X of a test box (VERDICT r2
"configs_untested").

Four ranks (tests/config4_rank.py under torch.distributed.run, gloo: RCCL needs one GPU per
rank) each own 16,384 of the 65,536 streams (shard_streams), gate and score them on their
own StreamEngine and hand their positives to rank 0 every 10 ticks through
PositiveCollector / gather_positives, the code bench.py's N > 1 streaming leg runs over
RCCL.  Input: bench.make_shifted_signal (stream s hears one long synthetic signal from tick
s on), 10 s prefill + 15 s.  Checks on what rank 0 received:

* the positives are exactly those of ONE engine holding all 65,536 streams (same stream,
  tick and length; scores within 1e-4 -- the shards score with the cooperative ring
  scorer, the single engine with one segment per wave, and both send the segments the
  float32 pass cannot decide to the same fp64 re-score -- every one a match);
* every scored event of that engine (positives and rejects) and every gathered positive
  is within 1e-4 of the oracle (oracle/mfcc_ref.py) with the oracle's decision;
* every gathered level-3 PCM equals wakeword.py:1019-1025's numpy normalisation of its
  segment, cut from the signal (bit for bit).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_TOTAL, WORLD, TICKS, SEED = 65536, 4, 250, 4242
RING = 160000


def _numpy_normalize(x):
    """wakeword.py:1019-1025 on the float64 ring slice (as tests/test_gpu_level3.py)."""
    a = np.asarray(x, dtype=np.float64)
    a = a - np.mean(a)
    max_val = np.max(np.abs(a))
    if max_val > 0:
        a = a / max_val
    a = a * 1.5
    return np.clip(a, -1.0, 1.0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_config4_sharded_positives_equal_one_engine(tmp_path):
    import torch
    import bench
    import easywakeword_amd as ewa
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import config4_rank

    torch.cuda.empty_cache()
    out = str(tmp_path / "rank0.npz")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(WORLD),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "config4_rank.py"), out, str(N_TOTAL), str(TICKS), str(SEED)]
    # the ranks' output goes to gpurun_out/ as it is written (stage lines: tests/config4_rank.py)
    from evidence import _out_dir, progress
    os.makedirs(_out_dir(), exist_ok=True)
    log = os.path.join(_out_dir(), "config4_ranks.log")
    with open(log, "w") as f:
        r = subprocess.run(cmd, stdout=f, stderr=subprocess.STDOUT, text=True, timeout=600, cwd=ROOT,
                           env=dict(os.environ, OMP_NUM_THREADS="2"))
    with open(log) as f:
        tail = f.read()[-3000:]
    assert r.returncode == 0, tail
    progress("config4: ranks done, single engine")
    got = np.load(out)
    assert int(got["world"]) == WORLD
    rec = got["rec"]

    # one engine holding every stream, the same input and push pattern
    dev = torch.device("cuda", 0)
    word = bench.load_word()
    sig = bench.make_shifted_signal(torch, dev, N_TOTAL, TICKS, SEED, word)
    se = ewa.StreamEngine(N_TOTAL)
    se.template_from_pcm(word)
    se_template = se.get_template()
    evs, t = [], 0
    while t < TICKS:
        nt = min(32 if t < config4_rank.PREFILL else 1, TICKS - t)
        se.push_device(sig.data_ptr() + t * 1600 * 4, 1600, 1600, nt)
        evs.append(se.poll())
        t += nt
    se.close()
    ev = np.concatenate(evs)
    pos = ev[(ev["match"] != 0) & ((ev["flags"] & 1) == 0)]
    assert len(pos) > 10000

    key1 = np.stack([pos["stream"].astype(np.int64), pos["tick"], pos["length"].astype(np.int64)], 1)
    o1 = np.lexsort(key1.T[::-1])
    o2 = np.lexsort(rec[:, :3].T[::-1])
    np.testing.assert_array_equal(rec[o2, :3], key1[o1])          # the same positives, none lost or doubled
    sc = rec[o2, 3].view(np.float64)
    assert float(np.max(np.abs(sc - pos["score"][o1]))) <= 1e-4   # MODE 1 vs MODE 2: one fp64 path
    assert np.all(sc >= 75.0)

    # every scored event of the 65,536 streams (positives and rejects) against the oracle, and
    # the gathered positives' scores: stream s hears the signal from tick
    # s on (its tick t is signal tick s + t), so events with equal (tick + s, request, length)
    # hold the same samples -- each distinct segment is scored once by the oracle
    # (tests/oracle_pool.py)
    from oracle_pool import oracle_scores
    progress(f"config4: {len(pos)} positives, oracle over the events")
    host = sig.cpu().numpy()
    sc_ev = ev[(ev["flags"] & 1) == 0]
    n_req = (sc_ev["tick"].astype(np.int64) * 1600 - sc_ev["ring_start"].astype(np.int64)) % RING
    p0 = sc_ev["tick"].astype(np.int64) * 1600 - n_req                    # offset in the stream
    key = np.stack([sc_ev["tick"].astype(np.int64) + sc_ev["stream"], n_req, sc_ev["length"].astype(np.int64)], 1)
    uniq, inv = np.unique(key, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    first = np.zeros(len(uniq), np.int64)
    first[inv[::-1]] = np.arange(len(sc_ev))[::-1]
    segs = [host[int(sc_ev["stream"][i]) * 1600 + int(p0[i]):][:int(sc_ev["length"][i])] for i in first]
    ref = oracle_scores(segs, *se_template)[inv]
    d = np.abs(sc_ev["score"] - ref)
    assert np.array_equal(np.isnan(sc_ev["score"]), np.isnan(ref))
    assert np.nanmax(d) <= 1e-4, (float(np.nanmax(d)), sc_ev[int(np.nanargmax(d))])
    np.testing.assert_array_equal(sc_ev["match"].astype(bool), ref >= 75.0)
    ref_pos = {(int(e["stream"]), int(e["tick"])): r for e, r in zip(sc_ev, ref)}
    gathered = np.array([ref_pos[(int(s), int(tk))] for s, tk in rec[o2, :2]])
    assert float(np.max(np.abs(sc - gathered))) <= 1e-4 and np.all(gathered >= 75.0)

    # the gathered level-3 PCM: each equals the normalisation of one positive's segment
    ring_start = {(int(e["stream"]), int(e["tick"])): int(e["ring_start"]) for e in pos}
    by_len = {}
    for s, tk, ln, _ in rec:
        by_len.setdefault(int(ln), []).append((int(s), int(tk)))
    lens = got["audio_lens"]
    assert len(lens) >= WORLD * 8 * 5                          # up to 8 per rank per gather
    off = 0
    for ln in lens:
        a = got["audio"][off:off + ln]
        off += ln
        ok = False
        for s, tk in by_len[int(ln)]:
            n_req = (tk * 1600 - ring_start[(s, tk)]) % RING
            p0 = s * 1600 + tk * 1600 - n_req
            if np.array_equal(a, _numpy_normalize(host[p0:p0 + ln])):
                ok = True
                break
        assert ok, int(ln)
