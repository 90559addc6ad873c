"""One rank of the configs[3] rehearsal (tests/test_gpu_config4_shards.py), started by
torch.distributed.run: this rank's contiguous shard of the streams (shard_streams) gated and
scored on its own StreamEngine, its positive detections gathered to rank 0 every 10 ticks
by PositiveCollector (counts all_gather + point-to-point records and level-3 PCM), exactly
as bench.py's N > 1 streaming leg does.  The backend is gloo: every rank runs on the one
MI355X of the test box, so the collectives run on CPU copies (RCCL needs one GPU per rank).

Usage: config4_rank.py <out.npz> <total streams> <ticks> <seed>
Rank 0 writes the gathered records [stream, tick, length, score bits] and PCM to out.npz.
"""
import os
import sys
import time

import numpy as np

t_start = time.time()

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PREFILL = 100        # ticks pushed 32 per call (ring fill), then one tick per call
AUDIO_CAP = 8        # level-3 PCM of the newest 8 positives per rank per gather


def main():
    import torch
    import torch.distributed as dist
    import bench
    import easywakeword_amd as ewa
    from easywakeword_amd.shard import PositiveCollector, shard_streams

    out_path, n_total, ticks, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    say = lambda m: print(f"[rank {rank} {time.time() - t_start:.1f} s] {m}", flush=True)
    say("imports done")
    dist.init_process_group("gloo")
    say("process group up")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    word = bench.load_word()
    first, n = shard_streams(n_total, rank, world)
    sig = bench.make_shifted_signal(torch, dev, n_total, ticks, seed, word)   # stream s hears it from tick s
    se = ewa.StreamEngine(n)
    se.template_from_pcm(word)
    say(f"engine with {n} streams")
    cpu = torch.device("cpu")
    col = PositiveCollector(first, cpu, every=10, audio_cap=AUDIO_CAP,
                            audio_fn=lambda e: [a.cpu() for a in se.normalize_events_device(e)])
    recs, auds = [], []

    def keep(r, a):
        if r is not None:
            recs.append(r.numpy())
            auds.extend(x.numpy() for x in a)

    base = sig.data_ptr() + first * 1600 * 4
    t = 0
    while t < ticks:
        nt = min(32 if t < PREFILL else 1, ticks - t)
        se.push_device(base + t * 1600 * 4, 1600, 1600, nt)
        col.add(se.poll())
        keep(*col.tick(nt))
        t += nt
        if t % 50 == 0:
            say(f"tick {t}")
    keep(*col.flush())
    if rank == 0:
        rec = np.concatenate(recs) if recs else np.zeros((0, 4), np.int64)
        lens = np.array([len(a) for a in auds], np.int64)
        pcm = np.concatenate(auds) if auds else np.zeros(0)
        np.savez(out_path, rec=rec, audio_lens=lens, audio=pcm, world=world)
    se.close()
    dist.barrier()
    dist.destroy_process_group()
    say("done")


if __name__ == "__main__":
    main()
