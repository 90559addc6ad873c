"""Multi-GPU layout of the hot path: one process per GPU.

Streams are independent, so they are partitioned across ranks with no data-path
collective (weak scaling): rank r owns a contiguous block of streams, gates them
and scores their segments on its own GPU.  The only exchange is the gather of
level-2 decisions (score, match) to every rank -- the input of the optional
level-3 confirm, which the reference runs once per detection
(wakeword.py:1120-1130).  Over RCCL (backend "nccl") on MI355X; the same code
runs over gloo on CPU tensors in the tests.
"""
from __future__ import annotations


def shard_streams(n_streams: int, rank: int, world: int) -> tuple[int, int]:
    """(first stream, count) owned by `rank`: contiguous blocks, sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    if n_streams < 0:
        raise ValueError("n_streams must be >= 0")
    base, extra = divmod(n_streams, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


class DecisionGather:
    """All-gather of every rank's per-segment (score, match) arrays.

    Buffers are allocated once for a fixed per-rank segment count (the bench's
    step shape) so the collective runs without allocation inside the timed loop.
    `__call__` returns the world's scores and matches concatenated in rank order.
    """

    def __init__(self, score, match, group=None):
        import torch.distributed as dist
        self._dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.score_parts = [score.new_empty(score.shape) for _ in range(self.world)]
        self.match_parts = [match.new_empty(match.shape) for _ in range(self.world)]

    def __call__(self, score, match):
        self._dist.all_gather(self.score_parts, score, group=self.group)
        self._dist.all_gather(self.match_parts, match, group=self.group)
        return self.score_parts, self.match_parts

    def concatenated(self):
        import torch
        return torch.cat(self.score_parts), torch.cat(self.match_parts)


def gather_positives(records, audio=None, group=None, dst: int = 0):
    """Gather every rank's positive detections to rank `dst`.

    records: [n, k] int64 tensor on this rank, k >= 3 with column 2 = segment length
             (the event fields: stream, tick, length, score bits, ...);
    audio:   optional list of n 1-D float tensors (the segments' PCM, lengths as in column 2).
    Collectives: an all_gather of the per-rank counts (and PCM totals), an all_gather
    of the count-padded records, then point-to-point sends of each rank's packed PCM
    to `dst` (batch_isend_irecv).  Returns (records, audio list) on `dst`, (None, None)
    elsewhere.  The tensors must live where the backend expects them (CUDA for RCCL,
    CPU for gloo).
    """
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    n = records.shape[0]
    k = records.shape[1] if records.dim() == 2 else 0
    flat = torch.cat([a.reshape(-1) for a in audio]) if audio else None
    total = 0 if flat is None else flat.numel()
    meta = torch.tensor([n, total], dtype=torch.int64, device=records.device)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    counts = [int(m[0]) for m in metas]
    totals = [int(m[1]) for m in metas]
    cap = max(1, max(counts))
    padded = records.new_zeros((cap, k))
    if n:
        padded[:n] = records
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    out_rec = torch.cat([parts[r][:counts[r]] for r in range(world)]) if rank == dst else None
    out_audio = None
    if audio is not None:
        ops, bufs = [], {}
        if rank == dst:
            for r in range(world):
                if r == dst or totals[r] == 0:
                    continue
                bufs[r] = torch.empty(totals[r], dtype=flat.dtype if flat is not None else torch.float32,
                                      device=records.device)
                ops.append(dist.P2POp(dist.irecv, bufs[r], r, group=group))
            if flat is not None:
                bufs[dst] = flat
        elif total:
            ops.append(dist.P2POp(dist.isend, flat, dst, group=group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if rank == dst:
            out_audio = []
            for r in range(world):
                lens = [int(x) for x in parts[r][:counts[r], 2]] if counts[r] else []
                buf, o = bufs.get(r), 0
                for ln in lens:
                    out_audio.append(buf[o:o + ln])
                    o += ln
    return out_rec, out_audio


def positives(scores, matches, first_stream_of_rank, segments_per_stream: int):
    """Global (stream, segment) ids of the gathered matches -- what rank 0 hands to the confirm stage."""
    import torch
    out = []
    for r, (s, m) in enumerate(zip(scores, matches)):
        idx = torch.nonzero(m.to(torch.bool), as_tuple=False).flatten()
        for i in idx.tolist():
            out.append((first_stream_of_rank[r] + i // segments_per_stream, i % segments_per_stream,
                        float(s[i])))
    return out
