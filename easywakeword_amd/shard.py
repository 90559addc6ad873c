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
