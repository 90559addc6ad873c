"""Multi-GPU layout of the hot path: one process per GPU.

Streams are independent, so they are partitioned across ranks with no data-path
collective (weak scaling): rank r owns a contiguous block of streams, gates them
and scores their segments on its own GPU.  The only exchange is the gather of
POSITIVE detections to one rank -- the input of the optional level-3 confirm,
which the reference runs once per detection (wakeword.py:1120-1130):

* ``MatchGather``       (batch scorer steps) device-side compaction of the matched
                        segments' (id, score, step) records, appended step after
                        step with no host sync, then one ``gather_positives`` per
                        flush (every K steps);
* ``PositiveCollector`` (streaming) accumulates each tick's polled positives and
                        gathers them every ``every`` ticks, with the level-3 input
                        PCM of up to ``audio_cap`` of them per rank;
* ``gather_positives``  one all_gather of the per-rank counts (three int64 per
                        rank), then point-to-point sends of each rank's records and
                        packed PCM to ``dst`` (batch_isend_irecv), sized by the counts.

Over RCCL (backend "nccl") on MI355X; the same code runs over gloo on CPU tensors
in the tests (tests/test_dist_gloo.py).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from ._lib import RingOverwrittenError


def shard_streams(n_streams: int, rank: int, world: int) -> tuple[int, int]:
    """(first stream, count) owned by `rank`: contiguous blocks, sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    if n_streams < 0:
        raise ValueError("n_streams must be >= 0")
    base, extra = divmod(n_streams, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def gather_positives(records, audio=None, count=None, group=None, dst: int = 0):
    """Gather every rank's positive detections to rank `dst`.

    records: [n, k] int64 tensor on this rank, k >= 3 with column 2 = segment length
             (the event fields: stream, tick, length, score bits, ...);
    count:   optional 0-d/1-element int64 tensor on the records' device: only
             records[:count] are sent (device-side compaction leaves the count on the
             GPU; it is read once, with the other ranks' counts, after the all_gather);
    audio:   optional list of 1-D float tensors, the PCM of the FIRST len(audio)
             records (lengths as in their column 2).
    Collectives: an all_gather of (count, PCM total, PCM records) per rank, then
    point-to-point sends of each rank's records and packed PCM to `dst`.
    Returns (records, audio list) on `dst`, (None, None) elsewhere; the tensors must
    live where the backend expects them (CUDA for RCCL, CPU for gloo).
    """
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = records.device
    k = records.shape[1] if records.dim() == 2 else 0
    flat = torch.cat([a.reshape(-1) for a in audio]) if audio else None
    total = 0 if flat is None else flat.numel()
    n_audio = len(audio) if audio else 0
    n = count.reshape(1).to(torch.int64) if count is not None else \
        torch.tensor([records.shape[0]], dtype=torch.int64, device=dev)
    meta = torch.cat([n, torch.tensor([total, n_audio], dtype=torch.int64, device=dev)])
    # a collective first: later point-to-point calls may then involve a subset of ranks
    parts = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(parts, meta, group=group)
    m = torch.stack(parts).cpu().tolist()           # the one host sync of a gather
    counts, totals, n_aud = [r[0] for r in m], [r[1] for r in m], [r[2] for r in m]
    ops, rec_bufs, pcm_bufs = [], {}, {}
    dtype = flat.dtype if flat is not None else torch.float64
    if rank == dst:
        for r in range(world):
            if r == dst:
                continue
            if counts[r]:
                rec_bufs[r] = torch.empty((counts[r], k), dtype=records.dtype, device=dev)
                ops.append(dist.P2POp(dist.irecv, rec_bufs[r], r, group=group))
            if totals[r]:
                pcm_bufs[r] = torch.empty(totals[r], dtype=dtype, device=dev)
                ops.append(dist.P2POp(dist.irecv, pcm_bufs[r], r, group=group))
        rec_bufs[dst] = records[:counts[dst]]
        if flat is not None:
            pcm_bufs[dst] = flat
    else:
        if counts[rank]:
            ops.append(dist.P2POp(dist.isend, records[:counts[rank]].contiguous(), dst, group=group))
        if total:
            ops.append(dist.P2POp(dist.isend, flat, dst, group=group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != dst:
        return None, None
    out_rec = torch.cat([rec_bufs[r] for r in range(world) if counts[r]]) if sum(counts) else \
        records.new_zeros((0, k))
    out_audio = None
    if audio is not None:
        out_audio = []
        for r in range(world):
            if not n_aud[r]:
                continue
            lens = [int(x) for x in rec_bufs[r][:n_aud[r], 2].tolist()]
            buf, o = pcm_bufs[r], 0
            for ln in lens:
                out_audio.append(buf[o:o + ln])
                o += ln
    return out_rec, out_audio


class MatchGather:
    """Batch scorer steps on N ranks: the matched segments' records go to `dst`.

    Device-side compaction into a persistent [steps * n_seg + 1, 3] int64 buffer
    (column 0 = global segment id first_id + i, column 1 = the float64 score's bits,
    column 2 = the step index since the last flush), with the running count left on the
    device: ``add`` appends one step's positives without any host sync, ``flush``
    gathers everything held so far -- one counts all_gather (the only host sync) plus
    point-to-point records per flush, however many steps it covers -- and only
    positives cross xGMI (never the per-segment score/match arrays).
    """

    def __init__(self, n_seg: int, first_id: int, device, steps: int = 1, group=None, dst: int = 0):
        import torch
        if steps < 1:
            raise ValueError("steps must be >= 1")
        self.n_seg, self.first_id, self.steps, self.group, self.dst = n_seg, first_id, steps, group, dst
        self.cap = n_seg * steps
        self.buf = torch.zeros((self.cap + 1, 3), dtype=torch.int64, device=device)   # row cap: discard slot
        self.ids = torch.arange(first_id, first_id + n_seg, dtype=torch.int64, device=device)
        self.count = torch.zeros(1, dtype=torch.int64, device=device)
        self.held = 0   # steps added since the last flush (host-side: no sync needed)

    def add(self, score, match) -> None:
        """Append one step's matches (device ops only; raises once `steps` are held)."""
        import torch
        if self.held >= self.steps:
            raise RuntimeError(f"MatchGather holds {self.steps} steps: flush() first")
        m = match.reshape(-1).to(torch.int64)
        pos = self.count + torch.cumsum(m, 0) - 1
        tgt = torch.where(m.bool(), pos, torch.full_like(pos, self.cap))
        vals = torch.stack([self.ids, score.reshape(-1).to(torch.float64).view(torch.int64),
                            torch.full_like(self.ids, self.held)], 1)
        self.buf.index_copy_(0, tgt, vals)
        self.count += m.sum()
        self.held += 1

    def compact(self, score, match):
        """One step on its own: (records [cap + 1, 3], count [1]), records[:count] in index order."""
        self.count.zero_()
        self.held = 0
        self.add(score, match)
        return self.buf, self.count

    def flush(self):
        """Gather every held record to `dst` (records on `dst`, None elsewhere) and re-arm."""
        rec = gather_positives(self.buf, count=self.count, group=self.group, dst=self.dst)[0]
        if rec is not None:
            rec = rec.clone()   # the buffer is reused by the next add()
        self.count.zero_()
        self.held = 0
        return rec

    def __call__(self, score, match):
        self.compact(score, match)
        return self.flush()


class PositiveCollector:
    """Streaming level-3 feed on N ranks: each tick's polled positives (match, not
    skipped) are kept on the host and gathered to `dst` every `every` ticks, records
    {global stream, tick, length, score bits} plus the level-3 input PCM of the newest
    `audio_cap` of them per rank (`audio_fn(events) -> list of 1-D tensors`, e.g.
    StreamEngine.normalize_events_device: the normalised audio, wakeword.py:1019-1025,
    straight from the rings).

    The PCM is captured in ``add`` -- right after the poll that returned the events, while
    the segments are still in the rings (a compact ring keeps only the longest request
    plus one tick; ten ticks later the start of a long utterance is gone) -- and only the
    newest `audio_cap` captures are kept until the flush.
    """

    def __init__(self, first_stream: int, device, every: int = 10, audio_cap: int = 64,
                 audio_fn: Optional[Callable] = None, group=None, dst: int = 0):
        self.first_stream, self.device, self.every, self.audio_cap = first_stream, device, every, audio_cap
        self.audio_fn, self.group, self.dst = audio_fn, group, dst
        self.pending = []      # positives without captured PCM
        self.captured = []     # [(events, pcm list)] newest first, <= audio_cap events in all
        self.ticks = 0
        self.gathered = 0
        self.gathered_audio = 0

    @staticmethod
    def _newest_first(ev: np.ndarray) -> np.ndarray:
        return ev[np.lexsort((ev["stream"], -ev["tick"]))]

    def add(self, events: np.ndarray) -> None:
        pos = events[(events["match"] != 0) & ((events["flags"] & 1) == 0)]
        if not len(pos):
            return
        if self.audio_fn is None or self.audio_cap <= 0:
            self.pending.append(pos)
            return
        pos = self._newest_first(pos)
        take = pos[:self.audio_cap]
        if len(pos) > len(take):
            self.pending.append(pos[len(take):])
        try:
            pcm = list(self.audio_fn(take))
        except RingOverwrittenError:
            # some events' samples were overwritten in their ring before this poll (a poll
            # more than (ring - request) / block ticks behind the cut: multi-tick pushes,
            # compact rings): those go on as records without PCM, the rest keep theirs
            keep, pcm, lost = [], [], []
            for i in range(len(take)):
                try:
                    pcm.extend(self.audio_fn(take[i:i + 1]))
                    keep.append(i)
                except RingOverwrittenError:   # (any other error is a bug: it propagates)
                    lost.append(i)
            if lost:
                self.pending.append(take[lost])
            take = take[keep]
            if not len(take):
                return
        self.captured.insert(0, (take, pcm))   # polls arrive in tick order
        kept = 0
        for i, (ev, pcm) in enumerate(self.captured):   # keep the newest audio_cap captures
            room = self.audio_cap - kept
            if room <= 0:
                self.pending.extend(e for e, _ in self.captured[i:])
                del self.captured[i:]
                break
            if len(ev) > room:
                self.pending.append(ev[room:])
                self.captured[i] = (ev[:room], pcm[:room])
            kept += len(self.captured[i][0])

    def tick(self, n: int = 1):
        """Count n ticks; gathers when `every` ticks have passed (returns flush()'s result)."""
        self.ticks += n
        if self.ticks >= self.every:
            return self.flush()
        return None, None

    def flush(self):
        import torch
        self.ticks = 0
        cap_ev = [e for e, _ in self.captured]
        audio = [x for _, pcm in self.captured for x in pcm] if self.audio_fn is not None else None
        rest = np.concatenate(self.pending) if self.pending else None
        rest = self._newest_first(rest) if rest is not None and len(rest) else None
        parts = cap_ev + ([rest] if rest is not None else [])
        self.pending, self.captured = [], []
        if parts:
            # the records with captured PCM first, in the order of their PCM
            ev = np.concatenate(parts)
            rec = np.stack([ev["stream"].astype(np.int64) + self.first_stream, ev["tick"].astype(np.int64),
                            ev["length"].astype(np.int64), ev["score"].astype(np.float64).view(np.int64)], axis=1)
        else:
            rec = np.zeros((0, 4), np.int64)
        out_rec, out_audio = gather_positives(torch.from_numpy(rec).to(self.device), audio=audio,
                                              group=self.group, dst=self.dst)
        if out_rec is not None:
            self.gathered += int(out_rec.shape[0])
            self.gathered_audio += len(out_audio) if out_audio is not None else 0
        return out_rec, out_audio
