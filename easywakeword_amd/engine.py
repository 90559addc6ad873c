"""Thin Python owners of an ``ewk_engine`` (the C ABI in include/ewk.h).

``Engine``       -- scorer-only engine (level 2): the WordMatcher hot path.
``StreamEngine`` -- N concurrent streams on one GPU (levels 1 + 2): the
                    SoundBuffer + _detect_word hot loop for many microphones.

No CPU fallback exists: construction raises when libewk.so or a GPU is missing.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import N_MFCC, check

FREQUENCY = 16000


def _f32(audio) -> np.ndarray:
    a = np.asarray(audio)
    if a.ndim != 1:
        a = a.reshape(-1)
    return np.ascontiguousarray(a, dtype=np.float32)


class Engine:
    """Owns one ewk_engine on `gpu` (scorer-only unless n_streams > 0)."""

    def __init__(self, gpu: int = 0, n_streams: int = 0, config: Optional[_lib.EwkConfig] = None, **cfg):
        self._lib = _lib.load()
        self._h = C.c_void_p()
        if config is None:
            config = _lib.default_config(**cfg)
        self.config = config
        check(self._lib.ewk_create(C.byref(self._h), int(gpu), int(n_streams), C.byref(config)))
        self.gpu = int(gpu)
        self.n_streams = int(n_streams)

    # -- lifetime ------------------------------------------------------------
    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.ewk_destroy(h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def stream_handle(self) -> int:
        return int(self._lib.ewk_stream_handle(self._h) or 0)

    def sync(self) -> None:
        check(self._lib.ewk_sync(self._h))

    # -- measurement ---------------------------------------------------------
    def profile(self, on: bool = True) -> None:
        check(self._lib.ewk_profile_enable(self._h, int(bool(on))))

    def profile_read(self, kind: int = 0):
        """(total_ms, launches) of the kernel family since the last read
        (0 = fp32 scorer, 1 = fp64 re-scorer, 2 = gate)."""
        ms = C.c_double(0.0)
        n = C.c_int64(0)
        check(self._lib.ewk_profile_read(self._h, int(kind), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    # -- template ------------------------------------------------------------
    def template_from_pcm(self, audio) -> None:
        a = _f32(audio)
        check(self._lib.ewk_template_from_pcm(self._h, _lib.fptr(a), len(a)))

    def set_template(self, mean, std) -> None:
        m = _f32(mean)
        s = _f32(std)
        if m.size != N_MFCC or s.size != N_MFCC:
            raise ValueError(f"template must be {N_MFCC} means and {N_MFCC} stds")
        check(self._lib.ewk_set_template(self._h, _lib.fptr(m), _lib.fptr(s)))

    def get_template(self) -> Tuple[np.ndarray, np.ndarray]:
        m = np.zeros(N_MFCC, np.float32)
        s = np.zeros(N_MFCC, np.float32)
        check(self._lib.ewk_get_template(self._h, _lib.fptr(m), _lib.fptr(s)))
        return m, s

    def set_threshold(self, threshold: float) -> None:
        check(self._lib.ewk_set_similarity_threshold(self._h, float(threshold)))
        self.config.similarity_threshold = float(threshold)

    # -- level 2 over ragged host batches ------------------------------------
    def score(self, segments, require_template: bool = True, candidate_dtype: str = "auto"):
        """MFCC stats + score of a list of 1-D arrays.  Returns
        (mean[n,20] f32, std[n,20] f32, score[n] f64, match[n] bool).

        candidate_dtype selects the reference arithmetic of the score:
        "float64" (SoundBuffer slices, the streaming path), "float32"
        (WordMatcher fed float32 audio) or "auto" (float32 iff every segment is)."""
        if candidate_dtype == "auto":
            f32 = all(np.asarray(s).dtype == np.float32 for s in segments) and len(segments) > 0
        else:
            f32 = np.dtype(candidate_dtype) == np.float32
        segs = [_f32(s) for s in segments]
        n = len(segs)
        lengths = np.array([len(s) for s in segs], dtype=np.int32)
        offsets = np.zeros(n, dtype=np.int64)
        if n:
            offsets[1:] = np.cumsum(lengths[:-1], dtype=np.int64)
        pcm = np.concatenate(segs) if n else np.zeros(0, np.float32)
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        return self.score_packed(pcm, offsets, lengths, require_template, f32)

    def score_packed(self, pcm: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
                     require_template: bool = True, f32_candidates: bool = False):
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        lengths = np.ascontiguousarray(lengths, dtype=np.int32)
        n = len(lengths)
        mean = np.zeros((n, N_MFCC), np.float32)
        std = np.zeros((n, N_MFCC), np.float32)
        score = np.full(n, np.nan, np.float64)
        match = np.zeros(n, np.uint8)
        check(self._lib.ewk_score_segments(self._h, _lib.fptr(pcm), len(pcm), _lib.i64ptr(offsets),
                                           _lib.i32ptr(lengths), n, _lib.fptr(mean), _lib.fptr(std),
                                           _lib.dptr(score), _lib.u8ptr(match), self._flags(require_template,
                                                                                            f32_candidates)))
        return mean, std, score, match.astype(bool)

    @staticmethod
    def _flags(require_template: bool, f32: bool) -> int:
        return (_lib.EWK_SCORE_REQUIRE_TEMPLATE if require_template else 0) | \
            (_lib.EWK_SCORE_F32_CANDIDATES if f32 else 0)

    def score_f64(self, segments, candidate_dtype: str = "float64"):
        """Reference-precision (float64) path: (mean[n,20], std[n,20], score[n])."""
        f32 = np.dtype(candidate_dtype) == np.float32
        segs = [_f32(s) for s in segments]
        n = len(segs)
        lengths = np.array([len(s) for s in segs], dtype=np.int32)
        offsets = np.zeros(n, dtype=np.int64)
        if n:
            offsets[1:] = np.cumsum(lengths[:-1], dtype=np.int64)
        pcm = np.ascontiguousarray(np.concatenate(segs) if n else np.zeros(0, np.float32), dtype=np.float32)
        mean = np.zeros((n, N_MFCC), np.float64)
        std = np.zeros((n, N_MFCC), np.float64)
        score = np.full(n, np.nan, np.float64)
        check(self._lib.ewk_score_segments_f64(self._h, _lib.fptr(pcm), len(pcm), _lib.i64ptr(offsets),
                                               _lib.i32ptr(lengths), n, _lib.dptr(mean), _lib.dptr(std),
                                               _lib.dptr(score), self._flags(False, f32)))
        return mean, std, score

    def normalize(self, segments) -> list:
        """Level-3 pre-processing of each segment on the GPU (wakeword.py:1019-1025):
        float64, bit-identical to the reference's numpy (see include/ewk.h)."""
        segs = [_f32(s) for s in segments]
        n = len(segs)
        if n == 0:
            return []
        lengths = np.array([len(s) for s in segs], dtype=np.int32)
        offsets = np.zeros(n, dtype=np.int64)
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.int64)
        pcm = np.ascontiguousarray(np.concatenate(segs), dtype=np.float32)
        out = np.zeros(max(1, int(lengths.sum())), np.float64)
        check(self._lib.ewk_normalize_segments(self._h, pcm.ctypes.data_as(C.c_void_p), len(pcm),
                                               _lib.i64ptr(offsets), _lib.i32ptr(lengths), n,
                                               out.ctypes.data_as(C.c_void_p), 0))
        return [out[o:o + l] for o, l in zip(offsets, lengths)]

    def decode_pcm16(self, pcm16: np.ndarray) -> np.ndarray:
        """int16 PCM -> float32 (x / 32768, librosa.load's value for 16 kHz PCM16) on the GPU."""
        a = np.ascontiguousarray(pcm16, dtype=np.int16)
        out = np.zeros(a.shape, np.float32)
        if a.size:
            check(self._lib.ewk_decode_pcm16(self._h, a.ctypes.data_as(C.c_void_p), a.size,
                                             out.ctypes.data_as(C.c_void_p), 0))
        return out

    def score_device(self, pcm_ptr: int, offsets_ptr: int, lengths_ptr: int, n: int, mean_ptr: int,
                     std_ptr: int, score_ptr: int, match_ptr: int, stream: int = 0,
                     f32_candidates: bool = False) -> None:
        """Device-resident batch (e.g. torch tensor data_ptr()s); asynchronous on `stream`."""
        check(self._lib.ewk_score_segments_device(self._h, C.c_void_p(pcm_ptr), C.c_void_p(offsets_ptr),
                                                  C.c_void_p(lengths_ptr), int(n), C.c_void_p(mean_ptr or None),
                                                  C.c_void_p(std_ptr or None), C.c_void_p(score_ptr or None),
                                                  C.c_void_p(match_ptr or None), self._flags(False, f32_candidates),
                                                  C.c_void_p(stream or None)))


    def compact_positives_device(self, score_ptr: int, match_ptr: int, n: int, first_id: int, out_ptr: int,
                                 count_ptr: int, step: int = 0, append: bool = False, stream: int = 0) -> None:
        """Matched segments of a device batch -> ewk_positive records {id, score, step} at
        out_ptr (device, segment order) and their int32 count at count_ptr (device); with
        append=True after the count already there.  Asynchronous on `stream`, no host sync:
        the buffers go straight to an RCCL gather (include/ewk.h, ewk_compact_positives)."""
        check(self._lib.ewk_compact_positives(self._h, C.c_void_p(score_ptr or None), C.c_void_p(match_ptr or None),
                                              int(n), int(first_id), int(step), C.c_void_p(out_ptr or None),
                                              C.c_void_p(count_ptr or None),
                                              _lib.EWK_COMPACT_APPEND if append else 0, C.c_void_p(stream or None)))


class StreamEngine(Engine):
    """N concurrent 16 kHz streams on one GPU: ring + adaptive threshold + timing
    FSM per stream (level 1) and MFCC matching of every gated segment (level 2)."""

    def __init__(self, n_streams: int, gpu: int = 0, config: Optional[_lib.EwkConfig] = None, **cfg):
        if n_streams <= 0:
            raise ValueError("n_streams must be positive")
        super().__init__(gpu=gpu, n_streams=n_streams, config=config, **cfg)
        self.block = int(self.config.block)
        self.ring_len = int(self.config.buffer_seconds) * FREQUENCY          # the reference ring
        self.sample_ring = int(self.config.ring_samples) or self.ring_len    # samples kept per stream

    def push(self, blocks: np.ndarray) -> None:
        """One tick: `blocks` is float32 [n_streams, block] (host)."""
        b = np.ascontiguousarray(blocks, dtype=np.float32)
        if b.shape != (self.n_streams, self.block):
            raise ValueError(f"expected blocks of shape {(self.n_streams, self.block)}, got {b.shape}")
        check(self._lib.ewk_push(self._h, b.ctypes.data_as(C.c_void_p), self.block, 0))

    def push_many(self, pcm: np.ndarray) -> None:
        """Several ticks: float32 [n_streams, n_ticks * block] (host)."""
        a = np.ascontiguousarray(pcm, dtype=np.float32)
        if a.ndim != 2 or a.shape[0] != self.n_streams or a.shape[1] % self.block:
            raise ValueError("pcm must be [n_streams, n_ticks*block]")
        nt = a.shape[1] // self.block
        if nt:
            check(self._lib.ewk_push_many(self._h, a.ctypes.data_as(C.c_void_p), a.shape[1], self.block, nt, 0))

    def push_pcm16(self, pcm16: np.ndarray) -> None:
        """Ticks of int16 PCM [n_streams, n_ticks * block] (host), decoded on the device."""
        a = np.ascontiguousarray(pcm16, dtype=np.int16)
        if a.ndim != 2 or a.shape[0] != self.n_streams or a.shape[1] % self.block:
            raise ValueError("pcm16 must be [n_streams, n_ticks*block]")
        nt = a.shape[1] // self.block
        if nt:
            check(self._lib.ewk_push_many_pcm16(self._h, a.ctypes.data_as(C.c_void_p), a.shape[1], self.block,
                                                nt, 0))

    def normalize_events(self, events: np.ndarray) -> list:
        """Level-3 pre-processing of polled events straight from the rings (float64 per event)."""
        ev = np.ascontiguousarray(events, dtype=_lib.EVENT_DTYPE)
        n = len(ev)
        if n == 0:
            return []
        lengths = ev["length"].astype(np.int64)
        out = np.zeros(max(1, int(lengths.sum())), np.float64)
        check(self._lib.ewk_normalize_events(self._h, ev.ctypes.data_as(C.POINTER(_lib.EwkEvent)), n,
                                             out.ctypes.data_as(C.c_void_p), 0))
        offs = np.concatenate([[0], np.cumsum(lengths)[:-1]])
        return [out[o:o + l] for o, l in zip(offs, lengths)]

    def normalize_events_device(self, events: np.ndarray) -> list:
        """normalize_events with the float64 output left in GPU memory: a list of torch
        views on this engine's device (level 3 without the host round trip)."""
        import torch
        ev = np.ascontiguousarray(events, dtype=_lib.EVENT_DTYPE)
        n = len(ev)
        if n == 0:
            return []
        lengths = ev["length"].astype(np.int64)
        out = torch.empty(max(1, int(lengths.sum())), dtype=torch.float64, device=torch.device("cuda", self.gpu))
        check(self._lib.ewk_normalize_events(self._h, ev.ctypes.data_as(C.POINTER(_lib.EwkEvent)), n,
                                             C.c_void_p(out.data_ptr()), _lib.EWK_OUT_DEVICE))
        offs = np.concatenate([[0], np.cumsum(lengths)[:-1]])
        return [out[int(o):int(o) + int(l)] for o, l in zip(offs, lengths)]

    def push_device(self, ptr: int, stride: int, tick_stride: int = 0, n_ticks: int = 1) -> None:
        """Device-resident float32 ticks: stream s, tick t at ptr + 4 * (s * stride + t * tick_stride)."""
        check(self._lib.ewk_push_many(self._h, C.c_void_p(ptr), int(stride), int(tick_stride), int(n_ticks),
                                      _lib.EWK_PUSH_DEVICE))

    def push_device_pcm16(self, ptr: int, stride: int, tick_stride: int = 0, n_ticks: int = 1) -> None:
        """Device-resident int16 PCM ticks (indexing as push_device, 2-byte samples)."""
        check(self._lib.ewk_push_many_pcm16(self._h, C.c_void_p(ptr), int(stride), int(tick_stride), int(n_ticks),
                                            _lib.EWK_PUSH_DEVICE))

    def poll(self, cap: Optional[int] = None, lagged: bool = False) -> np.ndarray:
        """Drain queued events as a structured array (see _lib.EVENT_DTYPE).
        lagged=True: the events of the pushes before the previous lagged poll, without
        waiting for the latest push (pipelined serving; see include/ewk.h)."""
        # a non-lagged poll drains both event banks (each holds up to the engine's queue
        # capacity after a lagged poll), so its default buffer holds two banks
        cap = int(cap or (1 if lagged else 2) * max(4096, 4 * self.n_streams))
        if getattr(self, "_poll_buf", None) is None or len(self._poll_buf) < cap:
            self._poll_buf = np.zeros(cap, dtype=_lib.EVENT_DTYPE)   # reused: polled every tick
            self._poll_n = C.c_int32(0)
        fn = self._lib.ewk_poll_lagged if lagged else self._lib.ewk_poll
        check(fn(self._h, self._poll_buf.ctypes.data_as(C.POINTER(_lib.EwkEvent)), cap, C.byref(self._poll_n)))
        return self._poll_buf[: self._poll_n.value].copy()

    def state(self, stream: int) -> dict:
        st = _lib.EwkStreamState()
        check(self._lib.ewk_get_stream_state(self._h, int(stream), C.byref(st)))
        return {f: getattr(st, f) for f, _ in st._fields_}

    def read_last(self, stream: int, n_samples: int) -> np.ndarray:
        out = np.zeros(max(0, int(n_samples)), np.float32)
        n = C.c_int64(0)
        check(self._lib.ewk_read_last(self._h, int(stream), int(n_samples), _lib.fptr(out), C.byref(n)))
        return out[: n.value]

    def read_segment(self, stream: int, ring_start: int, length: int) -> np.ndarray:
        out = np.zeros(int(length), np.float32)
        check(self._lib.ewk_read_segment(self._h, int(stream), int(ring_start), int(length), _lib.fptr(out)))
        return out

    def reset(self) -> None:
        check(self._lib.ewk_reset_streams(self._h))

    def reenter(self, stream: int = -1, reentry_timeout: float = 0.0) -> None:
        """A new _detect_word call (wakeword.py:1048-1057) on `stream` (-1 = all) and the
        re-entry timeout for later pushes (0 = continuous, > 0 = start() mode)."""
        check(self._lib.ewk_reenter(self._h, int(stream), float(reentry_timeout)))
        self.config.reentry_timeout = float(reentry_timeout)
