"""CPU oracle for the level-1 gate (ring + adaptive threshold + timing FSM) --
TEST INFRASTRUCTURE ONLY (imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py; never by the product package).

Restates, on a *virtual clock*, the reference's
  * ``SoundBuffer._add_sound_to_buffer``   wakeword.py:454-470   (ring ingest)
  * ``SoundBuffer._adjust_silence_threshold`` wakeword.py:472-486 (block RMS + pct25)
  * ``SoundBuffer.is_silent`` / ``return_last_n_seconds`` wakeword.py:488-513
  * ``WakeWord._detect_word`` FSM + segment cut  wakeword.py:1048-1118
using numpy exactly as the reference does (float64 ring, ``np.mean``,
``np.percentile``), so every float64 comparison is bit-identical.  The
per-sample Python loop of the reference is replaced by a vectorised copy, which
writes the same values into the same slots.

Virtual clock (shared with the HIP engine and with
``tests/golden/make_golden.py``, which drives the *real* reference code):
tick ``k`` (k = 1, 2, ...) delivers one callback block, then the detector
observes; ``time(k) = float(k) * tick_seconds`` (float64).  Detection starts at
the first tick at which the ring is full (``_wait_for_buffer``); the entry
``is_silent()`` check (wakeword.py:1055-1057) happens at that tick without a
push, and every later tick steps the FSM once (``time.sleep(0.1)`` = one push).
The state after an emitted segment returns to "waiting" whatever the score
(level 3 never confirms in the reference snapshot: SURVEY.md section 0.2), so
the level-1 event stream does not depend on level 2.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

FREQUENCY = 16000
MIN_THRESHOLD = 0.005
INITIAL_THRESHOLD = 0.01

WAITING, IN_SILENCE, IN_SOUND, AFTER_SOUND = 0, 1, 2, 3
STATE_NAMES = {WAITING: "waiting", IN_SILENCE: "in_silence", IN_SOUND: "in_sound", AFTER_SOUND: "after_sound"}


def pairwise_sum_f64(a: np.ndarray) -> float:
    """numpy's float64 add.reduce order for a contiguous 1-D array, written out.

    Chunks of 8192 (ufunc buffer) accumulated sequentially from 0.0; inside a
    chunk: n<8 plain loop; n<=128 eight accumulators + tree + tail; else split
    at n2 = (n//2) - (n//2)%8.  The HIP gate kernel implements this order; the
    tests check this function against ``np.add.reduce`` bit for bit."""
    def pw(x, s, n):
        if n < 8:
            r = 0.0
            for i in range(n):
                r += float(x[s + i])
            return r
        if n <= 128:
            r = [float(x[s + j]) for j in range(8)]
            i = 8
            lim = n - (n % 8)
            while i < lim:
                for j in range(8):
                    r[j] += float(x[s + i + j])
                i += 8
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
            while i < n:
                res += float(x[s + i])
                i += 1
            return res
        n2 = n // 2
        n2 -= n2 % 8
        return pw(x, s, n2) + pw(x, s + n2, n - n2)

    acc = 0.0
    for c in range(0, len(a), 8192):
        acc += pw(a, c, min(8192, len(a) - c))
    return acc


class SoundBufferRef:
    """float64 circular buffer restating reference SoundBuffer (wakeword.py:405-517)."""

    FREQUENCY = FREQUENCY
    MIN_THRESHOLD = MIN_THRESHOLD

    def __init__(self, seconds: int = 10):
        self.buffer_seconds = seconds
        self.buffer_length = seconds * FREQUENCY
        self.data = np.zeros(self.buffer_length)
        self.pointer = 0
        self.frame_size = 0
        self.silence_threshold = INITIAL_THRESHOLD
        self.samples_collected = 0

    def push(self, block: np.ndarray) -> None:
        """_add_sound_to_buffer (wakeword.py:454-470) for one callback block."""
        new = np.asarray(block, dtype=np.float32).astype(np.float64).ravel()
        if self.frame_size == 0:
            self.frame_size = len(new)
        n = len(new)
        L = self.buffer_length
        if n >= L:   # the per-sample loop leaves the last L samples in place
            tail = new[n - L:]
            start = (self.pointer + n - L) % L
            idx = (start + np.arange(L)) % L
            self.data[idx] = tail
        else:
            idx = (self.pointer + np.arange(n)) % L
            self.data[idx] = new
        self.pointer = (self.pointer + n) % L
        self.samples_collected = min(self.samples_collected + n, L)
        if self.samples_collected < L:
            return
        self._adjust_silence_threshold()

    def _adjust_silence_threshold(self) -> None:
        if self.frame_size == 0:
            return
        num_frames = len(self.data) // self.frame_size
        all_rms = []
        for i in range(num_frames):
            frame = self.data[i * self.frame_size:(i + 1) * self.frame_size]
            all_rms.append(np.sqrt(np.mean(frame ** 2)))
        if all_rms:
            new_threshold = np.percentile(all_rms, 25) * 1.5
            self.silence_threshold = max(new_threshold, self.MIN_THRESHOLD)

    def block_rms(self) -> np.ndarray:
        fs = self.frame_size
        nb = len(self.data) // fs
        return np.array([np.sqrt(np.mean(self.data[i * fs:(i + 1) * fs] ** 2)) for i in range(nb)])

    def last_rms(self) -> float:
        recent = self.return_last_n_seconds(0.1)
        return float(np.sqrt(np.mean(recent ** 2)))

    def is_silent(self) -> bool:
        if len(self.data) == 0 or self.frame_size == 0:
            return True
        recent = self.return_last_n_seconds(0.1)
        if len(recent) == 0:
            return True
        rms = np.sqrt(np.mean(recent ** 2))
        return bool(rms < self.silence_threshold)

    def return_last_n_seconds(self, n: float) -> np.ndarray:
        n_samples = int(n * self.FREQUENCY)
        if n_samples > len(self.data):
            n_samples = len(self.data)
        if n_samples == 0:
            return np.array([])
        start = (self.pointer - n_samples) % self.buffer_length
        if start < self.pointer:
            return self.data[start:self.pointer].copy()
        return np.concatenate((self.data[start:], self.data[:self.pointer])).copy()

    def is_buffer_full(self) -> bool:
        return self.samples_collected >= self.buffer_length


@dataclass
class GateConfig:
    pre_speech_silence: float = 0.8
    speech_duration_min: float = 0.3
    speech_duration_max: float = 2.0
    post_speech_silence: float = 0.4
    buffer_seconds: int = 10
    block: int = 1600
    tick_seconds: float = 0.1
    padding: float = 0.05
    max_segment_seconds: float = 3.0
    # start()-mode quirk (wakeword.py:1061-1062, 1202-1211): when set, a
    # TimeoutError re-enters _detect_word every `reentry_timeout` seconds,
    # resetting the FSM through the entry is_silent() check.  None = continuous.
    reentry_timeout: Optional[float] = None


@dataclass
class SegmentEvent:
    tick: int                 # virtual tick at which level 1 passed
    time: float               # float64 virtual time of that tick
    n_request: int            # int(abs(extract_start) * 16000), capped at the ring length
    end_trim: int             # word_end_idx = int(abs(extract_end) * 16000)
    length: int               # len(word_audio)
    skipped: bool             # True when len/16000 > 3.0 (no level-2 call)
    audio: Optional[np.ndarray] = field(default=None, repr=False)


def slice_stop(length: int, trim: int) -> int:
    """Python's ``a[: length - trim]`` stop, resolved to a count."""
    stop = length - trim
    if stop < 0:
        stop = max(0, length + stop)
    return min(stop, length)


class DetectorRef:
    """Restates WakeWord._detect_word (wakeword.py:1036-1159) on the virtual clock,
    running continuously (level 3 absent -> every emitted segment returns to waiting)."""

    def __init__(self, cfg: GateConfig, keep_audio: bool = True):
        self.cfg = cfg
        self.buf = SoundBufferRef(cfg.buffer_seconds)
        self.keep_audio = keep_audio
        self.tick = 0
        self.started = False
        self.state = WAITING
        self.silence_start = None
        self.sound_start = None
        self.sound_end = None
        self.events: List[SegmentEvent] = []
        self.silent_trace: List[bool] = []
        self.start_time = None
        self.reentries = 0

    def now(self) -> float:
        return float(self.tick) * self.cfg.tick_seconds

    def _enter(self) -> None:
        """Entry of _detect_word (wakeword.py:1048-1057)."""
        self.state = WAITING
        self.start_time = self.now()
        if self.buf.is_silent():
            self.state = IN_SILENCE
            self.silence_start = self.now()

    def push_tick(self, block: np.ndarray) -> Optional[SegmentEvent]:
        if (self.started and self.cfg.reentry_timeout is not None
                and self.now() - self.start_time > self.cfg.reentry_timeout):
            self.reentries += 1
            self._enter()
        self.tick += 1
        self.buf.push(block)
        if not self.started:
            if self.buf.is_buffer_full():
                self.started = True
                self._enter()
            return None
        return self._step()

    def _step(self) -> Optional[SegmentEvent]:
        cfg = self.cfg
        silent = self.buf.is_silent()
        self.silent_trace.append(silent)
        t = self.now()
        st = self.state
        if st == WAITING:
            if silent:
                self.state = IN_SILENCE
                self.silence_start = t
        elif st == IN_SILENCE:
            if not silent:
                if t - self.silence_start >= cfg.pre_speech_silence:
                    self.state = IN_SOUND
                    self.sound_start = t
                else:
                    self.state = WAITING
        elif st == IN_SOUND:
            d = t - self.sound_start
            if not silent:
                if d > cfg.speech_duration_max:
                    self.state = WAITING
            else:
                if cfg.speech_duration_min <= d <= cfg.speech_duration_max:
                    self.state = AFTER_SOUND
                    self.sound_end = t
                else:
                    self.state = WAITING
        elif st == AFTER_SOUND:
            if silent:
                if t - self.sound_end >= cfg.post_speech_silence:
                    ev = self._cut(t)
                    self.state = WAITING
                    return ev
            else:
                self.state = WAITING
        return None

    def _cut(self, t: float) -> SegmentEvent:
        cfg = self.cfg
        extract_start = self.sound_start - t - cfg.padding
        extract_end = self.sound_end - t + cfg.padding
        samples = self.buf.return_last_n_seconds(abs(extract_start))
        n_req = len(samples)
        e = int(abs(extract_end) * FREQUENCY)
        stop = slice_stop(len(samples), e)
        audio = samples[:stop]
        skipped = (len(audio) / FREQUENCY) > cfg.max_segment_seconds
        ev = SegmentEvent(self.tick, t, n_req, e, len(audio), skipped,
                          audio if self.keep_audio else None)
        self.events.append(ev)
        return ev


def run_stream(pcm: np.ndarray, cfg: GateConfig, keep_audio: bool = True) -> DetectorRef:
    """Feed a whole float32 stream through the gate in ``cfg.block`` callbacks."""
    det = DetectorRef(cfg, keep_audio=keep_audio)
    nb = len(pcm) // cfg.block
    for k in range(nb):
        det.push_tick(pcm[k * cfg.block:(k + 1) * cfg.block])
    return det


def normalize_level3(audio: np.ndarray) -> np.ndarray:
    """WakeWord._transcribe_audio's input normalisation (wakeword.py:1019-1025) on the
    float64 segment: remove the mean, scale to max |y| = 1 when non-zero, x1.5, clip."""
    a = np.asarray(audio, dtype=np.float64)
    a = a - np.mean(a)
    max_val = np.max(np.abs(a))
    if max_val > 0:
        a = a / max_val
    a = a * 1.5
    return np.clip(a, -1.0, 1.0)
