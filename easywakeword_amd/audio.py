"""Audio I/O for the drop-in facade: WAV decode and block sources.

``load_wav`` replaces ``librosa.load(path, sr=16000)`` (reference wakeword.py:588,
866-870): PCM16 -> float32 int16/32768 (libsndfile scaling), PCM32 -> /2**31,
8-bit unsigned -> (x-128)/128, channel mean for multi-channel files
(librosa.to_mono).  16 kHz files are bit-exact with librosa.  Other rates are
resampled to 16 kHz on the host with a polyphase Kaiser FIR
(scipy.signal.resample_poly); librosa's default there is soxr 'HQ' (soxr is absent
from this image), so resampled audio is close to, not bit-identical with, the
reference's -- parity unpinned for non-16 kHz files.

Sources replace the PortAudio input stream of SoundBuffer (wakeword.py:438-444):
each yields float32 blocks of ``block`` samples, one per 0.1 s tick.
"""
from __future__ import annotations

import wave
from typing import Iterator, Optional

import numpy as np

FREQUENCY = 16000


def load_wav(path: str, sr: int = FREQUENCY) -> np.ndarray:
    with wave.open(str(path), "rb") as w:
        nch, sw, rate, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if sw == 2:
        x = np.frombuffer(raw, dtype="<i2").astype(np.float32) / np.float32(32768.0)
    elif sw == 4:
        x = (np.frombuffer(raw, dtype="<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
    elif sw == 1:
        x = (np.frombuffer(raw, dtype=np.uint8).astype(np.float32) - np.float32(128.0)) / np.float32(128.0)
    else:
        raise ValueError(f"{path}: unsupported sample width {sw}")
    if nch > 1:
        x = np.mean(x.reshape(-1, nch).T, axis=0).astype(np.float32)
    if rate != sr:
        x = resample(x, rate, sr)
    return np.ascontiguousarray(x, dtype=np.float32)


def resample(x: np.ndarray, orig_sr: int, target_sr: int) -> np.ndarray:
    """Band-limited resampling orig_sr -> target_sr (polyphase FIR, Kaiser beta 5.0),
    float64 internally, float32 out, length ceil(n * target / orig) like librosa."""
    from math import gcd
    from scipy.signal import resample_poly
    if orig_sr <= 0 or target_sr <= 0:
        raise ValueError("sample rates must be positive")
    g = gcd(int(orig_sr), int(target_sr))
    up, down = int(target_sr) // g, int(orig_sr) // g
    y = resample_poly(np.asarray(x, np.float64), up, down, window=("kaiser", 5.0))
    n = int(np.ceil(len(x) * target_sr / orig_sr))
    return y[:n].astype(np.float32)


def write_wav(path: str, audio, sr: int = FREQUENCY) -> None:
    """PCM16 writer with libsndfile's float scaling (x * 32767)."""
    q = np.clip(np.round(np.asarray(audio, np.float64) * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(q.tobytes())


class ArraySource:
    """Blocks from an in-memory float32 signal; zeros after the end (a silent mic)."""

    realtime = False

    def __init__(self, audio, block: int = 1600, loop: bool = False):
        self.audio = np.ascontiguousarray(np.asarray(audio, dtype=np.float32).reshape(-1))
        self.block = int(block)
        self.loop = loop
        self.pos = 0

    def blocks(self) -> Iterator[np.ndarray]:
        while True:
            b = self.read()
            yield b

    def read(self) -> np.ndarray:
        n = self.block
        a = self.audio
        if self.loop and len(a):
            idx = (self.pos + np.arange(n)) % len(a)
            out = a[idx]
        else:
            out = np.zeros(n, np.float32)
            if self.pos < len(a):
                chunk = a[self.pos:self.pos + n]
                out[:len(chunk)] = chunk
        self.pos += n
        return out

    @property
    def exhausted(self) -> bool:
        return not self.loop and self.pos >= len(self.audio)

    def start(self):
        pass

    def stop(self):
        pass


class WavSource(ArraySource):
    def __init__(self, path: str, block: int = 1600, loop: bool = False):
        super().__init__(load_wav(path), block=block, loop=loop)


class MicSource:
    """PortAudio microphone through ``sounddevice`` (only when installed); `device` is a
    PortAudio index -- easywakeword_amd.devices.AudioDeviceManager resolves names and
    the reference's magic words."""

    realtime = True

    def __init__(self, device: Optional[int] = None, block: int = 1600):
        import queue

        import sounddevice as sd  # noqa: F401  (raises ImportError/OSError when absent)
        self._sd = sd
        self.block = int(block)
        self.q: "queue.Queue[np.ndarray]" = queue.Queue()
        self.stream = sd.InputStream(samplerate=FREQUENCY, channels=1, blocksize=self.block, device=device,
                                     callback=lambda indata, frames, t, status: self.q.put(
                                         np.array(indata, dtype=np.float32).reshape(-1).copy()))

    def start(self):
        self.stream.start()

    def stop(self):
        self.stream.stop()

    def read(self) -> np.ndarray:
        return self.q.get()

    exhausted = False
