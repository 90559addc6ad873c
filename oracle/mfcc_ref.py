"""CPU oracle for the level-2 matcher (MFCC + cosine) -- TEST INFRASTRUCTURE ONLY.

This module is the *checker* for the HIP segment scorer.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it.  The product path (``easywakeword_amd``) never imports or calls it.

What it restates
----------------
``WordMatcher.extract_mfcc`` (reference ``easywakeword/wakeword.py:544-567``)
calls ``librosa.feature.mfcc(y, sr=16000, n_mfcc=20, n_fft=512,
hop_length=160)``.  librosa is a third-party dependency that is *absent* from
``/root/reference`` and from this image; its pinned version is **librosa
0.11.0** (``uv.lock:324-325``).  This file restates the published librosa
0.11.0 algorithm for exactly those arguments:

* ``stft``: periodic Hann window (``scipy.signal.get_window('hann', 512,
  fftbins=True)``), ``center=True`` with ``pad_mode="constant"`` (256 zeros on
  each side), hop 160, ``T = 1 + len(y)//160`` frames.  The window is float64;
  the windowed frame is float64 and the rfft runs in float64; the result is
  stored as complex64 for float32 input and complex128 for float64 input
  (``util.dtype_r2c``).
* power spectrogram ``|X|**2`` (dtype of the stft's real part).
* Slaney mel filterbank ``filters.mel(sr=16000, n_fft=512, n_mels=128,
  fmin=0, fmax=8000, htk=False, norm="slaney", dtype=float32)`` projected with
  ``np.einsum("...ft,mf->...mt", S, mel_basis, optimize=True)``.
* ``power_to_db(ref=1.0, amin=1e-10, top_db=80.0)`` -- the ``top_db`` clamp is
  against the max of the *whole segment*.
* ``scipy.fft.dct(type=2, norm="ortho", axis=-2)[:20]``.

``scipy`` (1.15.3) and ``numpy`` (2.2.6) are the reference's own pinned
dependencies (``uv.lock:474-479, 726-731``) and are used directly, not
restated: ``scipy.fft.dct``, ``scipy.signal.get_window`` and
``scipy.spatial.distance.cosine``.

Parity pinning (see ``tests/test_oracle_pinning.py``): librosa itself cannot be
run here, so a6 is pinned by the reference's own tests (self-match == 100.0,
880 Hz / noise < 100, half-amplitude > 50, 20 finite coefficients --
``tests/test_wakeword_simulated.py:104-205, 347-360`` and
``tests/test_cross_platform.py:69-109``) and by the observations published at
``LEARNINGS.md:92-94`` (880 Hz ~89 %, noise ~77 %, silence NaN).
"""
from __future__ import annotations

import numpy as np
import scipy.fft
import scipy.signal
from scipy.spatial.distance import cosine

SAMPLE_RATE = 16000
N_FFT = 512
HOP = 160
N_MELS = 128
N_MFCC = 20
TOP_DB = 80.0
AMIN = 1e-10


# --- librosa.filters.mel (Slaney) ------------------------------------------------
def _hz_to_mel(freq):
    """librosa.core.convert.hz_to_mel, htk=False (Slaney scale)."""
    freq = np.asanyarray(freq, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = freq / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if freq.ndim:
        log_t = freq >= min_log_hz
        mels[log_t] = min_log_mel + np.log(freq[log_t] / min_log_hz) / logstep
    elif freq >= min_log_hz:
        mels = min_log_mel + np.log(freq / min_log_hz) / logstep
    return mels


def _mel_to_hz(mels):
    """librosa.core.convert.mel_to_hz, htk=False."""
    mels = np.asanyarray(mels, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * mels
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    log_t = mels >= min_log_mel
    freqs[log_t] = min_log_hz * np.exp(logstep * (mels[log_t] - min_log_mel))
    return freqs


def mel_filterbank(sr: int = SAMPLE_RATE, n_fft: int = N_FFT, n_mels: int = N_MELS) -> np.ndarray:
    """Restates librosa.filters.mel(sr, n_fft, n_mels, fmin=0, fmax=sr/2,
    htk=False, norm='slaney', dtype=float32) -> float32 [n_mels, 1+n_fft//2].

    Note the double rounding librosa performs: each triangle row is assigned
    into a float32 array, then ``weights *= enorm`` multiplies float32 by a
    float64 vector in place (computed in float64, stored float32)."""
    fmax = float(sr) / 2
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    min_mel = _hz_to_mel(0.0)
    max_mel = _hz_to_mel(fmax)
    mel_f = _mel_to_hz(np.linspace(min_mel, max_mel, n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


_MEL = None
_WIN = None


def _tables():
    global _MEL, _WIN
    if _MEL is None:
        _MEL = mel_filterbank()
        _WIN = scipy.signal.get_window("hann", N_FFT, fftbins=True)  # float64
    return _MEL, _WIN


def hann_window() -> np.ndarray:
    return _tables()[1].copy()


# --- librosa.stft / melspectrogram / power_to_db / mfcc ---------------------------
def n_frames(n_samples: int) -> int:
    """Frames produced by stft(center=True, n_fft=512, hop=160)."""
    return 1 + int(n_samples) // HOP


def frames(y: np.ndarray) -> np.ndarray:
    """[T, 512] frames of the zero-padded signal (center=True, constant pad)."""
    pad = np.zeros(len(y) + N_FFT, dtype=y.dtype)
    pad[N_FFT // 2:N_FFT // 2 + len(y)] = y
    T = n_frames(len(y))
    idx = np.arange(T)[:, None] * HOP + np.arange(N_FFT)[None, :]
    return pad[idx]


def power_spectrogram(y: np.ndarray) -> np.ndarray:
    """|stft|**2 as [257, T] in the stft's real dtype (float32 for float32 y)."""
    _, win = _tables()
    fr = frames(y)                               # [T, 512] in y.dtype
    spec = np.fft.rfft(win[None, :] * fr, axis=-1)   # float64 product, complex128 fft
    cdt = np.complex64 if y.dtype == np.float32 else np.complex128
    spec = spec.astype(cdt).T                    # librosa stores into the r2c dtype
    return np.abs(spec) ** 2.0


def log_mel(y: np.ndarray) -> np.ndarray:
    """power_to_db(melspectrogram(y)) -> [128, T] (top_db clamp applied)."""
    mel_basis, _ = _tables()
    S = power_spectrogram(y)
    melspec = np.einsum("...ft,mf->...mt", S, mel_basis, optimize=True)
    log_spec = 10.0 * np.log10(np.maximum(AMIN, melspec))
    log_spec -= 10.0 * np.log10(np.maximum(AMIN, 1.0))
    log_spec = np.maximum(log_spec, log_spec.max() - TOP_DB)
    return log_spec


def mfcc(y: np.ndarray) -> np.ndarray:
    """librosa.feature.mfcc(y, sr=16000, n_mfcc=20, n_fft=512, hop_length=160) -> [20, T]."""
    y = np.asarray(y)
    if y.dtype not in (np.float32, np.float64):
        y = y.astype(np.float32)
    S = log_mel(y)
    return scipy.fft.dct(S, axis=-2, type=2, norm="ortho")[..., :N_MFCC, :]


def extract_mfcc(y: np.ndarray):
    """WordMatcher.extract_mfcc (wakeword.py:544-567): mean and population std over time."""
    m = mfcc(y)
    return np.mean(m, axis=1), np.std(m, axis=1)


def similarity_from_stats(ref_mean, ref_std, cand_mean, cand_std):
    """WordMatcher.calculate_similarity (wakeword.py:591-625) on precomputed stats."""
    with np.errstate(all="ignore"):
        sim_mean = 1 - cosine(ref_mean, cand_mean)
        sim_std = 1 - cosine(ref_std, cand_std)
        combined = sim_mean * 0.7 + sim_std * 0.3
        percent = combined * 100
        return percent ** 1.5 / (100 ** 0.5)


class WordMatcherRef:
    """Oracle twin of the reference ``WordMatcher`` (wakeword.py:520-639)."""

    def __init__(self, sample_rate: int = SAMPLE_RATE):
        self.sample_rate = sample_rate
        self.reference_mfcc_mean = None
        self.reference_mfcc_std = None
        self.reference_word = None

    def set_reference(self, audio, word_name="target"):
        self.reference_word = word_name
        self.reference_mfcc_mean, self.reference_mfcc_std = extract_mfcc(audio)

    def calculate_similarity(self, audio) -> float:
        if self.reference_mfcc_mean is None:
            raise ValueError("No reference word set. Call set_reference() first.")
        cm, cs = extract_mfcc(audio)
        return similarity_from_stats(self.reference_mfcc_mean, self.reference_mfcc_std, cm, cs)

    def matches(self, audio, threshold: float = 75.0):
        s = self.calculate_similarity(audio)
        return s >= threshold, s


# --- librosa.load for 16 kHz PCM16 WAV ----------------------------------------
def load_wav_pcm16(path: str) -> np.ndarray:
    """librosa.load(path, sr=16000) for a 16 kHz PCM16 file: float32 int16/32768,
    channel mean for multi-channel input (soundfile + librosa.to_mono)."""
    import wave
    with wave.open(str(path), "rb") as w:
        nch, sw, sr, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if sw != 2 or sr != SAMPLE_RATE:
        raise ValueError(f"oracle loader supports 16 kHz PCM16 only (got sw={sw}, sr={sr})")
    x = np.frombuffer(raw, dtype="<i2").astype(np.float32) / np.float32(32768.0)
    if nch > 1:
        x = np.mean(x.reshape(-1, nch).T, axis=0)
    return x


def rms_frames(y: np.ndarray, frame_length: int = 400, hop_length: int = 160) -> np.ndarray:
    """librosa.feature.rms(y, frame_length, hop_length) (center=True, constant pad) -> [1, T]."""
    y = np.asarray(y)
    pad = np.pad(y, (frame_length // 2, frame_length // 2), mode="constant")
    T = 1 + (len(pad) - frame_length) // hop_length
    idx = np.arange(T)[:, None] * hop_length + np.arange(frame_length)[None, :]
    x = pad[idx].T                                   # [frame_length, T]
    power = np.mean(np.abs(x) ** 2, axis=-2, keepdims=True)
    return np.sqrt(power)
