"""Drop-in facade of the reference API on the MI355X engine.

Mirrors ``easywakeword/wakeword.py`` of the reference:

* ``WordMatcher``  (wakeword.py:520-639)  -- set_reference / load_reference_from_file /
  extract_mfcc / calculate_similarity / matches, computed by the HIP scorer.
* ``SoundBuffer``  (wakeword.py:405-517)  -- the duck-typed buffer protocol
  (is_buffer_full / is_silent / return_last_n_seconds / start / stop) backed by
  a one-stream GPU engine fed from an audio source.
* ``WakeWord``     (wakeword.py:642-1240) -- waitforit() / start() / stop() /
  is_listening() / check_transcriber_health(), same constructor, same
  ValueError / TimeoutError conventions, callback on a background thread.

Level 1 (ring, adaptive threshold, timing FSM) and level 2 (MFCC + cosine) run
on the GPU through libewk.so; there is no CPU fallback.  Level 3 (Whisper) is an
optional ``confirm`` callable: the reference's own level 3 can never confirm
(its ``transcribe(..., initial_prompt=)`` call raises TypeError that is swallowed,
SURVEY.md section 0.2), so without ``confirm`` a level-2 match is the detection.

Time is the engine's virtual clock (tick * 0.1 s, one 1600-sample block per
tick): a WAV or array source runs faster than real time
with the same decisions a live microphone would give at 0.1 s polling.
"""
from __future__ import annotations

import logging
import threading
from typing import Callable, Dict, Optional, Tuple, Union

import numpy as np

from . import audio as _audio
from .engine import Engine, StreamEngine

logger = logging.getLogger(__name__)

DEFAULT_BUFFER_SECONDS = 10
DEFAULT_RETRY_COUNT = 3
DEFAULT_RETRY_BACKOFF = 0.5
DEFAULT_PRE_SPEECH_SILENCE = 0.8
DEFAULT_SPEECH_DURATION_MIN = 0.3
DEFAULT_SPEECH_DURATION_MAX = 2.0
DEFAULT_POST_SPEECH_SILENCE = 0.4
AUTO_CALCULATE = None
VOICE_ACTIVITY_THRESHOLD = 0.1
MIN_DETECTED_DURATION = 0.2
FREQUENCY = 16000
BLOCK = 1600


class WordMatcher:
    """MFCC + cosine matcher (reference wakeword.py:520-639) on the GPU scorer.

    ``extract_mfcc`` returns the mean/std of librosa-equivalent MFCCs (n_mfcc=20,
    n_fft=512, hop=160) in the input's dtype like the reference: float32 input on the
    fp32 scorer, float64 input on the device's fp64 path (k_score_f64, within 1e-9 of
    the float64 reference).  ``calculate_similarity`` / ``matches`` score on the fp32
    scorer (within 1e-4 of the reference; a score within ``rescore_margin`` of the
    threshold is re-scored in float64 on the device, so decisions are exact).

    A matcher built with ``engine=`` shares that engine; ``matches(audio, threshold)``
    applies its threshold for that call only and restores the engine's afterwards."""

    def __init__(self, sample_rate: int = FREQUENCY, gpu: int = 0, engine: Optional[Engine] = None) -> None:
        if sample_rate != FREQUENCY:
            raise ValueError("only 16 kHz audio is supported")
        self.sample_rate = sample_rate
        self.reference_mfcc_mean: Optional[np.ndarray] = None
        self.reference_mfcc_std: Optional[np.ndarray] = None
        self.reference_word: Optional[str] = None
        self._engine = engine if engine is not None else Engine(gpu=gpu)

    @property
    def engine(self) -> Engine:
        return self._engine

    def extract_mfcc(self, audio: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        a = np.asarray(audio)
        if a.dtype == np.float64:   # the reference's float64 candidate path (wakeword.py:544-567)
            m, s, _ = self._engine.score_f64([a])
            return m[0], s[0]
        m, s, _, _ = self._engine.score([audio], require_template=False)
        return m[0], s[0]

    def set_reference(self, audio: np.ndarray, word_name: str = "target") -> None:
        self.reference_word = word_name
        self._engine.template_from_pcm(audio)
        self.reference_mfcc_mean, self.reference_mfcc_std = self._engine.get_template()

    def load_reference_from_file(self, filepath: str, word_name: str = "target") -> None:
        self.set_reference(_audio.load_wav(filepath, sr=self.sample_rate), word_name)

    def _sync_template(self) -> None:
        if self.reference_mfcc_mean is None:
            raise ValueError("No reference word set. Call set_reference() first.")
        # attributes may have been assigned directly (as the reference allows)
        m, s = self._engine.get_template() if self._has_engine_template() else (None, None)
        if m is None or not (np.array_equal(m, np.asarray(self.reference_mfcc_mean, np.float32))
                             and np.array_equal(s, np.asarray(self.reference_mfcc_std, np.float32))):
            self._engine.set_template(self.reference_mfcc_mean, self.reference_mfcc_std)

    def _has_engine_template(self) -> bool:
        try:
            self._engine.get_template()
            return True
        except ValueError:
            return False

    def calculate_similarity(self, audio: np.ndarray) -> float:
        self._sync_template()
        _, _, score, _ = self._engine.score([audio])
        return float(score[0])

    def _score_at(self, segments, threshold: float):
        """Score with `threshold` for this call only (a shared engine keeps its own)."""
        self._sync_template()
        old = self._engine.config.similarity_threshold
        if float(threshold) == old:
            return self._engine.score(segments)
        self._engine.set_threshold(threshold)
        try:
            return self._engine.score(segments)
        finally:
            self._engine.set_threshold(old)

    def matches(self, audio: np.ndarray, threshold: float = 75.0) -> Tuple[bool, float]:
        _, _, score, match = self._score_at([audio], threshold)
        return bool(match[0]), float(score[0])

    def matches_batch(self, segments, threshold: float = 75.0):
        """Many candidates in one launch: (matches[n] bool, scores[n] float64)."""
        _, _, score, match = self._score_at(segments, threshold)
        return match, score


class SoundBuffer:
    """The reference SoundBuffer protocol (wakeword.py:405-517) on a 1-stream
    GPU engine.  ``source`` replaces the PortAudio InputStream; ``pump()``
    delivers one callback block (what PortAudio does every 0.1 s)."""

    FREQUENCY = FREQUENCY
    MIN_THRESHOLD = 0.005

    def __init__(self, seconds: int = DEFAULT_BUFFER_SECONDS, device=None, source=None,
                 engine: Optional[StreamEngine] = None, gpu: int = 0, **cfg):
        self.buffer_seconds = seconds
        self.buffer_length = seconds * FREQUENCY
        if source is None:
            source = _default_source(device)
        self.source = source
        self.engine = engine or StreamEngine(1, gpu=gpu, buffer_seconds=seconds, block=source.block, **cfg)
        self.source.start()

    def pump(self) -> np.ndarray:
        blk = self.source.read()
        self.engine.push(np.asarray(blk, np.float32).reshape(1, -1))
        return blk

    def start(self) -> None:
        self.source.start()

    def stop(self) -> None:
        self.source.stop()

    @property
    def silence_threshold(self) -> float:
        return self.engine.state(0)["silence_threshold"]

    def is_buffer_full(self) -> bool:
        return self.engine.state(0)["samples_collected"] >= self.buffer_length

    def is_silent(self) -> bool:
        st = self.engine.state(0)
        if st["tick"] == 0:
            return True
        return bool(st["last_silent"])

    def return_last_n_seconds(self, n: float) -> np.ndarray:
        n_samples = int(n * self.FREQUENCY)
        if n_samples > self.buffer_length:
            n_samples = self.buffer_length
        if n_samples == 0:
            return np.array([])
        return self.engine.read_last(0, n_samples).astype(np.float64)


def _default_source(device):
    """The microphone `device` names (None, index, name pattern, "default"/"best"/"first"),
    resolved like the reference's AudioDeviceManager.select_device (wakeword.py:128-185,
    437); an unmatched spec raises ValueError instead of falling back to the default mic."""
    from .devices import AudioDeviceManager, NoInputDeviceError
    try:
        index = AudioDeviceManager.select_device(device)
        return _audio.MicSource(device=index, block=BLOCK)
    except (ImportError, OSError, NoInputDeviceError) as exc:   # a spec matching nothing stays ValueError
        raise OSError("no audio input available (sounddevice/PortAudio missing); "
                      "pass source=ArraySource(...) or WavSource(...)") from exc


def normalize_for_transcription(audio_samples: np.ndarray, engine=None) -> np.ndarray:
    """_transcribe_audio's pre-processing (wakeword.py:1019-1025) on the GPU:
    x - mean, / max|.| if > 0, * 1.5, clip [-1, 1], float64 as numpy computes it."""
    from .engine import Engine
    eng = engine if engine is not None else Engine()
    return eng.normalize([np.asarray(audio_samples)])[0]


class WakeWord:
    """Wake word detector (reference wakeword.py:642-1240) on the MI355X engine.

    Extra keyword-only arguments (not in the reference):
      source  -- audio source (ArraySource / WavSource / MicSource); default: microphone
      gpu     -- HIP device index
      confirm -- optional level-3 callable(audio float64 normalised) -> str | None
    """

    def __init__(
        self,
        textword: str,
        wavword: str,
        numberofwords: int = 2,
        timeout: int = 30,
        callback: Optional[Callable[[str], None]] = None,
        device: Optional[Union[int, str]] = None,
        similarity_threshold: float = 75.0,
        pre_speech_silence: float = DEFAULT_PRE_SPEECH_SILENCE,
        speech_duration_min: Optional[float] = AUTO_CALCULATE,
        speech_duration_max: Optional[float] = AUTO_CALCULATE,
        post_speech_silence: float = DEFAULT_POST_SPEECH_SILENCE,
        buffer_seconds: int = DEFAULT_BUFFER_SECONDS,
        verbose: bool = False,
        retry_count: int = DEFAULT_RETRY_COUNT,
        retry_backoff: float = DEFAULT_RETRY_BACKOFF,
        external_whisper_url: Optional[str] = None,
        stt_backend: str = "bundled",
        session_headers: Optional[Dict[str, str]] = None,
        *,
        source=None,
        gpu: int = 0,
        confirm: Optional[Callable[[np.ndarray], Optional[str]]] = None,
    ):
        # parameter validation: same order and messages as wakeword.py:744-763
        if numberofwords < 1:
            raise ValueError("numberofwords must be at least 1")
        if buffer_seconds <= 0:
            raise ValueError("buffer_seconds must be positive")
        if retry_count < 0:
            raise ValueError("retry_count must be non-negative")
        if retry_backoff < 0:
            raise ValueError("retry_backoff must be non-negative")
        if pre_speech_silence <= 0:
            raise ValueError("pre_speech_silence must be positive")
        if speech_duration_min is not None and speech_duration_min <= 0:
            raise ValueError("speech_duration_min must be positive")
        if speech_duration_max is not None and speech_duration_max <= 0:
            raise ValueError("speech_duration_max must be positive")
        if (speech_duration_min is not None and speech_duration_max is not None
                and speech_duration_min > speech_duration_max):
            raise ValueError("speech_duration_min must be <= speech_duration_max")
        if post_speech_silence <= 0:
            raise ValueError("post_speech_silence must be positive")

        self.textword = textword.lower().strip()
        self.wavword = wavword
        self.numberofwords = numberofwords
        self.timeout = timeout
        self.callback = callback
        self.device = device
        self.similarity_threshold = similarity_threshold
        self.buffer_seconds = buffer_seconds
        self.verbose = verbose
        self.retry_count = retry_count
        self.retry_backoff = retry_backoff
        self.external_whisper_url = external_whisper_url
        self.stt_backend = stt_backend
        self.session_headers = session_headers
        self._user_speech_duration_min = speech_duration_min
        self._user_speech_duration_max = speech_duration_max
        self.pre_speech_silence = pre_speech_silence
        self.post_speech_silence = post_speech_silence
        self._auto_calculate_speech_durations()

        self._source = source
        self._gpu = gpu
        self._confirm = confirm
        self._sound_buffer: Optional[SoundBuffer] = None
        self._matcher: Optional[WordMatcher] = None
        self._listening = False
        self._listen_thread: Optional[threading.Thread] = None
        self._stop_event = threading.Event()
        self._log(f"Initialized WakeWord detector for '{self.textword}'")

    # ---- helpers kept from the reference -----------------------------------
    def _log(self, message: str, level: int = logging.DEBUG) -> None:
        if self.verbose:
            logger.log(level, message)

    def check_transcriber_health(self) -> Dict[str, Union[bool, str, float]]:
        return {"healthy": True, "model_loaded": self._confirm is not None,
                "backend": "confirm_callable" if self._confirm is not None else "mfcc_only"}

    def _analyze_reference_audio_duration(self) -> Optional[float]:
        """RMS voice-activity duration of the reference WAV (wakeword.py:854-898):
        librosa.feature.rms(frame 400, hop 160, centred, zero pad) > 0.1 x max,
        (last - first) * 160 / 16000, at least 0.2 s."""
        try:
            audio = _audio.load_wav(self.wavword)
            frame_length, hop_length = int(0.025 * FREQUENCY), int(0.010 * FREQUENCY)
            pad = np.pad(audio, (frame_length // 2, frame_length // 2), mode="constant")
            T = 1 + (len(pad) - frame_length) // hop_length
            idx = np.arange(T)[:, None] * hop_length + np.arange(frame_length)[None, :]
            rms = np.sqrt(np.mean(np.abs(pad[idx].T) ** 2, axis=-2))
            threshold = np.max(rms) * VOICE_ACTIVITY_THRESHOLD
            voice = np.where(rms > threshold)[0]
            if voice.size:
                duration = (voice[-1] - voice[0]) * hop_length / FREQUENCY
                return max(duration, MIN_DETECTED_DURATION)
        except Exception as e:  # noqa: BLE001 - reference swallows and logs
            self._log(f"Could not analyze reference audio duration: {e}", logging.WARNING)
        return None

    def _auto_calculate_speech_durations(self) -> None:
        """Called by the reference constructor (wakeword.py:786) but missing from
        the snapshot; behaviour pinned by tests/test_wakeword_simulated.py:687-775:
        min = analysed WAV speech duration (fallback 0.3), max = 2 x min unless the
        user gave one (fallback 2.0)."""
        user_min = getattr(self, "_user_speech_duration_min", None)
        user_max = getattr(self, "_user_speech_duration_max", None)
        d = None   # the WAV is analysed once, and only when a default needs it
        if user_min is not None:
            smin = float(user_min)
        else:
            d = self._analyze_reference_audio_duration()
            smin = float(d) if d is not None else DEFAULT_SPEECH_DURATION_MIN
        if user_max is not None:
            smax = float(user_max)
        elif user_min is None and d is None:   # no duration in the WAV: both fallbacks
            smax = DEFAULT_SPEECH_DURATION_MAX
        else:
            smax = 2.0 * smin
        if smax < smin:
            smax = smin
        self.speech_duration_min = smin
        self.speech_duration_max = smax

    def _set_thresholds_from_audio_duration(self, audio_duration: float) -> None:
        if getattr(self, "pre_speech_silence", None) is None:
            self.pre_speech_silence = max(0.8, audio_duration * 0.8)
        if getattr(self, "speech_duration_min", None) is None:
            self.speech_duration_min = max(0.3, audio_duration * 0.6)
        if getattr(self, "speech_duration_max", None) is None:
            self.speech_duration_max = min(3.0, audio_duration * 1.8)
        if getattr(self, "post_speech_silence", None) is None:
            self.post_speech_silence = max(0.3, audio_duration * 0.4)

    def _calculate_detection_thresholds(self) -> None:
        if (self.pre_speech_silence is not None and self.speech_duration_min is not None
                and self.speech_duration_max is not None and self.post_speech_silence is not None):
            return
        d = self._analyze_reference_audio_duration()
        if d is not None:
            self._set_thresholds_from_audio_duration(d)
        else:
            self._set_thresholds_from_text_heuristics()

    def _set_thresholds_from_text_heuristics(self) -> None:
        est = self._estimate_syllables(self.textword.lower()) * 0.3
        self._set_thresholds_from_audio_duration(max(0.5, min(2.5, est)))

    @staticmethod
    def _estimate_syllables(text: str) -> int:
        words = "".join(c for c in text if c.isalnum() or c.isspace()).split()
        total = 0
        for word in words:
            word = word.lower().strip()
            if not word:
                continue
            count, prev = 0, False
            for ch in word:
                v = ch in "aeiouy"
                if v and not prev:
                    count += 1
                prev = v
            count = max(1, count)
            if word.endswith("e"):
                count = max(1, count - 1)
            if word.endswith(("es", "ed")) and len(word) > 2:
                count = max(1, count - 1)
            total += count
        return max(1, total)

    # ---- engine plumbing ----------------------------------------------------
    def _gate_config(self, reentry: bool) -> dict:
        return dict(buffer_seconds=int(self.buffer_seconds), block=BLOCK,
                    pre_speech_silence=float(self.pre_speech_silence),
                    speech_duration_min=float(self.speech_duration_min),
                    speech_duration_max=float(self.speech_duration_max),
                    post_speech_silence=float(self.post_speech_silence),
                    similarity_threshold=float(self.similarity_threshold),
                    reentry_timeout=float(self.timeout) if reentry else 0.0)

    def _initialize_audio(self, reentry: bool = False) -> None:
        """Buffer + matcher on first use; every call is a new _detect_word entry
        (wakeword.py:1048-1057) in the mode of its caller: waitforit() continuous,
        start() with the re-entry timeout."""
        if self._sound_buffer is None:
            src = self._source if self._source is not None else _default_source(self.device)
            self._sound_buffer = SoundBuffer(self.buffer_seconds, source=src, gpu=self._gpu,
                                             **{k: v for k, v in self._gate_config(reentry).items()
                                                if k not in ("buffer_seconds", "block")})
        else:
            self._sound_buffer.engine.reenter(0, float(self.timeout) if reentry else 0.0)
        if self._matcher is None:
            # its own scorer engine: matches(threshold=...) must not move the stream's threshold
            self._matcher = WordMatcher(sample_rate=FREQUENCY, gpu=self._gpu)
            self._matcher.load_reference_from_file(self.wavword, self.textword)
            self._sound_buffer.engine.set_template(self._matcher.reference_mfcc_mean,
                                                   self._matcher.reference_mfcc_std)

    def _wait_for_buffer(self) -> None:
        while not self._sound_buffer.is_buffer_full():
            if self._stop_event.is_set():
                return
            self._sound_buffer.pump()

    def _transcribe_audio(self, audio_samples: np.ndarray) -> Optional[str]:
        if self._confirm is None:
            return None
        try:
            return self._confirm(normalize_for_transcription(audio_samples, self._sound_buffer.engine))
        except Exception as e:  # noqa: BLE001 - reference swallows (wakeword.py:1032-1034)
            self._log(f"Transcription failed: {e}", logging.ERROR)
            return None

    def _check_transcription(self, transcription: Optional[str]) -> Optional[str]:
        """Level-3 word checks (wakeword.py:1129-1153)."""
        if not transcription:
            return None
        clean = transcription.strip().lower().rstrip(".,!?;:")
        words = clean.split()
        if len(words) != self.numberofwords:
            return None
        if all(w in words for w in self.textword.split()):
            return transcription
        return None

    def _handle_events(self, events) -> Optional[str]:
        for ev in events:
            if ev["flags"] & 1:   # too long: skipped (wakeword.py:1113-1118)
                continue
            self._log(f"MFCC similarity: {ev['score']:.1f}%")
            if not ev["match"]:
                continue
            if self._confirm is None:
                return self.textword
            audio = self._sound_buffer.engine.read_segment(0, int(ev["ring_start"]), int(ev["length"]))
            res = self._check_transcription(self._transcribe_audio(audio))
            if res:
                return res
        return None

    def _detect_word(self) -> Optional[str]:
        """Tick loop (wakeword.py:1036-1159) on the GPU engine's virtual clock."""
        eng = self._sound_buffer.engine
        start_tick = eng.state(0)["tick"]
        while not self._stop_event.is_set():
            tick = eng.state(0)["tick"]
            if (tick - start_tick) * 0.1 > self.timeout:
                raise TimeoutError(f"Wake word detection timed out after {self.timeout} seconds")
            self._sound_buffer.pump()
            res = self._handle_events(eng.poll())
            if res is not None:
                return res
        return None

    # ---- public API -----------------------------------------------------------
    def waitforit(self) -> str:
        self._initialize_audio()
        self._stop_event.clear()
        self._listening = True
        try:
            self._wait_for_buffer()
            result = self._detect_word()
            if result is None:
                raise TimeoutError(f"Wake word detection timed out after {self.timeout} seconds")
            return result
        finally:
            self._listening = False

    def start(self) -> None:
        if self.callback is None:
            raise ValueError("Callback must be set for async operation. Use waitforit() for synchronous operation.")
        if self._listening:
            return
        self._initialize_audio(reentry=True)
        self._stop_event.clear()
        self._listening = True

        def listen_loop():
            try:
                self._wait_for_buffer()
                eng = self._sound_buffer.engine
                while not self._stop_event.is_set():
                    self._sound_buffer.pump()   # a finite source keeps feeding silence, like an idle mic
                    res = self._handle_events(eng.poll())
                    if res and self.callback:
                        self.callback(res)
                        eng.reenter(0, float(self.timeout))   # _detect_word returned: the loop calls it again
            finally:
                self._listening = False

        self._listen_thread = threading.Thread(target=listen_loop, daemon=True)
        self._listen_thread.start()

    def stop(self) -> None:
        if hasattr(self, "_stop_event") and self._stop_event:
            self._stop_event.set()
        if hasattr(self, "_listen_thread") and self._listen_thread and self._listen_thread.is_alive():
            self._listen_thread.join(timeout=2.0)
        if hasattr(self, "_sound_buffer") and self._sound_buffer:
            self._sound_buffer.stop()
        if hasattr(self, "_listening"):
            self._listening = False

    def is_listening(self) -> bool:
        return self._listening

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass
