"""Generate the golden fixtures by running the REAL reference code (test infra).

Run in the build container (where ``/root/reference`` exists):

    python tests/golden/make_golden.py

The reference (``/root/reference/easywakeword/wakeword.py``) is imported with
the same kind of stubs its own tests use (``tests/test_helpers.py:22-46``):

* ``sounddevice`` -> MagicMock (no PortAudio);
* ``soundfile``   -> stdlib ``wave`` PCM16 (libsndfile scaling: write x*32767,
  read /32768);
* ``librosa``     -> the oracle restatement (``oracle/mfcc_ref.py``) for
  ``load``, ``feature.mfcc`` and ``feature.rms`` (librosa 0.11.0 is absent).

With those stubs the reference's own ``SoundBuffer`` (a1-a3),
``WakeWord._detect_word`` (a4-a5), ``WordMatcher.calculate_similarity`` /
``matches`` (a7) and the WAV template path run unmodified.  ``_detect_word`` is
driven on the virtual clock of ``oracle/gate_ref.py``: ``time.time()`` returns
``k * 0.1`` and ``time.sleep(0.1)`` delivers the next 1600-sample block through
the reference's own ``_add_sound_to_buffer`` callback.  Level 3 is stubbed to
return None (the snapshot's ``_transcribe_audio`` always fails,
SURVEY.md section 0.2), and every ``matches`` call is recorded.

Nothing from the reference is copied into the repo: only the recorded inputs
(as seeds / hashes) and outputs land in ``tests/golden/*.json|npz``.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import types
import wave
from unittest.mock import MagicMock

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from oracle import mfcc_ref  # noqa: E402
import synth  # noqa: E402


# ----------------------------------------------------------------------------- stubs
def _install_stubs():
    sd = MagicMock()
    sd.query_devices.return_value = []
    sd.query_hostapis.return_value = [{"name": "Mock Host API"}]
    sd.default.device = (-1, -1)
    sys.modules["sounddevice"] = sd

    sf = types.ModuleType("soundfile")

    def sf_read(path, dtype="float64", **kw):
        with wave.open(str(path), "rb") as w:
            nch, sr, n = w.getnchannels(), w.getframerate(), w.getnframes()
            raw = w.readframes(n)
        x = np.frombuffer(raw, dtype="<i2").astype(dtype) / 32768.0
        if nch > 1:
            x = x.reshape(-1, nch)
        return x, sr

    def sf_write(path, data, sr, **kw):
        q = np.clip(np.round(np.asarray(data, np.float64) * 32767.0), -32768, 32767).astype("<i2")
        with wave.open(str(path), "wb") as w:
            w.setnchannels(1 if q.ndim == 1 else q.shape[1])
            w.setsampwidth(2)
            w.setframerate(sr)
            w.writeframes(q.tobytes())

    sf.read = sf_read
    sf.write = sf_write
    sys.modules["soundfile"] = sf

    lb = types.ModuleType("librosa")
    feat = types.ModuleType("librosa.feature")

    def lb_load(path, sr=22050, **kw):
        x = mfcc_ref.load_wav_pcm16(path)
        if sr is not None and sr != 16000:
            raise ValueError("stub librosa.load supports 16 kHz only")
        return x, 16000

    def lb_mfcc(y=None, sr=16000, n_mfcc=20, n_fft=512, hop_length=160, **kw):
        assert (sr, n_mfcc, n_fft, hop_length) == (16000, 20, 512, 160)
        return mfcc_ref.mfcc(np.asarray(y))

    def lb_rms(y=None, frame_length=2048, hop_length=512, **kw):
        return mfcc_ref.rms_frames(np.asarray(y), frame_length, hop_length)

    lb.load = lb_load
    feat.mfcc = lb_mfcc
    feat.rms = lb_rms
    lb.feature = feat
    sys.modules["librosa"] = lb
    sys.modules["librosa.feature"] = feat


_install_stubs()
sys.path.insert(0, REF)
from easywakeword import wakeword as ref  # noqa: E402


def sha(x: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def f64list(x):
    return [float(v) for v in np.asarray(x, dtype=np.float64).ravel()]


def nanable(v):
    v = float(v)
    return None if np.isnan(v) else v


# ----------------------------------------------------------------------------- matcher
def matcher_fixtures():
    """Template + segment->score cases through the reference WordMatcher."""
    m = ref.WordMatcher(sample_rate=16000)
    m.load_reference_from_file(synth.WAV, "computer")
    tmean, tstd = m.reference_mfcc_mean, m.reference_mfcc_std
    assert tmean.dtype == np.float32

    cases = synth.matcher_cases()
    word = synth.load_word()

    out = {"template": {"mean": f64list(tmean), "std": f64list(tstd), "wav": "reference_word.wav",
                        "n_samples": int(len(word))},
           "cases": []}
    audio = {}
    for name, x in cases:
        x = np.ascontiguousarray(x, dtype=np.float32)
        rec = {"name": name, "n": int(len(x)), "sha256_f32": sha(x)}
        for dt in ("float64", "float32"):
            y = x.astype(dt)
            cm, cs = m.extract_mfcc(y)
            ok, s = m.matches(y, threshold=75.0)
            rec[dt] = {"mean": f64list(cm), "std": f64list(cs), "score": nanable(s), "match": bool(ok)}
        out["cases"].append(rec)
        audio[name] = x
    return m, out, audio


# ----------------------------------------------------------------------------- gate
class _StreamEnd(Exception):
    pass


class VirtualClock:
    """Patches wakeword.time: time() = k*0.1, sleep() pushes the next block."""

    def __init__(self, buf, pcm, block=1600, tick=0.1):
        self.buf, self.pcm, self.block, self.tick_s = buf, pcm, block, tick
        self.k = 0
        self.nblocks = len(pcm) // block

    def time(self):
        return float(self.k) * self.tick_s

    def sleep(self, dt):
        if self.k >= self.nblocks:
            raise _StreamEnd()
        blk = self.pcm[self.k * self.block:(self.k + 1) * self.block].reshape(-1, 1)
        self.buf._add_sound_to_buffer(blk, self.block, None, None)
        self.k += 1


def run_reference_gate(pcm, matcher, cfg, reentry_timeout=None):
    """Drive the reference SoundBuffer + _detect_word over `pcm`; return events."""
    buf = ref.SoundBuffer(seconds=cfg.get("buffer_seconds", 10))
    clock = VirtualClock(buf, pcm, cfg.get("block", 1600))
    ww = object.__new__(ref.WakeWord)
    ww.textword = "computer"
    ww.numberofwords = 1
    ww.timeout = 1e9 if reentry_timeout is None else reentry_timeout
    ww.similarity_threshold = 75.0
    ww.pre_speech_silence = cfg["pre_speech_silence"]
    ww.speech_duration_min = cfg["speech_duration_min"]
    ww.speech_duration_max = cfg["speech_duration_max"]
    ww.post_speech_silence = cfg["post_speech_silence"]
    ww.verbose = False
    ww.callback = None
    import threading
    ww._stop_event = threading.Event()
    ww._sound_buffer = buf
    ww._matcher = matcher
    ww._listening = True
    ww._transcribe_audio = lambda audio: None

    events = []
    real_matches = matcher.matches

    def rec_matches(audio, threshold=75.0):
        ok, s = real_matches(audio, threshold=threshold)
        events.append({"tick": clock.k, "time": clock.time(), "length": int(len(audio)),
                       "dtype": str(audio.dtype), "sha256": sha(np.asarray(audio)),
                       "score": nanable(s), "match": bool(ok)})
        return ok, s

    silent_log = []
    real_is_silent = buf.is_silent

    def rec_is_silent():
        r = real_is_silent()
        silent_log.append((clock.k, bool(r), float(buf.silence_threshold)))
        return r

    buf.is_silent = rec_is_silent
    matcher.matches = rec_matches
    old_time = ref.time
    ref.time = clock
    reentries = 0
    try:
        ww._wait_for_buffer()
        while True:
            try:
                ww._detect_word()
            except TimeoutError:
                reentries += 1
                if reentry_timeout is None:
                    raise
                continue
    except _StreamEnd:
        pass
    finally:
        ref.time = old_time
        matcher.matches = real_matches
    return events, silent_log, reentries


STREAMS = [
    # name, make_stream kwargs, gate overrides
    ("config1_word_x8", dict(seed=1234, n_words=8, sigma=1e-3, gain=1.0), {}),
    ("gain0.3_noise2e-3", dict(seed=1235, n_words=6, sigma=2e-3, gain=0.3), {}),
    ("gain2.5_noise1e-4", dict(seed=1236, n_words=6, sigma=1e-4, gain=2.5), {}),
    ("distractors_a", dict(seed=1237, n_words=8, sigma=1e-3, gain=1.0, distractors=True), {}),
    ("distractors_b", dict(seed=1238, n_words=8, sigma=3e-3, gain=0.7, distractors=True), {}),
    ("tight_windows", dict(seed=1239, n_words=6, sigma=1e-3, gain=1.2),
     {"pre_speech_silence": 0.5, "speech_duration_min": 0.69, "speech_duration_max": 1.38,
      "post_speech_silence": 0.3}),
    # level-2 rejects, near-threshold scores, negative-similarity NaNs and a segment
    # straddling the ring wrap (tick 311: first sample before the physical end)
    ("rejects_gain3", dict(seed=1300, n_words=8, sigma=1e-3, gain=3.0, kinds=["hp", "white", "hp_near", "hp"]), {}),
    ("rejects_gain5", dict(seed=1300, n_words=8, sigma=1e-3, gain=5.0, kinds=["hp", "white", "hp_near", "hp"]), {}),
    # segments longer than max_segment_seconds: the reference skips level 2 (wakeword.py:1113-1118)
    ("skip_long", dict(seed=1301, n_words=6, sigma=1e-3, gain=1.0, kinds=["long", "word", "long"]),
     {"speech_duration_max": 3.5}),
    # frame_size 512: 312 physical blocks, unaligned pointer (wakeword.py:472-486)
    ("frame512_bursts", dict(seed=1302, n_words=8, sigma=1e-3, gain=1.0, kinds=["burst", "hp", "burst", "word"],
                             block=512), {"block": 512, "speech_duration_max": 6.0}),
]


def gate_fixtures(matcher):
    base = {"pre_speech_silence": 0.8, "speech_duration_min": 0.3, "speech_duration_max": 2.0,
            "post_speech_silence": 0.4, "buffer_seconds": 10, "block": 1600}
    out = []
    for name, kw, over in STREAMS:
        cfg = dict(base, **over)
        pcm, truth = synth.make_stream(**kw)
        events, silent_log, _ = run_reference_gate(pcm, matcher, cfg)
        out.append({"name": name, "stream": kw, "gate": cfg, "n_samples": int(len(pcm)),
                    "sha256_f32": sha(pcm), "truth": [[int(p), k] for p, k in truth],
                    "events": events,
                    "silent": [[k, s] for k, s, _ in silent_log],
                    "threshold": [thr for _, _, thr in silent_log]})
    # start()-mode: TimeoutError re-entry every 5 s of virtual time
    cfg = dict(base)
    pcm, truth = synth.make_stream(seed=1240, n_words=8, sigma=1e-3, gain=1.0)
    events, silent_log, reentries = run_reference_gate(pcm, matcher, cfg, reentry_timeout=5.0)
    out.append({"name": "reentry_timeout5", "stream": dict(seed=1240, n_words=8, sigma=1e-3, gain=1.0),
                "gate": dict(cfg, reentry_timeout=5.0), "n_samples": int(len(pcm)),
                "sha256_f32": sha(pcm), "truth": [[int(p), k] for p, k in truth], "events": events,
                "silent": [[k, s] for k, s, _ in silent_log],
                "threshold": [thr for _, _, thr in silent_log], "reentries": reentries})
    return out


def duration_fixture():
    """_analyze_reference_audio_duration (wakeword.py:854-898) on reference_word.wav."""
    ww = object.__new__(ref.WakeWord)
    ww.wavword = synth.WAV
    ww.verbose = False
    return {"reference_word.wav": ww._analyze_reference_audio_duration()}


def main():
    matcher, mfix, audio = matcher_fixtures()
    with open(os.path.join(HERE, "matcher_cases.json"), "w") as f:
        json.dump(mfix, f, indent=1)
    gfix = gate_fixtures(matcher)
    with open(os.path.join(HERE, "gate_traces.json"), "w") as f:
        json.dump(gfix, f)
    with open(os.path.join(HERE, "durations.json"), "w") as f:
        json.dump(duration_fixture(), f, indent=1)
    n_ev = sum(len(g["events"]) for g in gfix)
    print(f"matcher cases: {len(mfix['cases'])}, gate streams: {len(gfix)}, events: {n_ev}")


if __name__ == "__main__":
    main()
