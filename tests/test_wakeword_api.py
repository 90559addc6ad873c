"""a8: the public API -- WakeWord(textword, wavword).waitforit() / start() / stop()
(reference easywakeword/wakeword.py:642-1240) on the MI355X engine.

CPU part (no device is touched): the constructor's validation order and messages
(wakeword.py:744-763), the auto speech durations pinned by the reference tests
(tests/test_wakeword_simulated.py:687-775), start() without a callback
(:779-788), stop() safe when not listening / on a partially built object
(:809-817), the level-3 word checks (wakeword.py:1129-1153), and no silent CPU
fallback when the detector needs the GPU.

GPU part: waitforit() over the golden reference streams returns at the tick of the
first matching level-2 call of the REAL reference _detect_word
(tests/golden/gate_traces.json), raises TimeoutError on a stream with no word,
start() calls the callback from a background thread, and the optional level-3
confirm callable sees the GPU-normalised segment.
"""
import json
import os
import threading

import numpy as np
import pytest

from golden_io import GOLD, gate_fixture, stream_pcm

WAV = os.path.join(GOLD, "reference_word.wav")


def _ww(**kw):
    from easywakeword_amd import WakeWord
    kw.setdefault("source", None)
    return WakeWord("hello", WAV, **kw)


# ---------------------------------------------------------------- CPU: construction
@pytest.mark.parametrize("kw,msg", [
    (dict(numberofwords=0), "numberofwords must be at least 1"),
    (dict(buffer_seconds=0), "buffer_seconds must be positive"),
    (dict(retry_count=-1), "retry_count must be non-negative"),
    (dict(retry_backoff=-0.5), "retry_backoff must be non-negative"),
    (dict(pre_speech_silence=0), "pre_speech_silence must be positive"),
    (dict(speech_duration_min=-1.0), "speech_duration_min must be positive"),
    (dict(speech_duration_max=0.0), "speech_duration_max must be positive"),
    (dict(speech_duration_min=2.0, speech_duration_max=1.0), "speech_duration_min must be <= speech_duration_max"),
    (dict(post_speech_silence=-0.1), "post_speech_silence must be positive"),
    # the reference checks in this order: the first failing rule names the error
    (dict(numberofwords=0, buffer_seconds=0), "numberofwords must be at least 1"),
])
def test_parameter_validation(kw, msg):
    with pytest.raises(ValueError, match=msg):
        _ww(**kw)


def test_auto_durations_from_reference_wav():
    # reference_word.wav: RMS voice activity 0.69 s (tests/golden/durations.json, from the reference)
    with open(os.path.join(GOLD, "durations.json")) as f:
        want = json.load(f)["reference_word.wav"]
    ww = _ww()
    assert ww.speech_duration_min == pytest.approx(want, abs=1e-12)
    assert abs(ww.speech_duration_max - 2 * ww.speech_duration_min) < 1e-3
    assert ww._user_speech_duration_min is None and ww._user_speech_duration_max is None


def test_user_duration_overrides():
    ww = _ww(speech_duration_min=0.5)
    assert (ww.speech_duration_min, ww.speech_duration_max) == (0.5, 1.0)
    ww = _ww(speech_duration_min=0.4, speech_duration_max=1.5)
    assert (ww.speech_duration_min, ww.speech_duration_max) == (0.4, 1.5)
    assert (ww._user_speech_duration_min, ww._user_speech_duration_max) == (0.4, 1.5)


def test_auto_durations_speech_like_and_fallback(tmp_path):
    import synth
    from easywakeword_amd import WakeWord, write_wav
    p = tmp_path / "speech.wav"
    write_wav(str(p), synth.speech_like(0.8))
    ww = WakeWord("hello", str(p))
    assert 0.4 <= ww.speech_duration_min <= 1.2          # test_wakeword_simulated.py:689-700
    assert abs(ww.speech_duration_max - 2 * ww.speech_duration_min) < 1e-3
    q = tmp_path / "tiny.wav"
    write_wav(str(q), np.zeros(100, np.float32))          # :742-756: analysis fails -> defaults
    ww = WakeWord("hello", str(q))
    assert ww.speech_duration_min > 0 and ww.speech_duration_max >= ww.speech_duration_min
    ww = WakeWord("hello", str(tmp_path / "missing.wav"))
    assert (ww.speech_duration_min, ww.speech_duration_max) == (0.3, 2.0)


def test_start_requires_callback_and_stop_is_safe():
    ww = _ww()
    assert ww.is_listening() is False
    with pytest.raises(ValueError, match="Callback must be set"):
        ww.start()
    ww.stop()
    ww.stop()
    assert ww.is_listening() is False
    from easywakeword_amd import WakeWord
    half = object.__new__(WakeWord)   # partially built, as the reference tests make them
    half.stop()


def test_level3_word_checks():
    ww = _ww(numberofwords=2)
    ww.textword = "hello world"
    assert ww._check_transcription("Hello world.") == "Hello world."
    assert ww._check_transcription("  hello WORLD!? ") == "  hello WORLD!? "
    assert ww._check_transcription("hello") is None          # word count differs
    assert ww._check_transcription("hello there") is None    # target word missing
    assert ww._check_transcription(None) is None and ww._check_transcription("") is None
    assert ww._estimate_syllables("hello computer") == 5


def test_waitforit_needs_the_gpu_without_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: the GPU tests cover the real path")
    from easywakeword_amd import ArraySource
    ww = _ww(source=ArraySource(np.zeros(16000, np.float32)))
    with pytest.raises(Exception) as ei:
        ww.waitforit()
    assert not isinstance(ei.value, TimeoutError)


# ---------------------------------------------------------------- GPU: the detector
def _gate_kw(rec):
    g = rec["gate"]
    return dict(pre_speech_silence=g["pre_speech_silence"], speech_duration_min=g["speech_duration_min"],
                speech_duration_max=g["speech_duration_max"], post_speech_silence=g["post_speech_silence"],
                buffer_seconds=g["buffer_seconds"])


def _trace(name):
    return next(r for r in gate_fixture() if r["name"] == name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["config1_word_x8", "distractors_b", "tight_windows"])
def test_waitforit_returns_at_the_references_first_match(name):
    from easywakeword_amd import ArraySource, WakeWord
    rec = _trace(name)
    first = next(e for e in rec["events"] if e["match"])
    ww = WakeWord("hello", WAV, timeout=60, source=ArraySource(stream_pcm(rec)), **_gate_kw(rec))
    assert ww.waitforit() == "hello"
    assert ww._sound_buffer.engine.state(0)["tick"] == first["tick"]
    assert ww.is_listening() is False
    ww.stop()


@pytest.mark.gpu
def test_waitforit_timeout_without_a_word():
    from easywakeword_amd import ArraySource, WakeWord
    rec = _trace("gain0.3_noise2e-3")          # the reference makes no level-2 call on it
    assert not rec["events"]
    ww = WakeWord("hello", WAV, timeout=5, source=ArraySource(stream_pcm(rec)), **_gate_kw(rec))
    with pytest.raises(TimeoutError, match="timed out after 5 seconds"):
        ww.waitforit()
    full = ww._sound_buffer.engine.state(0)["tick"]
    assert full == 100 + 51                        # buffer fill, then 5 s of virtual clock
    ww.stop()


@pytest.mark.gpu
def test_start_calls_back_on_a_background_thread():
    from easywakeword_amd import ArraySource, WakeWord
    rec = _trace("config1_word_x8")
    got, threads = [], []
    done = threading.Event()

    def cb(text):
        got.append(text)
        threads.append(threading.get_ident())
        if len(got) >= 3:
            done.set()

    ww = WakeWord("hello", WAV, timeout=60, callback=cb, source=ArraySource(stream_pcm(rec)), **_gate_kw(rec))
    ww.start()
    assert ww.is_listening()
    ww.start()                                     # already listening: no second thread
    assert done.wait(60), got
    ww.stop()
    assert ww.is_listening() is False
    assert got[:3] == ["hello"] * 3
    assert threading.get_ident() not in threads
    ww.stop()                                      # idempotent


@pytest.mark.gpu
def test_confirm_sees_the_normalised_segment():
    from easywakeword_amd import ArraySource, WakeWord
    rec = _trace("config1_word_x8")
    seen = []

    def confirm(audio):
        seen.append(audio)
        return "Hello there." if len(seen) == 1 else "hello world"

    ww = WakeWord("hello world", WAV, numberofwords=2, timeout=60, confirm=confirm,
                  source=ArraySource(stream_pcm(rec)), **_gate_kw(rec))
    assert ww.waitforit() == "hello world"        # the first confirm fails the word check
    assert len(seen) == 2
    matches = [e for e in rec["events"] if e["match"]]
    for a, ev in zip(seen, matches):
        assert a.dtype == np.float64 and len(a) == ev["length"]
        assert np.max(np.abs(a)) <= 1.0 and abs(float(np.mean(a))) < 0.05
    assert ww._sound_buffer.engine.state(0)["tick"] == matches[1]["tick"]


@pytest.mark.gpu
def test_torch_usable_after_the_engine_loads():
    """libewk.so (system ROCm runtime) loaded before torch (its bundled runtime) must
    leave torch able to use the GPU: _lib.load() imports torch first."""
    import subprocess
    import sys
    code = ("from easywakeword_amd import _lib; assert _lib.device_count() > 0; "
            "import torch; x = torch.ones(4, device='cuda'); print(float(x.sum()))")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(GOLD)))
    assert r.returncode == 0 and r.stdout.strip().endswith("4.0"), r.stderr[-2000:]


@pytest.mark.gpu
def test_reenter_matches_a_new_detect_word_call():
    """every waitforit()/start() is a new _detect_word entry in its own mode.
    ewk_reenter at tick k equals the oracle re-entering (DetectorRef._enter) at k and
    then running in start() mode (re-entry every 5 s)."""
    from easywakeword_amd import StreamEngine
    from oracle.gate_ref import DetectorRef, GateConfig
    rec = _trace("config1_word_x8")
    pcm = stream_pcm(rec)
    eng = StreamEngine(1)
    det = DetectorRef(GateConfig())
    k_switch = 150
    got = []
    for k in range(len(pcm) // 1600):
        blk = pcm[k * 1600:(k + 1) * 1600]
        if k == k_switch:
            eng.reenter(0, 5.0)
            det.cfg.reentry_timeout = 5.0
            det._enter()
            st = eng.state(0)
            assert st["start_time"] == det.start_time and st["state"] == det.state
        eng.push(blk.reshape(1, -1))
        det.push_tick(blk)
        got.extend((int(e["tick"]), int(e["length"])) for e in eng.poll())
    assert got == [(e.tick, e.length) for e in det.events]
    assert det.reentries > 0
    eng.close()


@pytest.mark.gpu
def test_waitforit_then_start_and_matcher_threshold_isolated():
    from easywakeword_amd import ArraySource, WakeWord
    rec = _trace("config1_word_x8")
    got = []
    done = threading.Event()

    def cb(text):
        got.append(text)
        done.set()

    ww = WakeWord("hello", WAV, timeout=60, callback=cb, source=ArraySource(stream_pcm(rec)), **_gate_kw(rec))
    assert ww.waitforit() == "hello"
    eng = ww._sound_buffer.engine
    assert eng.config.reentry_timeout == 0.0                  # waitforit(): continuous
    ok, s = ww._matcher.matches(np.zeros(16000, np.float32) + 0.01, threshold=99.9)
    assert eng.config.similarity_threshold == 75.0            # the matcher has its own engine
    ww.start()
    assert done.wait(60), got
    assert eng.config.reentry_timeout == 60.0                 # start(): re-entry every timeout s
    ww.stop()
    assert got[0] == "hello"


@pytest.mark.gpu
def test_shared_engine_threshold_is_per_call():
    """WordMatcher(engine=shared).matches(x, threshold) applies the threshold to that call
    and leaves the shared engine's own threshold as it was."""
    import synth
    from easywakeword_amd import Engine, WordMatcher
    shared = Engine()
    m = WordMatcher(engine=shared)
    word = synth.load_word()
    m.set_reference(word)
    ok, s = m.matches(word, threshold=99.99)
    assert s == 100.0 and ok                                # 100.0 >= 99.99
    ok2, s2 = m.matches(word * np.float32(0.5), threshold=101.0)
    assert not ok2
    assert shared.config.similarity_threshold == 75.0
    _, _, _, match = shared.score([word])
    assert bool(match[0])
