"""Microphone selection for the live source (host-only).

Restates the reference's ``AudioDeviceManager`` (easywakeword/wakeword.py:51-402):
the same device specs -- ``None`` (auto: system default input, else the first
"microphone", else the first "input", else the first device), an ``int`` index, a
name pattern (exact, substring, then regex, case-insensitive), and the magic words
"default"/"system", "best" (highest RMS over a 0.1 s test recording) and "first"
(first device with signal) -- over the PortAudio device list from ``sounddevice``,
with system-audio capture / loopback devices filtered out.

One deliberate difference: where the reference prints a warning and returns None
(PortAudio then silently records from its default device), ``select_device``
raises ``ValueError`` -- a wake-word engine should not listen to a microphone the
caller did not ask for.  ``sd`` may be passed explicitly (tests use a stub).
"""
from __future__ import annotations

import re
from typing import Optional, Union

import numpy as np

_CAPTURE_PATTERNS = ("stereo mix", "what u hear", "wave out", "loopback", "capture", "monitor",
                     "system audio", "audio capture", "sound capture")
_OUTPUT_WORDS = ("speaker", "output", "headphone")
_MIC_WORDS = ("microphone", "mic", "input", "line-in", "aux")


def _sd(sd=None):
    if sd is not None:
        return sd
    import sounddevice  # raises ImportError / OSError without PortAudio
    return sounddevice


class NoInputDeviceError(ValueError):
    """No audio input device exists at all (as opposed to a spec that matches none)."""


class AudioDeviceManager:
    """Input-device selection (wakeword.py:51-402)."""

    @staticmethod
    def is_system_audio_capture_device(name: str) -> bool:
        """Loopback / monitor devices capture playback, not a microphone (wakeword.py:83-125)."""
        n = name.lower()
        if any(p in n for p in _CAPTURE_PATTERNS):
            return True
        return any(w in n for w in _OUTPUT_WORDS) and not any(w in n for w in _MIC_WORDS)

    @staticmethod
    def list_devices(sd=None) -> list:
        """Input devices as dicts {index, name, hostapi, default_samplerate, max_input_channels}."""
        sd = _sd(sd)
        apis = sd.query_hostapis()
        out = []
        for i, d in enumerate(sd.query_devices()):
            if d["max_input_channels"] > 0 and not AudioDeviceManager.is_system_audio_capture_device(d["name"]):
                out.append({"index": i, "name": d["name"], "hostapi": apis[d["hostapi"]]["name"],
                            "default_samplerate": d["default_samplerate"],
                            "max_input_channels": d["max_input_channels"]})
        return out

    @staticmethod
    def _system_default(sd) -> Optional[int]:
        try:
            idx = sd.default.device[0]
            if idx is not None and idx >= 0 and sd.query_devices()[idx]["max_input_channels"] > 0:
                return int(idx)
        except Exception:
            pass
        return None

    @staticmethod
    def test_device_audio_level(index: int, test_duration: float = 0.1, sd=None) -> float:
        """RMS of a short float32 recording (0.0 on any error), wakeword.py:270-304."""
        try:
            sd = _sd(sd)
            x = sd.rec(int(test_duration * 16000), samplerate=16000, channels=1, device=index, dtype=np.float32)
            sd.wait()
            x = np.asarray(x, np.float32).reshape(-1)
            return float(np.sqrt(np.mean(x ** 2))) if x.size else 0.0
        except Exception:
            return 0.0

    @staticmethod
    def find_best_device_by_audio_level(min_rms_threshold: float = 0.001, sd=None) -> Optional[int]:
        best, best_rms = None, 0.0
        for d in AudioDeviceManager.list_devices(sd):
            rms = AudioDeviceManager.test_device_audio_level(d["index"], sd=sd)
            if rms > min_rms_threshold and rms > best_rms:
                best, best_rms = d["index"], rms
        return best

    @staticmethod
    def find_first_working_device(min_rms_threshold: float = 0.001, sd=None) -> Optional[int]:
        for d in AudioDeviceManager.list_devices(sd):
            if AudioDeviceManager.test_device_audio_level(d["index"], sd=sd) > min_rms_threshold:
                return d["index"]
        return None

    @staticmethod
    def select_device(spec: Optional[Union[int, str]] = None, sd=None) -> int:
        """Device index for `spec` (see the module docstring); ValueError when nothing matches."""
        sd = _sd(sd)
        devices = AudioDeviceManager.list_devices(sd)
        if not devices:
            raise NoInputDeviceError("no audio input devices found")
        if spec is None:
            idx = AudioDeviceManager._system_default(sd)
            if idx is not None:
                return idx
            for word in ("microphone", "input"):
                for d in devices:
                    if word in d["name"].lower():
                        return d["index"]
            return devices[0]["index"]
        if isinstance(spec, bool) or not isinstance(spec, (int, str)):
            raise ValueError(f"invalid device specification: {spec!r}")
        if isinstance(spec, int):
            all_dev = sd.query_devices()
            if 0 <= spec < len(all_dev) and all_dev[spec]["max_input_channels"] > 0:
                return spec
            raise ValueError(f"device index {spec} is not valid or not an input device")
        word = spec.lower().strip()
        if word == "best":
            idx = AudioDeviceManager.find_best_device_by_audio_level(sd=sd)
        elif word == "first":
            idx = AudioDeviceManager.find_first_working_device(sd=sd)
        elif word in ("default", "system"):
            idx = AudioDeviceManager._system_default(sd)
        else:
            idx = AudioDeviceManager._select_by_name(devices, spec)
        if idx is None:
            raise ValueError(f"no audio input device matches {spec!r}")
        return idx

    @staticmethod
    def _select_by_name(devices: list, pattern: str) -> Optional[int]:
        """Exact name, then substring, then regex; case-insensitive (wakeword.py:249-281)."""
        p = pattern.lower()
        for d in devices:
            if d["name"].lower() == p:
                return d["index"]
        for d in devices:
            if p in d["name"].lower():
                return d["index"]
        try:
            rx = re.compile(pattern, re.IGNORECASE)
        except re.error:
            return None
        for d in devices:
            if rx.search(d["name"]):
                return d["index"]
        return None

    @staticmethod
    def print_device_list(sd=None) -> None:
        sd = _sd(sd)
        devices = AudioDeviceManager.list_devices(sd)
        if not devices:
            print("No audio input devices found.")
            return
        default = AudioDeviceManager._system_default(sd)
        print("Available audio input devices:")
        print("-" * 60)
        for d in devices:
            mark = " (default)" if d["index"] == default else ""
            print(f"{d['index']:2d}: {d['name']}{mark}")
            print(f"    Host API: {d['hostapi']}")
            print(f"    Channels: {d['max_input_channels']}, Sample Rate: {d['default_samplerate']}")
            print()
