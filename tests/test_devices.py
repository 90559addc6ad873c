"""Microphone selection (easywakeword_amd.devices) against the reference's
AudioDeviceManager rules (wakeword.py:51-402), on a stub PortAudio device list."""
import types

import numpy as np
import pytest

from easywakeword_amd.devices import AudioDeviceManager as ADM

DEVICES = [
    {"name": "Speakers (Realtek)", "max_input_channels": 2, "hostapi": 0, "default_samplerate": 48000.0},
    {"name": "HDMI Output", "max_input_channels": 0, "hostapi": 0, "default_samplerate": 48000.0},
    {"name": "Line In (USB Audio)", "max_input_channels": 1, "hostapi": 0, "default_samplerate": 44100.0},
    {"name": "Stereo Mix", "max_input_channels": 2, "hostapi": 0, "default_samplerate": 48000.0},
    {"name": "Headset Microphone", "max_input_channels": 1, "hostapi": 1, "default_samplerate": 16000.0},
    {"name": "Webcam Mic", "max_input_channels": 1, "hostapi": 1, "default_samplerate": 16000.0},
]


def stub(default_in=-1, levels=None):
    sd = types.SimpleNamespace()
    sd.query_devices = lambda: DEVICES
    sd.query_hostapis = lambda: [{"name": "MME"}, {"name": "WASAPI"}]
    sd.default = types.SimpleNamespace(device=(default_in, -1))
    state = {}

    def rec(n, samplerate, channels, device, dtype):
        state["dev"] = device
        return np.full((n, 1), (levels or {}).get(device, 0.0), np.float32)

    sd.rec = rec
    sd.wait = lambda: None
    return sd


def test_list_filters_outputs_and_loopback():
    names = [d["name"] for d in ADM.list_devices(stub())]
    assert names == ["Line In (USB Audio)", "Headset Microphone", "Webcam Mic"]
    assert ADM.is_system_audio_capture_device("Monitor of Built-in Audio")
    assert not ADM.is_system_audio_capture_device("Headphone Mic Input")   # output word + mic word


def test_auto_selection_order():
    assert ADM.select_device(None, sd=stub(default_in=5)) == 5        # system default input first
    assert ADM.select_device(None, sd=stub(default_in=1)) == 4        # default has no input -> "microphone"
    assert ADM.select_device(None, sd=stub()) == 4


def test_index_name_and_magic_words():
    sd = stub(default_in=2, levels={2: 0.0005, 4: 0.02, 5: 0.05})
    assert ADM.select_device(4, sd=sd) == 4
    assert ADM.select_device("webcam mic", sd=sd) == 5                # exact (case-insensitive)
    assert ADM.select_device("headset", sd=sd) == 4                   # substring
    assert ADM.select_device(r"line\s+in", sd=sd) == 2                # regex
    assert ADM.select_device("default", sd=sd) == 2
    assert ADM.select_device("best", sd=sd) == 5                      # highest RMS above 0.001
    assert ADM.select_device("first", sd=sd) == 4                     # first with signal


@pytest.mark.parametrize("spec", [1, 99, "no such mic", "best", 2.5])
def test_unmatched_spec_raises(spec):
    with pytest.raises(ValueError):
        ADM.select_device(spec, sd=stub())                            # no device has signal for "best"


def test_no_input_device_is_an_oserror_for_the_facade(monkeypatch):
    """No input device at all: select_device raises NoInputDeviceError (a ValueError); the
    facade's default source turns it into the documented OSError hint."""
    from easywakeword_amd import devices
    from easywakeword_amd.wakeword import _default_source
    sd = stub()
    sd.query_devices = lambda: [d for d in DEVICES if d["max_input_channels"] == 0]
    with pytest.raises(devices.NoInputDeviceError):
        ADM.select_device(None, sd=sd)

    def none(spec, sd=None):
        raise devices.NoInputDeviceError("no audio input devices found")
    monkeypatch.setattr(devices.AudioDeviceManager, "select_device", staticmethod(none))
    with pytest.raises(OSError, match="ArraySource"):
        _default_source(None)

    def unmatched(spec, sd=None):
        raise ValueError("no audio input device matches 'x'")
    monkeypatch.setattr(devices.AudioDeviceManager, "select_device", staticmethod(unmatched))
    with pytest.raises(ValueError, match="matches"):
        _default_source("x")
