"""The C-ABI library loads and exports every symbol include/ewk.h declares (CPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "ewk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ewk_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from easywakeword_amd import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(_lib.EXPORTS) == syms


def test_struct_layouts_match_header():
    from easywakeword_amd import _lib
    assert ctypes.sizeof(_lib.EwkConfig) == 4 * 4 + 12 * 8 + 2 * 4
    assert ctypes.sizeof(_lib.EwkEvent) == 48
    assert _lib.EVENT_DTYPE.itemsize == 48


def test_defaults_are_reference_constants():
    from easywakeword_amd import _lib
    c = _lib.default_config()
    assert (c.sample_rate, c.buffer_seconds, c.block) == (16000, 10, 1600)
    assert (c.pre_speech_silence, c.speech_duration_min, c.speech_duration_max, c.post_speech_silence) == \
        (0.8, 0.3, 2.0, 0.4)
    assert (c.padding, c.max_segment_seconds, c.similarity_threshold) == (0.05, 3.0, 75.0)
    assert (c.min_threshold, c.initial_threshold, c.tick_seconds) == (0.005, 0.01, 0.1)
    assert _lib.load().ewk_abi_version() == 4


def test_no_silent_cpu_fallback():
    """Without a GPU the engine must fail loudly, never compute on the CPU."""
    from easywakeword_amd import Engine, _lib
    if _lib.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no HIP device"):
        Engine()


def test_invalid_config_raises_valueerror_before_device_check():
    from easywakeword_amd import Engine
    with pytest.raises(ValueError, match="speech_duration_min must be <= speech_duration_max"):
        Engine(speech_duration_min=2.0, speech_duration_max=1.0)


@pytest.mark.parametrize("cfg, msg", [
    (dict(ring_samples=19200), "longest segment request"),         # < 2.55 s + one tick
    (dict(ring_samples=48000, block=512), "block to divide"),     # 160000 % 512 != 0
    (dict(ring_samples=48000 + 800), "block to divide"),           # not a whole number of ticks
    (dict(ring_samples=-1), "ring_samples must be in"),
    (dict(ring_samples=170000), "ring_samples must be in"),        # larger than the reference ring
])
def test_compact_ring_config_validated_before_device_check(cfg, msg):
    """ewk_config.ring_samples (compact sample rings) is checked on the host, GPU or not."""
    from easywakeword_amd import StreamEngine
    with pytest.raises(ValueError, match=msg):
        StreamEngine(4, **cfg)


def test_runtime_info_reports_the_bound_hip_runtime():
    """ewk_runtime_info: torch's bundled runtime when torch was imported first (the
    default of _lib.load), the system ROCm runtime in a torch-free process."""
    import json
    import subprocess
    import sys
    code = ("import json, sys; from easywakeword_amd import _lib; i = _lib.runtime_info(); "
            "i['torch'] = 'torch' in sys.modules; print(json.dumps(i))")
    env = dict(os.environ, EWK_NO_TORCH_PRELOAD="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert not info["torch"] and not info["torch_bundled"]
    assert os.path.basename(info["path"]).startswith("libamdhip64.so")
