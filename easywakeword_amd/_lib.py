"""ctypes binding of libewk.so (the C ABI declared in include/ewk.h).

There is no CPU fallback: if the shared library or a gfx950 device is missing,
every engine constructor raises.  Error codes map to the reference's exception
conventions (ValueError for bad parameters / missing template).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EWK_LIB") or os.path.join(HERE, "libewk.so")

N_MFCC = 20
EWK_OK = 0
EWK_EINVAL = -1
EWK_ENOTEMPLATE = -2
EWK_EHIP = -3
EWK_ENOMEM = -4
EWK_ENODEV = -5
EWK_EOVERWRITTEN = -6
EWK_EV_SKIPPED = 1
EWK_EV_RESCORED = 2
# |MFCC mean vector| below which a segment's score comes from the fp64 re-score (the scorer's
# kTinyMean, csrc/ewk_mfcc.hip; tests/test_rescore_criteria.py keeps the two equal)
RESCORE_TINY_MEAN = 32.0
# ... unless its float32 similarity percent is below -(NAN_MARGIN_A / |mean| + NAN_MARGIN_B): NaN in
# the reference beyond the float32 error, not re-scored (kNanMarginA / kNanMarginB, same test)
NAN_MARGIN_A = 0.5
NAN_MARGIN_B = 0.05
EWK_PUSH_DEVICE = 1
EWK_PCM_DEVICE = 1
EWK_OUT_DEVICE = 4
EWK_RING_F32 = 0
EWK_RING_I16 = 1
EWK_SCORE_REQUIRE_TEMPLATE = 1
EWK_SCORE_F32_CANDIDATES = 2
EWK_COMPACT_APPEND = 1

# Every symbol include/ewk.h declares (checked by tests/test_capi.py).
EXPORTS = [
    "ewk_default_config", "ewk_last_error", "ewk_abi_version", "ewk_device_count",
    "ewk_create", "ewk_destroy", "ewk_sync", "ewk_stream_handle",
    "ewk_template_from_pcm", "ewk_set_template", "ewk_get_template",
    "ewk_score_segments", "ewk_score_segments_device", "ewk_score_segments_f64",
    "ewk_push", "ewk_push_many", "ewk_poll", "ewk_get_stream_state", "ewk_read_last",
    "ewk_read_segment", "ewk_reset_streams", "ewk_set_similarity_threshold",
    "ewk_profile_enable", "ewk_profile_read",
    "ewk_push_pcm16", "ewk_push_many_pcm16", "ewk_normalize_segments", "ewk_normalize_events",
    "ewk_decode_pcm16", "ewk_poll_lagged", "ewk_runtime_info", "ewk_reenter", "ewk_compact_positives",
]


class EwkConfig(C.Structure):
    _fields_ = [
        ("sample_rate", C.c_int32), ("buffer_seconds", C.c_int32), ("block", C.c_int32),
        ("ring_samples", C.c_int32), ("tick_seconds", C.c_double), ("pre_speech_silence", C.c_double),
        ("speech_duration_min", C.c_double), ("speech_duration_max", C.c_double),
        ("post_speech_silence", C.c_double), ("padding", C.c_double), ("max_segment_seconds", C.c_double),
        ("similarity_threshold", C.c_double), ("reentry_timeout", C.c_double), ("min_threshold", C.c_double),
        ("initial_threshold", C.c_double), ("rescore_margin", C.c_double),
        ("ring_format", C.c_int32), ("reserved1", C.c_int32),
    ]


class EwkEvent(C.Structure):
    _fields_ = [
        ("stream", C.c_int32), ("length", C.c_int32), ("tick", C.c_int64), ("ring_start", C.c_int64),
        ("time", C.c_double), ("score", C.c_double), ("match", C.c_int32), ("flags", C.c_int32),
    ]


EVENT_DTYPE = np.dtype([("stream", "<i4"), ("length", "<i4"), ("tick", "<i8"), ("ring_start", "<i8"),
                        ("time", "<f8"), ("score", "<f8"), ("match", "<i4"), ("flags", "<i4")])
assert EVENT_DTYPE.itemsize == C.sizeof(EwkEvent)


class EwkPositive(C.Structure):
    _fields_ = [("id", C.c_int64), ("score", C.c_double), ("step", C.c_int64)]


POSITIVE_DTYPE = np.dtype([("id", "<i8"), ("score", "<f8"), ("step", "<i8")])
assert POSITIVE_DTYPE.itemsize == C.sizeof(EwkPositive)


class EwkStreamState(C.Structure):
    _fields_ = [
        ("samples_collected", C.c_int64), ("tick", C.c_int64), ("silence_threshold", C.c_double),
        ("last_rms", C.c_double), ("silence_start_time", C.c_double), ("sound_start_time", C.c_double),
        ("sound_end_time", C.c_double), ("start_time", C.c_double), ("pointer", C.c_int32),
        ("state", C.c_int32), ("started", C.c_int32), ("last_silent", C.c_int32),
    ]


_lib = None
_lock = threading.Lock()

_P = C.c_void_p
_fp = C.POINTER(C.c_float)
_dp = C.POINTER(C.c_double)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)


def load():
    """Load libewk.so (build it first if this checkout has none)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            from . import build as _build
            _build.build()
        # torch bundles its own HIP and HSA runtimes (sonames libamdhip64.so,
        # libhsa-runtime64.so) beside the system ROCm ones libewk.so links.  When the
        # system runtime opens the GPU first, torch's runtime later finds no device
        # (seen on MI355X: "no ROCm-capable device is detected"); the other order works
        # and device pointers pass between the two.  So torch, when installed, is
        # imported before libewk.so is opened.
        if os.environ.get("EWK_NO_TORCH_PRELOAD") != "1":
            try:
                import torch  # noqa: F401
            except Exception:
                pass
        lib = C.CDLL(LIB_PATH)
        sig = {
            "ewk_default_config": (None, [C.POINTER(EwkConfig)]),
            "ewk_last_error": (C.c_char_p, []),
            "ewk_abi_version": (C.c_int, []),
            "ewk_device_count": (C.c_int, []),
            "ewk_runtime_info": (C.c_int, [C.c_char_p, C.c_int32, _i32p]),
            "ewk_create": (C.c_int, [C.POINTER(_P), C.c_int, C.c_int32, C.POINTER(EwkConfig)]),
            "ewk_destroy": (None, [_P]),
            "ewk_sync": (C.c_int, [_P]),
            "ewk_stream_handle": (_P, [_P]),
            "ewk_template_from_pcm": (C.c_int, [_P, _fp, C.c_int64]),
            "ewk_set_template": (C.c_int, [_P, _fp, _fp]),
            "ewk_get_template": (C.c_int, [_P, _fp, _fp]),
            "ewk_set_similarity_threshold": (C.c_int, [_P, C.c_double]),
            "ewk_score_segments": (C.c_int, [_P, _fp, C.c_int64, _i64p, _i32p, C.c_int32, _fp, _fp, _dp, _u8p,
                                             C.c_int32]),
            "ewk_score_segments_device": (C.c_int, [_P, _P, _P, _P, C.c_int32, _P, _P, _P, _P, C.c_int32, _P]),
            "ewk_score_segments_f64": (C.c_int, [_P, _fp, C.c_int64, _i64p, _i32p, C.c_int32, _dp, _dp, _dp,
                                                 C.c_int32]),
            "ewk_push": (C.c_int, [_P, _P, C.c_int64, C.c_int32]),
            "ewk_push_many": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.c_int32, C.c_int32]),
            "ewk_poll": (C.c_int, [_P, C.POINTER(EwkEvent), C.c_int32, _i32p]),
            "ewk_poll_lagged": (C.c_int, [_P, C.POINTER(EwkEvent), C.c_int32, _i32p]),
            "ewk_get_stream_state": (C.c_int, [_P, C.c_int32, C.POINTER(EwkStreamState)]),
            "ewk_read_last": (C.c_int, [_P, C.c_int32, C.c_int64, _fp, _i64p]),
            "ewk_read_segment": (C.c_int, [_P, C.c_int32, C.c_int64, C.c_int32, _fp]),
            "ewk_reset_streams": (C.c_int, [_P]),
            "ewk_reenter": (C.c_int, [_P, C.c_int32, C.c_double]),
            "ewk_profile_enable": (C.c_int, [_P, C.c_int32]),
            "ewk_profile_read": (C.c_int, [_P, C.c_int32, _dp, _i64p]),
            "ewk_push_pcm16": (C.c_int, [_P, _P, C.c_int64, C.c_int32]),
            "ewk_push_many_pcm16": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.c_int32, C.c_int32]),
            "ewk_normalize_segments": (C.c_int, [_P, _P, C.c_int64, _i64p, _i32p, C.c_int32, _P, C.c_int32]),
            "ewk_normalize_events": (C.c_int, [_P, C.POINTER(EwkEvent), C.c_int32, _P, C.c_int32]),
            "ewk_decode_pcm16": (C.c_int, [_P, _P, C.c_int64, _P, C.c_int32]),
            "ewk_compact_positives": (C.c_int, [_P, _P, _P, C.c_int32, C.c_int64, C.c_int64, _P, _P, C.c_int32, _P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


class RingOverwrittenError(ValueError):
    """ewk_normalize_events: an event's samples were overwritten in its ring since its tick
    (EWK_EOVERWRITTEN).  A ValueError, so callers that caught the old EWK_EINVAL still do."""


def check(rc: int) -> None:
    if rc == EWK_OK:
        return
    msg = (load().ewk_last_error() or b"").decode(errors="replace")
    if rc == EWK_EOVERWRITTEN:
        raise RingOverwrittenError(msg)
    if rc in (EWK_EINVAL, EWK_ENOTEMPLATE):
        raise ValueError(msg)
    if rc == EWK_ENOMEM:
        raise MemoryError(msg)
    raise RuntimeError(f"ewk error {rc}: {msg}")


def default_config(**overrides) -> EwkConfig:
    cfg = EwkConfig()
    load().ewk_default_config(C.byref(cfg))
    for k, v in overrides.items():
        if not hasattr(cfg, k):
            raise TypeError(f"unknown config field {k!r}")
        setattr(cfg, k, v)
    return cfg


def runtime_info() -> dict:
    """The HIP runtime libewk.so's calls bind to: {"path": file defining hipLaunchKernel,
    "hip_version": hipRuntimeGetVersion or -1, "torch_bundled": path inside a torch wheel}."""
    buf = C.create_string_buffer(4096)
    v = C.c_int32(-1)
    check(load().ewk_runtime_info(buf, len(buf), C.byref(v)))
    path = buf.value.decode(errors="replace")
    return {"path": path, "hip_version": int(v.value),
            "torch_bundled": f"{os.sep}torch{os.sep}lib{os.sep}" in path}


def device_count() -> int:
    return int(load().ewk_device_count())


def fptr(a: np.ndarray):
    return a.ctypes.data_as(_fp)


def dptr(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def i64ptr(a: np.ndarray):
    return a.ctypes.data_as(_i64p)


def i32ptr(a: np.ndarray):
    return a.ctypes.data_as(_i32p)


def u8ptr(a: np.ndarray):
    return a.ctypes.data_as(_u8p)
