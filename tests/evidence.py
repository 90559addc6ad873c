"""Failure evidence for GPU parity tests (test infrastructure).

A GPU parity failure that does not repeat is only as good as what it left behind (round 5's
one-off ring-path score miss kept nothing but a 4-digit number).  `dump` writes the full
records of a failing case as JSON under gpurun_out/ (merged back from the GPU box by gpurun)
before the test asserts, so the next session starts from the data, not from a re-run.
"""
import json
import os
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _plain(x):
    if isinstance(x, dict):
        return {str(k): _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, np.ndarray):
        return _plain(x.tolist())
    if isinstance(x, (np.floating, float)):
        return repr(float(x))          # full precision, NaN-safe
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.bool_,)):
        return bool(x)
    return x


def _out_dir() -> str:
    return os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "gpurun_out")


def progress(msg: str) -> None:
    """Append a timestamped line to gpurun_out/progress.log: a long GPU test's stages (and the
    heartbeat of tests/conftest.py) stay visible while pytest captures its output."""
    try:
        os.makedirs(_out_dir(), exist_ok=True)
        with open(os.path.join(_out_dir(), "progress.log"), "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")
    except OSError:
        pass


def dump(name: str, payload: dict) -> str:
    """Write payload to gpurun_out/evidence_<name>_<time>.json; returns the path ('' if unwritable)."""
    out = _out_dir()
    try:
        os.makedirs(out, exist_ok=True)
        path = os.path.join(out, f"evidence_{name}_{int(time.time() * 1000)}.json")
        with open(path, "w") as f:
            json.dump(_plain(payload), f, indent=1)
        return path
    except OSError:
        return ""
