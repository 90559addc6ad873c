import os
import sys
import threading
import time

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libewk.so")
    config.addinivalue_line("markers", "slow: long-running")


def _gpu_available() -> bool:
    try:
        from easywakeword_amd import _lib
        return _lib.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _gpu_heartbeat(request):
    """GPU tests: a line in gpurun_out/progress.log every 30 s while the test runs (a test that
    spends minutes in subprocesses or the oracle pool prints nothing through pytest's capture)."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from evidence import progress
    stop = threading.Event()
    name, t0 = request.node.nodeid, time.time()
    progress(f"start {name}")

    def beat():
        while not stop.wait(30.0):
            progress(f"  {name}: {time.time() - t0:.0f} s")

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        stop.set()
        th.join()
        progress(f"end {name}: {time.time() - t0:.1f} s")
