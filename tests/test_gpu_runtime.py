"""Both HIP runtime bindings of libewk.so run the hot path on the GPU.

libewk.so links the system ROCm runtime.  In a process that imported torch first
(the default of easywakeword_amd._lib.load) its HIP calls bind to torch's bundled
runtime instead (RTLD_GLOBAL interposition); a C/ctypes host without torch binds
/opt/rocm's.  smoke() (a level-2 batch + a level-1/2 stream checked against the
oracle) runs in a fresh child process for each binding, and ewk_runtime_info
(dladdr of the resolved hipLaunchKernel) reports which one ran.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys
sys.path.insert(0, {root!r})
import __graft_entry__ as g
g.smoke()
from easywakeword_amd import _lib
info = _lib.runtime_info()
info["torch_imported"] = "torch" in sys.modules
print("RUNTIME " + json.dumps(info))
"""


@pytest.mark.parametrize("no_torch", [True, False], ids=["system-runtime-no-torch", "torch-runtime"])
def test_smoke_under_each_runtime_binding(no_torch):
    env = dict(os.environ)
    if no_torch:
        env["EWK_NO_TORCH_PRELOAD"] = "1"
    else:
        env.pop("EWK_NO_TORCH_PRELOAD", None)
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "smoke ok" in r.stdout
    info = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RUNTIME ")][-1][8:])
    print(info)
    assert "libamdhip64" in os.path.basename(info["path"])
    assert info["hip_version"] > 0
    if no_torch:
        assert not info["torch_imported"]
        assert not info["torch_bundled"]
    else:
        assert info["torch_imported"]
