"""ewk_db64 (csrc/ewk_db64.h), the fp64 re-score's 10 log10(x): built for the host with g++ and
checked against 80-bit long double over the range the re-score feeds it (x >= 1e-10 after
power_to_db's amin clamp, librosa 0.11.0 via wakeword.py:561-563), plus NaN / +inf.  The device
build differs only in the reciprocal seed (v_rcp_f64, refined by the same two Newton steps)."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "easywakeword_amd", "csrc", "ewk_db64.h")


@pytest.fixture(scope="module")
def db64(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("db64")
    src = d / "h.cpp"
    src.write_text(f'#include "{HDR}"\n'
                   'extern "C" void db64(const double* x, double* y, long n) '
                   '{ for (long i = 0; i < n; ++i) y[i] = ewk_db64(x[i]); }\n')
    lib = d / "libdb64.so"
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-ffp-contract=off", str(src), "-o", str(lib)], check=True)
    L = ctypes.CDLL(str(lib))

    def f(x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty_like(x)
        L.db64(x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(len(x)))
        return y
    return f


def test_db64_within_two_ulps_of_long_double(db64):
    rng = np.random.default_rng(0)
    x = np.concatenate([10 ** rng.uniform(-10, 14, 400_000), 2.0 ** np.arange(-33, 47),
                        np.nextafter(np.sqrt(0.5), [0.0, 1.0]), np.nextafter(1.0, [0.0, 2.0]),
                        [1e-10, 1.0, 2.0, 3.0, 10.0, 100.0, 1e10]])
    y = db64(x)
    ref = 10 * np.log10(x.astype(np.longdouble))
    ulp = np.spacing(np.abs(ref.astype(np.float64)))
    err = np.abs((y.astype(np.longdouble) - ref) / ulp).astype(np.float64)
    assert err.max() <= 2.0, err.max()
    # numpy's own 10.0 * np.log10 (two roundings) is within ~1.2 ulp: the two agree to ~3e-14 dB
    assert np.abs(y - 10.0 * np.log10(x)).max() <= 1e-13
    assert db64(np.array([1.0]))[0] == 0.0


def test_db64_nan_and_inf_pass_through(db64):
    y = db64(np.array([np.nan, np.inf]))
    assert np.isnan(y[0]) and y[1] == np.inf
