"""include/qldpc_libm.h (the reproducible tanh/atanh both the BP kernel and the
oracle use) stays within 3 ULP of NumPy's tanh/arctanh — the functions
BP_decoder calls (decoders.py:254-259) — over the BP domain."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    d = tmp_path_factory.mktemp("libm")
    src = d / "probe.c"
    src.write_text('#include "qldpc_libm.h"\n'
                   "void vt(const double*x,double*y,long n){for(long i=0;i<n;++i)y[i]=qldpc_tanh(x[i]);}\n"
                   "void va(const double*x,double*y,long n){for(long i=0;i<n;++i)y[i]=qldpc_atanh(x[i]);}\n")
    so = d / "probe.so"
    subprocess.run(["gcc", "-O2", "-mfma", "-fPIC", "-ffp-contract=off", "-shared", "-I",
                    os.path.join(ROOT, "include"), "-o", str(so), str(src)], check=True)
    return ctypes.CDLL(str(so))


def _run(L, fn, x):
    y = np.empty_like(x)
    getattr(L, fn)(x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p),
                   ctypes.c_long(len(x)))
    return y


def _ulps(a, b):
    return np.abs(a.view(np.int64) - b.view(np.int64))


def test_tanh_within_3ulp(probe):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-40, 40, 200000), rng.uniform(-1, 1, 100000),
                        10 ** rng.uniform(-12, 0, 50000) * rng.choice([-1, 1], 50000)])
    assert _ulps(_run(probe, "vt", x), np.tanh(x)).max() <= 3


def test_atanh_within_3ulp(probe):
    rng = np.random.default_rng(1)
    z = np.concatenate([rng.uniform(-1, 1, 100000), 1 - 10 ** rng.uniform(-16, 0, 100000),
                        -(1 - 10 ** rng.uniform(-16, 0, 30000)), 10 ** rng.uniform(-12, 0, 30000)])
    z = z[np.abs(z) < 1]
    assert _ulps(_run(probe, "va", z), np.arctanh(z)).max() <= 3


def test_special_values(probe):
    t = _run(probe, "vt", np.array([0.0, -0.0, np.inf, -np.inf, 22.0, -30.0, 1e-300]))
    assert t[0] == 0 and np.signbit(t[1]) and t[2] == 1 and t[3] == -1 and t[4] == 1 and t[5] == -1
    assert t[6] == 1e-300
    a = _run(probe, "va", np.array([0.0, 1.0, -1.0, 1 - 1e-9]))
    assert a[0] == 0 and np.isposinf(a[1]) and np.isneginf(a[2])
    assert abs(a[3] - np.arctanh(1 - 1e-9)) <= 4e-15 * abs(a[3])
