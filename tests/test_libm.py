"""include/qldpc_libm.h restates NumPy's own float64 tanh (simd_tanh_f64),
arctanh (SVML atanh8_ha) and log (SVML log8_ha) — the functions BP_decoder and
both decoders' priors call (decoders.py:147, :232, :254-259) — bit for bit:
checked here against NumPy itself on this host (the host class the golden
vectors were captured on)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _numpy_dispatch_matches_capture_host():
    """The restated code paths are the AVX512_SKX ones; elsewhere NumPy
    itself runs other code and cannot serve as the check."""
    try:
        from numpy._core._multiarray_umath import __cpu_features__
    except ImportError:
        return False
    return bool(__cpu_features__.get("AVX512_SKX"))


pytestmark = pytest.mark.skipif(not _numpy_dispatch_matches_capture_host(),
                                reason="NumPy here does not dispatch to its AVX512_SKX tanh/SVML kernels")


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    d = tmp_path_factory.mktemp("libm")
    src = d / "probe.c"
    src.write_text('#include "qldpc_libm.h"\n'
                   "void vt(const double*x,double*y,long n){for(long i=0;i<n;++i)y[i]=qldpc_tanh(x[i]);}\n"
                   "void va(const double*x,double*y,long n){for(long i=0;i<n;++i)y[i]=qldpc_atanh(x[i]);}\n"
                   "void vl(const double*x,double*y,long n){for(long i=0;i<n;++i)y[i]=qldpc_np_log(x[i]);}\n"
                   "void vp(const double*x,double*y,long n){for(long i=0;i<n;++i)y[i]=qldpc_prior_llr(x[i],1e-9);}\n")
    so = d / "probe.so"
    subprocess.run(["gcc", "-O2", "-mfma", "-fPIC", "-ffp-contract=off", "-shared", "-I",
                    os.path.join(ROOT, "include"), "-o", str(so), str(src)], check=True)
    return ctypes.CDLL(str(so))


def _run(L, fn, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    getattr(L, fn)(x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p),
                   ctypes.c_long(len(x)))
    return y


def _assert_bits(got, want, x):
    bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
    assert bad.size == 0, f"{bad.size} differ, e.g. x={x[bad[:4]]} got={got[bad[:4]]} numpy={want[bad[:4]]}"


def test_tanh_equals_numpy(probe):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-40, 40, 300000), rng.uniform(-1, 1, 200000),
                        10 ** rng.uniform(-12, 2, 200000) * rng.choice([-1, 1], 200000),
                        rng.standard_normal(200000) * 6,
                        [0.0, -0.0, 1e-300, 2.0 ** -1022, 1e308, np.inf, -np.inf]])
    _assert_bits(_run(probe, "vt", x), np.tanh(x), x)


def test_atanh_equals_numpy(probe):
    rng = np.random.default_rng(1)
    z = np.concatenate([rng.uniform(-1, 1, 300000), 1 - 10 ** rng.uniform(-16, 0, 200000),
                        -(1 - 10 ** rng.uniform(-16, 0, 100000)), 10 ** rng.uniform(-15, 0, 100000),
                        np.tanh(rng.standard_normal(200000) * 8) * (1 - 1e-9), [0.0, -0.0, 1e-300]])
    z = z[np.abs(z) < 1]
    _assert_bits(_run(probe, "va", z), np.arctanh(z), z)


def test_log_equals_numpy(probe):
    rng = np.random.default_rng(2)
    x = np.concatenate([np.exp(rng.uniform(-700, 700, 300000)), rng.uniform(0.5, 2, 200000),
                        rng.uniform(1, 1e9, 100000)])
    _assert_bits(_run(probe, "vl", x), np.log(x), x)


def test_prior_llr_equals_numpy_on_priors(probe):
    """L = np.log((1-p)/max(p, eps)) for the decoder priors p = p_phys/3:
    glibc's log differs from NumPy's on ~0.2 % of them."""
    rng = np.random.default_rng(3)
    p = np.concatenate([rng.uniform(0, 0.5, 200000), np.arange(1, 2000) / 3e3, [1e-12, 1e-9, 0.0]])
    want = np.array([np.log((1 - q) / max(q, 1e-9)) for q in p])
    _assert_bits(_run(probe, "vp", p), want, p)


def test_special_values(probe):
    t = _run(probe, "vt", np.array([0.0, -0.0, np.inf, -np.inf, 22.0, -30.0, 1e-300]))
    assert t[0] == 0 and np.signbit(t[1]) and t[2] == 1 and t[3] == -1 and t[4] == 1 and t[5] == -1
    a = _run(probe, "va", np.array([0.0, 1.0, -1.0, 1 - 1e-9, 2.0]))
    assert a[0] == 0 and np.isposinf(a[1]) and np.isneginf(a[2]) and np.isnan(a[4])
    assert a[3] == np.arctanh(1 - 1e-9)


def test_tanh_saturates_at_bp_threshold(probe):
    """decoder_kernels.hip's saturated check-node path (kBpTanhSat = 19.5)
    takes tanh(x) = +-1.0 exactly for every |x| >= 19.5: dense and random
    arguments over [19.5, 24) (the polynomial interval) and beyond, against
    the restatement and NumPy; just below, tanh is not yet 1 everywhere."""
    rng = np.random.default_rng(7)
    lo = np.nextafter(19.5, 0.0)
    x = np.concatenate([np.linspace(19.5, 24.0, 2_000_001), rng.uniform(19.5, 24.0, 2_000_000),
                        rng.uniform(24.0, 1e6, 200_000), [19.5, 24.0, np.nextafter(24.0, 0.0), 1e300]])
    for s in (1.0, -1.0):
        got = _run(probe, "vt", s * x)
        assert np.all(got == s), "restated tanh below 1 past the threshold"
        assert np.all(np.tanh(s * x) == s), "NumPy's tanh below 1 past the threshold"
    below = np.linspace(18.0, lo, 100_001)
    assert np.any(_run(probe, "vt", below) != 1.0)
