"""Run-time parity pins (decoders.numpy_order_pinned / numpy_libm_pinned /
parity_pins): the restated NumPy routines the kernels run — the OSD
reliability order (np.exp + np.argsort, decoders.py:320-325) and BP's tanh /
arctanh / the priors' log (decoders.py:147, :232, :254-259) — against the
running NumPy, with a warning that names the reason when they differ."""
import ctypes

import numpy as np
import pytest

from qldpcsim_amd import _lib, decoders


def _skx():
    try:
        from numpy._core._multiarray_umath import __cpu_features__
    except ImportError:
        return False
    return bool(__cpu_features__.get("AVX512_SKX")) and np.__version__ == "2.2.6"


@pytest.fixture
def fresh_pins(monkeypatch):
    monkeypatch.setattr(decoders, "_PINNED", {})
    yield


@pytest.mark.skipif(not _skx(), reason="the restatement is NumPy 2.2.6 AVX512_SKX's")
def test_pins_hold_on_the_capture_numpy(fresh_pins):
    pins = decoders.parity_pins()
    assert pins["order"] and pins["libm"], pins
    assert pins["numpy"] == np.__version__
    assert set(pins["reasons"]) == {"order", "libm"}


def test_libm_eval_host_matches_header_functions():
    """qldpc_libm_eval_host is element-wise and rejects unknown functions."""
    x = np.array([0.0, 0.25, -3.0, 19.5], np.float64)
    y = np.empty_like(x)
    _lib.check(_lib.lib.qldpc_libm_eval_host(0, _lib.ptr(x), x.size, _lib.ptr(y)))
    assert y[0] == 0.0 and y[3] == 1.0 and abs(y[2] - np.tanh(-3.0)) < 1e-15
    assert _lib.lib.qldpc_libm_eval_host(9, _lib.ptr(x), x.size, _lib.ptr(y)) != 0
    assert _lib.lib.qldpc_libm_eval_host(0, None, 0, None) == 0


def test_libm_pin_failure_warns_with_reason(fresh_pins, monkeypatch):
    def identity(fn, px, n, py):                      # a "libm" that returns its argument
        ctypes.memmove(py, px, 8 * n)
        return 0
    monkeypatch.setattr(_lib.lib, "qldpc_libm_eval_host", identity)
    with pytest.warns(RuntimeWarning, match="np.tanh differs"):
        assert decoders.numpy_libm_pinned() is False
    pins = decoders.parity_pins()
    assert pins["libm"] is False and "tanh" in pins["reasons"]["libm"]


def test_order_pin_failure_warns_and_routes_orders_to_numpy(fresh_pins, monkeypatch):
    def missing(*a):
        raise AttributeError("qldpc_osd_order_host")
    monkeypatch.setattr(_lib.lib, "qldpc_osd_order_host", missing)
    with pytest.warns(RuntimeWarning, match="reliability order"):
        assert decoders.numpy_order_pinned() is False
    # the orders then come from NumPy itself (decoders.py:320-325)
    post = np.random.default_rng(1).normal(0, 3, (5, 40))
    np.testing.assert_array_equal(decoders.osd_perms(post), np.stack([decoders.osd_perm(r) for r in post]))
    assert "AttributeError" in decoders.parity_pins()["reasons"]["order"]
