"""Reliability order for OSD (decoders.py:320-325) on the host: the batched
osd_perms must give NumPy's literal per-row order bit for bit, and the
library's restatement of NumPy's own functions — SVML's exp8_ha and
x86-simd-sort's argsort, which the device order kernel also runs — must equal
np.exp / np.argsort themselves (the reference's calls), ties included."""
import numpy as np
import pytest

from qldpcsim_amd import decoders


def _literal_rel(P):
    sat = np.where(np.abs(P) < 100.0, P, 100.0 * np.sign(P))
    prob = 1. / (1. + np.exp(sat))
    return np.where(prob > 0.5, prob, 1 - prob)


def _posteriors(rows, n, seed):
    rng = np.random.default_rng(seed)
    P = rng.normal(0, 4, (rows, n))
    P[::3, ::7] *= 1e12                                  # saturated: many reliability ties at 1.0
    P[::5, 2::9] = 2.5                                   # exact duplicates
    P[::5, 4::9] = -2.5                                  # +-x pairs (reliabilities may differ by an ulp)
    P[1, :12] = [0.0, -0.0, 100.0, -100.0, np.inf, -np.inf, 99.99999999999999,
                 -100.00000000000001, 1e-300, -1e-300, 36.7, -36.7]
    # MS-like posteriors: L + float32 sums (quantised, heavily tied)
    L = np.log((1 - 0.1 / 3) / (0.1 / 3))
    P[2::4] = L + rng.integers(-6, 7, (P[2::4].shape)).astype(np.float32) * np.float32(0.75 * 1.3)
    return P


@pytest.mark.parametrize("rows,n,threads", [(7, 1020, 1), (300, 544, 4), (1100, 1020, 8)])
def test_osd_perms_match_literal_reference(rows, n, threads):
    P = _posteriors(rows, n, rows)
    got = decoders.osd_perms(P, threads)
    assert got.dtype == np.int32 and got.shape == (rows, n)
    for r in range(rows):
        np.testing.assert_array_equal(got[r], np.argsort(_literal_rel(P[r])))
        np.testing.assert_array_equal(got[r], decoders.osd_perm(P[r]))


def test_fast_reliability_is_bit_identical():
    P = _posteriors(256, 1020, 3)
    t = np.clip(P, -100.0, 100.0)
    np.exp(t, out=t)
    np.add(t, 1.0, out=t)
    np.divide(1.0, t, out=t)
    np.maximum(t, np.subtract(1.0, t), out=t)
    np.testing.assert_array_equal(t.view(np.uint64), _literal_rel(P).view(np.uint64))


def _host(fn):
    from qldpcsim_amd import _lib
    return getattr(_lib.lib, fn), _lib.ptr


def _np_keys(P):
    return _literal_rel(np.asarray(P, np.float64))


def _pinned_numpy():
    """This restatement is NumPy 2.2.6's AVX512_SKX code path (SVML exp8_ha,
    x86-simd-sort argsort); other NumPy builds may dispatch elsewhere."""
    from numpy._core._multiarray_umath import __cpu_features__ as f
    return np.__version__.startswith("2.2.") and bool(f.get("AVX512_SKX"))


needs_pinned = pytest.mark.skipif(not _pinned_numpy(), reason="NumPy is not the pinned 2.2 / AVX512_SKX build")


@needs_pinned
def test_np_exp_restated_bit_exact():
    """np.exp (SVML __svml_exp8_ha) restated in include/qldpc_libm.h: every
    value of [-707, 707] sampled, the clip range densely, the 2^(j/16) table
    boundaries and their neighbours, signed zeros, subnormals, NaN."""
    f, ptr = _host("qldpc_osd_keys_host")
    rng = np.random.default_rng(11)
    k = np.arange(-16 * 1000, 16 * 1000) * (np.log(2) / 16)
    x = np.concatenate([rng.uniform(-707, 707, 2_000_000), rng.uniform(-100, 100, 3_000_000),
                        rng.normal(0, 1, 500_000), rng.normal(0, 1e-9, 50_000), k,
                        np.nextafter(k, np.inf), np.nextafter(k, -np.inf),
                        [0.0, -0.0, 5e-324, -5e-324, 1e-300, -1e-300, np.nan, 700.0, -700.0]])
    got = np.empty_like(x)
    f(ptr(x), x.size, ptr(got), 1)
    want = np.exp(x)
    same = (got.view(np.uint64) == want.view(np.uint64)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), x[~same][:8]


@needs_pinned
def test_osd_keys_restated_bit_exact():
    f, ptr = _host("qldpc_osd_keys_host")
    P = _posteriors(64, 1020, 5).ravel()
    P = np.concatenate([P, [np.inf, -np.inf, np.nan, 1e308, -1e308]])
    got = np.empty_like(P)
    f(ptr(P), P.size, ptr(got), 0)
    want = _np_keys(P)
    same = (got.view(np.uint64) == want.view(np.uint64)) | (np.isnan(got) & np.isnan(want))
    assert same.all()


def _argsort_cases(seed, count):
    rng = np.random.default_rng(seed)
    for i in range(count):
        n = int(rng.choice([rng.integers(1, 40), rng.integers(1, 300), rng.integers(250, 2100)]))
        kind = i % 8
        if kind == 0:
            a = rng.random(n)
        elif kind == 1:
            a = rng.integers(0, 3, n).astype(float)                 # few distinct keys
        elif kind == 2:
            a = rng.integers(0, 60, n).astype(float)
        elif kind == 3:
            a = np.where(rng.random(n) < 0.85, 1.0, rng.random(n))  # saturated: a long 1.0 run
        elif kind == 4:
            a = np.full(n, 0.75)                                    # all equal
        elif kind == 5:
            a = np.sort(rng.integers(0, 9, n).astype(float))        # sorted, tied
        elif kind == 6:
            a = np.sort(rng.random(n))[::-1].copy()                 # reversed
        else:
            a = np.where(rng.random(n) < 0.5, -0.0, 0.0) + rng.integers(0, 2, n)   # +-0 ties
        yield np.ascontiguousarray(a, np.float64)


@needs_pinned
def test_argsort_restated_matches_numpy_ties_included():
    """x86-simd-sort's argsort as np.argsort runs it (np_order.cpp): the
    permutation itself, equal keys included, on every case that does not end
    in the library's std::sort fallback (status 1: NumPy decides those)."""
    f, ptr = _host("qldpc_np_argsort_host")
    checked = fallback = 0
    for a in _argsort_cases(1, 6000):
        out = np.empty(a.size, np.int32)
        rc = f(ptr(a), a.size, ptr(out))
        if rc == 1:
            fallback += 1
            continue
        assert rc == 0
        np.testing.assert_array_equal(out, np.argsort(a))
        checked += 1
    assert checked > 5000


def test_argsort_restated_reports_nan_and_fallback():
    f, ptr = _host("qldpc_np_argsort_host")
    a = np.array([0.5, np.nan, 0.7])
    out = np.empty(3, np.int32)
    assert f(ptr(a), 3, ptr(out)) == 1
    # a segment whose pivot keeps being its smallest key exhausts the
    # 2 floor(log2 n) levels (x86-simd-sort then calls std::sort)
    rng = np.random.default_rng(4)
    hits = 0
    for _ in range(200):
        b = np.where(rng.random(2000) < 0.9, 0.5, rng.random(2000) + 0.5)
        o = np.empty(b.size, np.int32)
        hits += f(ptr(b), b.size, ptr(o)) == 1
    assert hits > 0


@needs_pinned
@pytest.mark.parametrize("fname", ["ms_LP118_2_osd50.npz", "ms_LP118_0_osd.npz", "bp_LP04_0_osd.npz"])
def test_osd_order_host_equals_numpy_on_reference_posteriors(fname):
    """The reference's own posteriors (golden captures of MS_decoder /
    BP_decoder): qldpc_osd_order_host == decoders.py:320-325 per row."""
    import os
    from conftest import GOLDEN, load_golden
    f, ptr = _host("qldpc_osd_order_host")
    rows = 0
    for c, a in load_golden(os.path.join(GOLDEN, fname)):
        P = np.ascontiguousarray(a["post"], np.float64)
        k, n = P.shape
        perm = np.empty((k, n), np.int32)
        st = np.empty(k, np.int32)
        assert f(ptr(P), k, n, ptr(perm), ptr(st), 4) == 0
        for r in range(k):
            if st[r] == 0:
                np.testing.assert_array_equal(perm[r], np.argsort(_literal_rel(P[r])))
                rows += 1
    assert rows > 0


@needs_pinned
def test_numpy_order_pinned_and_host_perms_exact():
    assert decoders.numpy_order_pinned()
    P = _posteriors(300, 1020, 9)
    P[5, 3] = np.nan                                       # a row NumPy itself must order
    got = decoders.osd_perms(P, 4)
    for r in range(P.shape[0]):
        np.testing.assert_array_equal(got[r], decoders.osd_perm(P[r]))
