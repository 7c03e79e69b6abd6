"""Host reliability order for OSD (decoders.py:320-325): the batched,
rewritten osd_perms must give NumPy's literal per-row order bit for bit —
the same reliabilities, so NumPy's argsort breaks every tie the same way."""
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


def test_numpy_exp_within_one_ulp_on_the_reliability_domain():
    """The device reliability order (qldpc_osd_order_device) certifies NumPy's
    order where adjacent keys differ by more than 64 units in the last place;
    that margin assumes NumPy's exp is within a few ulp of the true value on
    [-100, 100]. Checked here against long-double exp."""
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-100, 100, 400000), rng.uniform(-1, 1, 100000)])
    got = np.exp(x)
    ref = np.exp(x.astype(np.longdouble))
    ulp = np.spacing(got)
    err = np.abs((got.astype(np.longdouble) - ref) / ulp.astype(np.longdouble))
    assert float(err.max()) <= 1.0
