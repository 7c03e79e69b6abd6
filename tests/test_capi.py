"""C ABI (include/qldpc_decoder.h): the library loads on CPU, exports every
declared symbol, validates arguments with the reference's error types, and the
host-side services (OSD, CPython set order) work without a GPU. No decode
compute happens here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden_cases, half_matrix

from qldpcsim_amd import _lib


def _declared():
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h") and fn != "qldpc_libm.h":
            txt = open(os.path.join(ROOT, "include", fn)).read()
            names |= set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(qldpc_\w+)\s*\(", txt, re.M))
    return names


def test_every_declared_symbol_is_exported():
    declared = _declared()
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name


def test_library_options_roundtrip_and_unknown_names():
    """qldpc_set_option / qldpc_get_option: every documented name with its
    default, set / restore through the context manager, ValueError for an
    unknown name (the library itself never reads the environment)."""
    defaults = {"force_hbm": 0, "flood_generic": 0, "layered_generic": 0, "ms_lanes_per_check": 0, "bp_wave": 0,
                "bp_lg": 1, "bp_team_w": 0, "static_sched": 0, "waves_per_wg": 0, "wg_per_cu": 0,
                "osd_column": 0, "osd_tickets": 1, "osd_prof": 0, "osd_hbm": 0}
    for k, v in defaults.items():
        assert _lib.get_option(k) == v, k
    with _lib.options(force_hbm=1, bp_team_w=8):
        assert _lib.get_option("force_hbm") == 1 and _lib.get_option("bp_team_w") == 8
    assert _lib.get_option("force_hbm") == 0 and _lib.get_option("bp_team_w") == 0
    with pytest.raises(ValueError, match="unknown option"):
        _lib.set_option("no_such_option", 1)
    import glob
    import re
    for f in glob.glob(os.path.join(ROOT, "qldpcsim_amd", "csrc", "*.cpp")):
        # options never come from the environment; the one variable read is
        # the host thread budget's OMP_NUM_THREADS (hostcores.py's convention)
        calls = re.findall(r"getenv\(([^)]*)\)", open(f).read())
        assert set(calls) <= {'"OMP_NUM_THREADS"'}, (f, calls)


def test_version_and_device_count():
    assert b"gfx950" in _lib.lib.qldpc_version()
    assert _lib.device_count() >= 0


def test_schedule_validation_errors():
    Hx = np.eye(4, 6, dtype=np.uint8)
    code = _lib.Code(Hx)
    with pytest.raises(IndexError):                      # reference: IndexError (decoders.py:156)
        code.schedule(np.array([0, 2], np.int32), np.array([0, 7], np.int32))
    with pytest.raises(ValueError):
        code.schedule(np.array([0, 3, 1], np.int32), np.array([0, 1, 2], np.int32))


@pytest.mark.skipif(_lib.device_count() > 0, reason="checks the no-device failure mode")
def test_decode_fails_loudly_without_a_device():
    from qldpcsim_amd import decoders
    H = np.array([[1, 1, 0], [0, 1, 1]], np.int8)
    with pytest.raises(RuntimeError, match="no HIP device"):
        decoders.MS_decoder(H, np.array([1, 0]), 0.01, max_iter=5, layers=[np.arange(2)])


def test_cpython_set_difference_order_emulation():
    """infoSet = list(set(range(n)) - set(J)) (decoders.py:344): the emulated
    first element equals the interpreter's, including hash-table wrap cases."""
    rng = np.random.default_rng(0)
    for _ in range(1500):
        n = int(rng.integers(1, 2500))
        k = int(rng.integers(0, n + 1))
        J = rng.choice(n, size=k, replace=False).astype(np.int32)
        s = list(set(range(n)) - set(J.tolist()))
        want = s[0] if s else -1
        assert _lib.lib.qldpc_cpython_setdiff_first(n, _lib.ptr(J), k) == want


OSD = [(c, a) for c, a in golden_cases("_osd") if c["osd"] >= 0]
OSD50 = golden_cases("_osd50")


@pytest.mark.parametrize("ca", OSD, ids=[f"{c['algo']}-{c['code']}-osd{c['osd']}-{c['id']}" for c, _ in OSD])
def test_osd_matches_reference_golden(ca):
    """Host OSD (C++ bit-packed GF(2)) on the oracle's posteriors reproduces the
    reference's post-OSD error estimates (decoders.py:299-370)."""
    from oracle import oracle
    from qldpcsim_amd import decoders
    c, a = ca
    H = half_matrix(c)
    e, it, post, _ = oracle.decode_batch(c["algo"], H, a["syn"], c["p_phys"] / 3, c["max_iter"],
                                         a["layer_ptr"], a["layer_rows"])
    for k in range(len(it)):
        conv = np.all((H.astype(np.int64) @ e[k]) % 2 == a["syn"][k])
        ek = e[k].astype(np.int8)
        if not conv:
            ek = decoders.OSDdec(H, ek, a["syn"][k].astype(int), post[k], c["osd"])
        np.testing.assert_array_equal(ek.astype(np.uint8), a["ehat"][k])


@pytest.mark.parametrize("order", [0, 1])
def test_osd_matches_reference_golden_at_configs3_setting(order):
    """configs[3]'s setting (LP118_2, MS layered, 50 iterations, p = 0.1):
    for every non-converged golden shot, the host OSD on the reference's own
    final posteriors gives the reference's post-OSD estimate (OSD-0 and
    OSD-1, decoders.py:179-180 -> :299-370). These posteriors carry the exact
    min-sum ties that drive the GPU order's certification."""
    from qldpcsim_amd import decoders
    n_osd = 0
    for c, a in OSD50:
        H = half_matrix(c)
        for k in np.flatnonzero(a["conv"] == 0):
            ek = decoders.OSDdec(H, a["ehat"][k].astype(np.int8), a["syn"][k].astype(int), a["post"][k], order)
            np.testing.assert_array_equal(ek.astype(np.uint8), a[f"ehat_osd{order}"][k])
            n_osd += 1
    assert n_osd >= 64, n_osd


def test_osd_random_matches_oracle_restatement():
    """Random (H, syndrome, posterior) triples: C++ OSD == NumPy restatement
    for orders 0, 1, 2 (order >= 2 equals order 0)."""
    from oracle import oracle
    from qldpcsim_amd import codes, decoders
    rng = np.random.default_rng(5)
    Hx, Hz = codes.load_code("LP04_0")
    for trial in range(6):
        H = Hz if trial % 2 else Hx
        syn = rng.integers(0, 2, H.shape[0])
        post = rng.normal(0, 3, H.shape[1])
        post[rng.integers(0, H.shape[1], 10)] = 2.5           # ties in the reliability order
        e0 = (post < 0).astype(np.int8)
        for order in (0, 1, 2):
            want = oracle.osd_dec(H, e0.astype(np.int64), syn, post, order)
            got = decoders.OSDdec(H, e0.copy(), syn, post, order)
            np.testing.assert_array_equal(got, want)
            if order == 2:
                np.testing.assert_array_equal(got, decoders.OSDdec(H, e0.copy(), syn, post, 0))
