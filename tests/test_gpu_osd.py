"""GPU OSD (qldpc_osd_device) against the host C++ OSD and the reference's
golden post-OSD estimates; orders 0, 1, 2, 4 (SURVEY App. A.4 semantics)."""
import numpy as np
import pytest

from conftest import golden_cases, half_matrix

pytestmark = pytest.mark.gpu


def _gpu_osd(H, syn, e, post, order):
    import torch
    from qldpcsim_amd import _lib, decoders
    code = _lib.code_for(H, 0)
    perms = torch.as_tensor(decoders.osd_perms(post), device="cuda")
    s = torch.as_tensor(np.ascontiguousarray(syn, np.uint8), device="cuda")
    ed = torch.as_tensor(np.ascontiguousarray(e, np.uint8), device="cuda")
    st = torch.empty(len(e), dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.qldpc_osd_device(code.handle, len(e), s.data_ptr(), perms.data_ptr(), order,
                                         ed.data_ptr(), st.data_ptr(), None))
    torch.cuda.synchronize()
    return ed.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("code", ["steane", "LP04_0", "LP118_0", "LP118_2", "T", "bicycle"])
@pytest.mark.parametrize("order", [0, 1, 2, 4])
def test_gpu_osd_matches_host_osd(code, order):
    from qldpcsim_amd import _lib, codes, decoders
    Hx, Hz = codes.load_code(code)
    rng = np.random.default_rng(hash((code, order)) % 2**32)
    for H in (Hx, Hz):
        k = 48
        syn = rng.integers(0, 2, (k, H.shape[0])).astype(np.uint8)
        # half consistent syndromes (valid errors), half arbitrary (inconsistent)
        err = (rng.random((k // 2, H.shape[1])) < 0.05).astype(np.int64)
        syn[: k // 2] = (err @ H.T.astype(np.int64)) % 2
        post = rng.normal(0, 3, (k, H.shape[1]))
        post[:, ::5] = 1.75                         # ties in the reliability order
        e0 = (post < 0).astype(np.uint8)
        got, st = _gpu_osd(H, syn, e0, post, order)
        assert np.all(st == 0)
        code_h = _lib.code_for(H)
        want = e0.copy()
        perms = np.ascontiguousarray(decoders.osd_perms(post), np.int32)
        _lib.check(_lib.lib.qldpc_osd_decode_batch(code_h.handle, k, _lib.ptr(syn), _lib.ptr(perms),
                                                   order, _lib.ptr(want), 1))
        np.testing.assert_array_equal(got, want)
        # consistent syndromes are always satisfied after OSD
        np.testing.assert_array_equal((got[: k // 2].astype(np.int64) @ H.T) % 2, syn[: k // 2])


OSD = golden_cases("_osd")


@pytest.mark.parametrize("ca", OSD, ids=[f"{c['algo']}-{c['code']}-osd{c['osd']}-{c['id']}" for c, _ in OSD])
def test_gpu_osd_matches_reference_golden(ca):
    from oracle import oracle
    c, a = ca
    H = half_matrix(c)
    e, it, post, _ = oracle.decode_batch(c["algo"], H, a["syn"], c["p_phys"] / 3, c["max_iter"],
                                         a["layer_ptr"], a["layer_rows"])
    conv = np.all(((e.astype(np.int64) @ H.T.astype(np.int64)) % 2) == a["syn"], axis=1)
    if conv.all():
        return
    idx = np.flatnonzero(~conv)
    got, st = _gpu_osd(H, a["syn"][idx], e[idx], post[idx], c["osd"])
    assert np.all(st == 0)
    np.testing.assert_array_equal(got, a["ehat"][idx])


def test_gpu_osd_index_error_case():
    # rank-1 H whose first (least reliable) column is nonzero: the reference's
    # greedy loop never raises the rank again and indexes past column n-1
    H = np.array([[1, 1, 0, 1], [1, 1, 0, 1]], np.int8)
    got, st = _gpu_osd(H, np.array([[1, 1]], np.uint8), np.zeros((1, 4), np.uint8),
                       np.array([[0.1, 5.0, 6.0, 7.0]]), 0)
    assert st[0] == 1
    from qldpcsim_amd import decoders
    with pytest.raises(IndexError):
        decoders.OSDdec(H, np.zeros(4, np.int8), np.array([1, 1]), np.array([0.1, 5.0, 6.0, 7.0]), 0)
