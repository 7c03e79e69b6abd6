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
    import zlib
    Hx, Hz = codes.load_code(code)
    # a reproducible seed per case (Python's str hash is salted per process)
    rng = np.random.default_rng(zlib.crc32(f"{code}-{order}".encode()))
    for H in (Hx, Hz, Hx, Hz):
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


OSD = [(c, a) for c, a in golden_cases("_osd") if c["osd"] >= 0]


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


def _device_order(H, post):
    import torch
    from qldpcsim_amd import _lib
    code = _lib.code_for(H, 0)
    k, n = post.shape
    p = torch.as_tensor(np.ascontiguousarray(post, np.float64), device="cuda")
    perm = torch.empty((k, n), dtype=torch.int32, device="cuda")
    tie = torch.empty(k, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.qldpc_osd_order_device(code.handle, k, p.data_ptr(), perm.data_ptr(), tie.data_ptr(), None))
    torch.cuda.synchronize()
    return perm.cpu().numpy(), tie.cpu().numpy()


def _decoded_posteriors(code, p, shots, it, seed):
    """Posteriors of non-converged layered MS decodes (the shots OSD sees)."""
    from oracle import oracle
    from qldpcsim_amd import codes, schedule, simulator
    Hx, Hz = codes.load_code(code)
    lx, _ = schedule.select_layers(Hx, Hz, "L")
    lp, lr = schedule.pack_layers(lx, Hz.shape[0])
    syn = simulator.sample_channel(Hx, Hz, p, shots, np.random.default_rng(seed))[0]
    e, iters, post, _ = oracle.decode_batch("MS", Hz, syn, p / 3, it, lp, lr)
    bad = np.any(((e.astype(np.int64) @ Hz.T.astype(np.int64)) % 2) != syn, axis=1)
    return Hz, syn[bad], e[bad], post[bad]


def _host_order(post):
    """qldpc_osd_order_host: the library's host restatement (C++) of NumPy's
    reliability order; status 1 rows are NumPy's to decide."""
    from qldpcsim_amd import _lib
    P = np.ascontiguousarray(post, np.float64)
    k, n = P.shape
    perm = np.empty((k, n), np.int32)
    st = np.empty(k, np.int32)
    _lib.check(_lib.lib.qldpc_osd_order_host(_lib.ptr(P), k, n, _lib.ptr(perm), _lib.ptr(st), 8))
    return perm, st


def _pinned():
    from qldpcsim_amd import decoders
    return decoders.numpy_order_pinned()


@pytest.mark.parametrize("code,p", [("LP118_2", 0.1), ("LP118_0", 0.08), ("LP04_0", 0.12)])
def test_device_order_equals_numpy_exactly(code, p):
    """qldpc_osd_order_device is NumPy's order (decoders.py:320-325), every
    position, ties included: equal to the host restatement always, and to
    np.argsort itself when this host's NumPy is the pinned build, on the
    posteriors of real non-converged decodes and on random / tie-heavy /
    saturated / NaN rows."""
    from qldpcsim_amd import decoders
    H, syn, e, post = _decoded_posteriors(code, p, 600, 30, 7)
    rng = np.random.default_rng(2)
    n = H.shape[1]
    extra = rng.normal(0, 4, (72, n))
    extra[:16, ::3] = 2.5                                   # exact ties
    extra[16:32] = np.round(extra[16:32] * 4) / 4            # many ties
    extra[32:40, :7] = [150, -150, 99.5, -99.5, 37.0, -40.0, 0.0]   # clipped / saturated keys
    extra[40:48] *= 1e3                                      # mostly saturated: one long 1.0 run
    extra[48:56] = 1.0                                       # all keys equal
    extra[56:60, 3] = np.nan                                 # NumPy's NaN path: left to the host
    post = np.concatenate([post, extra])
    perm, tie = _device_order(H, post)
    hperm, hst = _host_order(post)
    nanrow = np.isnan(post).any(axis=1)
    np.testing.assert_array_equal(tie, np.where(hst == 0, n, -1))
    assert (tie[nanrow] == -1).all() and (tie[~nanrow] == n).mean() > 0.95
    ok = tie == n
    np.testing.assert_array_equal(perm[ok], hperm[ok])
    if _pinned():
        want = decoders.osd_perms(post)
        np.testing.assert_array_equal(perm[ok], want[ok])


@pytest.mark.parametrize("n", [1, 2, 7, 100, 255, 256, 257, 300, 511, 700, 1500, 2047, 2048])
def test_device_order_any_size(n):
    """Every segment path of the device argsort (one bitonic network, one
    partition level, several, the scalar steps of every residue mod 32) on
    sizes 1 .. 2048, with key distributions that end in each of x86-simd-sort's
    cases, including its std::sort fallback (tiepos -1, as the host's status 1)."""
    rng = np.random.default_rng(n)
    H = (rng.random((max(1, n // 3), n)) < 0.05).astype(np.uint8)
    H[0, :] = 1
    rows = [rng.normal(0, 5, n), np.round(rng.normal(0, 3, n)), rng.normal(0, 5, n) * 1e3,
            np.full(n, 1.5), np.where(rng.random(n) < 0.9, 0.0, rng.normal(0, 3, n)),
            np.where(rng.random(n) < 0.5, 50.0, -50.0) * rng.integers(1, 3, n)]
    rows += [np.round(rng.normal(0, 2, n) * 2) / 2 for _ in range(26)]
    post = np.stack(rows)
    perm, tie = _device_order(H, post)
    hperm, hst = _host_order(post)
    np.testing.assert_array_equal(tie, np.where(hst == 0, n, -1))
    ok = tie == n
    np.testing.assert_array_equal(perm[ok], hperm[ok])
    if _pinned():
        from qldpcsim_amd import decoders
        for r in np.flatnonzero(ok):
            np.testing.assert_array_equal(perm[r], decoders.osd_perm(post[r]))


def test_device_order_equals_numpy_on_a_configs3_batch():
    """Every OSD shot of a configs[3] batch (LP118_2 MS layered, 50 iterations,
    p = 0.1, device sampler and decoder): the device order equals the host
    restatement on every shot and np.argsort on every shot (pinned NumPy),
    and no shot is left to the host."""
    import torch
    from qldpcsim_amd import _lib, codes, decoders, schedule, simulator
    Hx, Hz = codes.load_code("LP118_2")
    lx, _ = schedule.select_layers(Hx, Hz, "L")
    lp, lr = schedule.pack_layers(lx, Hz.shape[0])
    dev = torch.device("cuda", 0)
    ch = simulator.DeviceChannel(Hx, Hz, dev, 20260101)
    sy_z = ch.sample(0.1, 16384)[0]
    r = decoders.decode_batch(Hz, sy_z, 0.1 / 3, 50, algo="MS", want_post=True, layer_ptr=lp, layer_rows=lr)
    bad = ((r.flags & _lib.FLAG_CONVERGED) == 0).nonzero().flatten()
    post = r.post.index_select(0, bad).cpu().numpy()
    assert post.shape[0] > 4000
    perm, tie = _device_order(Hz, post)
    assert (tie == Hz.shape[1]).all()
    hperm, hst = _host_order(post)
    assert (hst == 0).all()
    np.testing.assert_array_equal(perm, hperm)
    if _pinned():
        np.testing.assert_array_equal(perm, decoders.osd_perms(post))


@pytest.mark.parametrize("code,p,order", [("LP118_2", 0.1, 0), ("LP118_0", 0.08, 1), ("LP04_0", 0.12, 4)])
def test_ordered_device_osd_equals_numpy_ordered_osd(code, p, order, osdpol):
    """qldpc_osd_device_ordered gives the NumPy-ordered result on every shot
    (status 0: the device order is NumPy's); the apply_osd_device path equals
    the host OSD with NumPy's order on every shot."""
    import torch
    from qldpcsim_amd import _lib, decoders
    H, syn, e, post = _decoded_posteriors(code, p, 800, 30, 9)
    k = len(syn)
    code_h = _lib.code_for(H, 0)
    d = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dt), device="cuda")  # noqa: E731
    s_d, p_d, e_d = d(syn, np.uint8), d(post, np.float64), d(e, np.uint8)
    st = torch.empty(k, dtype=torch.int32, device="cuda")
    perm = torch.empty((k, H.shape[1]), dtype=torch.int32, device="cuda")
    tie = torch.empty(k, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.qldpc_osd_device_ordered(code_h.handle, k, s_d.data_ptr(), p_d.data_ptr(), order,
                                                 e_d.data_ptr(), st.data_ptr(), perm.data_ptr(), tie.data_ptr(),
                                                 None))
    got, status = e_d.cpu().numpy(), st.cpu().numpy()
    want, wst = _gpu_osd(H, syn, e, post, order)
    assert np.all(wst == 0) and np.all(status == 0)
    np.testing.assert_array_equal(got, want)
    # the full device path with the host fallback (device order at any count)
    osdpol(device_min=1)
    res = decoders.DecodeResult(d(e, np.uint8), torch.zeros(k, dtype=torch.int32, device="cuda"), p_d,
                                torch.zeros(k, dtype=torch.int32, device="cuda"))
    decoders.apply_osd_device(H, s_d, res, order)
    np.testing.assert_array_equal(res.ehat.cpu().numpy(), want)


@pytest.mark.parametrize("code", ["LP04_0", "LP118_2", "bicycle"])
def test_block_kernel_matches_column_kernel(code, qopt):
    """The block elimination (pivots by row index, default) and the exact-REF
    column kernel (option osd_column) agree shot for shot, on consistent
    and inconsistent syndromes (the latter take the column kernel's second
    pass inside the block path)."""
    from qldpcsim_amd import codes
    Hx, _ = codes.load_code(code)
    rng = np.random.default_rng(5)
    k = 96
    syn = rng.integers(0, 2, (k, Hx.shape[0])).astype(np.uint8)
    err = (rng.random((k // 2, Hx.shape[1])) < 0.06).astype(np.int64)
    syn[: k // 2] = (err @ Hx.T.astype(np.int64)) % 2
    post = rng.normal(0, 3, (k, Hx.shape[1]))
    e0 = (post < 0).astype(np.uint8)
    for order in (0, 1):
        blk, sb = _gpu_osd(Hx, syn, e0, post, order)
        qopt(osd_column=1)
        col, sc = _gpu_osd(Hx, syn, e0, post, order)
        qopt(osd_column=0)
        assert np.all(sb == 0) and np.all(sc == 0)
        np.testing.assert_array_equal(blk, col)


def test_osd_zero_column_code():
    """An H with an all-zero column: the reference reads e_J off REF's own row
    order when column 0 of H[:, perm] has no pivot, so such codes use the
    column kernel; results equal the host OSD."""
    from qldpcsim_amd import _lib, codes, decoders
    Hx, _ = codes.load_code("steane")
    H = np.concatenate([np.zeros((Hx.shape[0], 1), Hx.dtype), Hx], axis=1)
    # a redundant row: rank(H) < m, so e_J's extra entry (J holds the zero
    # column besides rank(H) pivots) reads a non-pivot row, as REF leaves them
    # (with rank(H) = m the reference's e_J assignment itself fails to broadcast)
    H = np.concatenate([H, (H[:1] + H[1:2]) % 2], axis=0)
    rng = np.random.default_rng(11)
    k = 32
    syn = rng.integers(0, 2, (k, H.shape[0])).astype(np.uint8)
    post = rng.normal(0, 3, (k, H.shape[1]))
    post[: k // 2, 0] = 0.0                                  # the zero column first in the order
    e0 = (post < 0).astype(np.uint8)
    for order in (0, 1):
        got, st = _gpu_osd(H, syn, e0, post, order)
        want = e0.copy()
        perms = np.ascontiguousarray(decoders.osd_perms(post), np.int32)
        code_h = _lib.code_for(H)
        _lib.check(_lib.lib.qldpc_osd_decode_batch(code_h.handle, k, _lib.ptr(syn), _lib.ptr(perms),
                                                   order, _lib.ptr(want), 1))
        assert np.all(st == 0)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("code,order", [("LP118_2", 0), ("LP118_0", 1), ("LP04_0", 0)])
def test_ordered_device_osd_tie_runs(code, order):
    """Posteriors with many exact and near ties inside the decision prefix:
    the device path decides every shot (status 0) and equals the host OSD
    under NumPy's order."""
    import torch
    from qldpcsim_amd import _lib, decoders
    H, syn, e, post = _decoded_posteriors(code, 0.1 if code != "LP04_0" else 0.12, 800, 30, 13)
    rng = np.random.default_rng(4)
    q = post.copy()
    for r in range(0, len(q), 2):                              # exact tie pairs among the least
        idx = np.argsort(np.abs(q[r]), kind="stable")[4:24]    # reliable columns (inside the
        q[r, idx[1::2]] = q[r, idx[0::2]]                      # decision prefix)
    q[2::8] = np.round(q[2::8] * 2) / 2                         # tie-heavy rows
    q[1::4] += rng.normal(0, 1e-14, q[1::4].shape)             # near ties (within the margin)
    k = len(q)
    code_h = _lib.code_for(H, 0)
    d = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dt), device="cuda")  # noqa: E731
    s_d, p_d, e_d = d(syn, np.uint8), d(q, np.float64), d(e, np.uint8)
    st = torch.empty(k, dtype=torch.int32, device="cuda")
    perm = torch.empty((k, H.shape[1]), dtype=torch.int32, device="cuda")
    tie = torch.empty(k, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.qldpc_osd_device_ordered(code_h.handle, k, s_d.data_ptr(), p_d.data_ptr(), order,
                                                 e_d.data_ptr(), st.data_ptr(), perm.data_ptr(), tie.data_ptr(),
                                                 None))
    got, status, tie = e_d.cpu().numpy(), st.cpu().numpy(), tie.cpu().numpy()
    want = e.copy()
    perms = np.ascontiguousarray(decoders.osd_perms(q), np.int32)
    _lib.check(_lib.lib.qldpc_osd_decode_batch(_lib.code_for(H).handle, k, _lib.ptr(syn), _lib.ptr(perms),
                                               order, _lib.ptr(want), 1))
    assert np.all(status == 0) and np.all(tie == H.shape[1])
    np.testing.assert_array_equal(got, want)


def test_ordered_osd_spill_matches_status():
    """qldpc_osd_device_ordered_ex: every status-2 shot (a NaN posterior:
    NumPy's NaN path is the host's) and only those spills its posterior row
    and index; results equal the plain ordered call."""
    import torch
    from qldpcsim_amd import _lib
    H, syn, e, post = _decoded_posteriors("LP118_2", 0.1, 600, 30, 21)
    q = post.copy()
    q[::3, 17] = np.nan                                        # shots left to the host
    k, n = q.shape
    code_h = _lib.code_for(H, 0)
    d = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dt), device="cuda")  # noqa: E731
    outs = []
    for spill in (False, True):
        s_d, p_d, e_d = d(syn, np.uint8), d(q, np.float64), d(e, np.uint8)
        st = torch.empty(k, dtype=torch.int32, device="cuda")
        perm = torch.empty((k, n), dtype=torch.int32, device="cuda")
        tie = torch.empty(k, dtype=torch.int32, device="cuda")
        if spill:
            cap = k
            sp_post = torch.full((cap, n), np.nan, dtype=torch.float64, device="cuda")
            sp_idx = torch.full((cap,), -1, dtype=torch.int32, device="cuda")
            sp_cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
            _lib.check(_lib.lib.qldpc_osd_device_ordered_ex(
                code_h.handle, k, s_d.data_ptr(), p_d.data_ptr(), 0, e_d.data_ptr(), st.data_ptr(),
                perm.data_ptr(), tie.data_ptr(), sp_post.data_ptr(), sp_idx.data_ptr(), sp_cnt.data_ptr(), cap,
                None))
        else:
            _lib.check(_lib.lib.qldpc_osd_device_ordered(
                code_h.handle, k, s_d.data_ptr(), p_d.data_ptr(), 0, e_d.data_ptr(), st.data_ptr(),
                perm.data_ptr(), tie.data_ptr(), None))
        torch.cuda.synchronize()
        outs.append((e_d.cpu().numpy(), st.cpu().numpy()))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    status = outs[1][1]
    c = int(sp_cnt.item())
    two = np.flatnonzero(status == 2)
    assert c == two.size > 0
    idx = sp_idx[:c].cpu().numpy()
    assert sorted(idx.tolist()) == two.tolist()
    np.testing.assert_array_equal(sp_post[:c].cpu().numpy().view(np.uint64), q[idx].view(np.uint64))


def test_apply_osd_device_on_explicit_stream_and_rejects_packed_formats(osdpol):
    """apply_osd_device(..., stream=s) queues every kernel, copy and event on
    `s` (same result as torch's current stream), and refuses bit-packed
    decodes (int64 word syndromes / ehat_bits) instead of letting the byte-
    wide OSD kernels read and write past them."""
    import torch
    from qldpcsim_amd import decoders
    osdpol(device_min=1)
    H, syn, e, post = _decoded_posteriors("LP118_2", 0.1, 600, 30, 13)
    k = len(syn)
    d = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dt), device="cuda")  # noqa: E731
    want, _ = _gpu_osd(H, syn, e, post, 0)
    s = torch.cuda.Stream()
    res = decoders.DecodeResult(d(e, np.uint8), torch.zeros(k, dtype=torch.int32, device="cuda"),
                                d(post, np.float64), torch.zeros(k, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
    decoders.apply_osd_device(H, d(syn, np.uint8), res, 0, stream=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(res.ehat.cpu().numpy(), want)
    # bit-packed syndromes / estimates are refused
    s_bits = decoders.pack_bits(d(syn, np.uint8))
    with pytest.raises(ValueError):
        decoders.apply_osd_device(H, s_bits, res, 0)
    res_b = decoders.DecodeResult(decoders.pack_bits(d(e, np.uint8)), res.iters, res.post, res.flags)
    with pytest.raises(ValueError):
        decoders.apply_osd_device(H, d(syn, np.uint8), res_b, 0)


@pytest.mark.parametrize("device_min", ["1", "4096"])    # device reliability order / host order
@pytest.mark.parametrize("order", [0, 1])
def test_device_osd_pipeline_matches_reference_at_configs3(order, device_min, osdpol):
    """configs[3]'s setting from the reference itself (tests/golden/
    ms_LP118_2_osd50.npz: LP118_2 MS layered, 50 iterations, p = 0.1): the
    device decode reproduces the reference's iterations and posteriors, then
    the full device OSD path reproduces the reference's OSD-0 / OSD-1
    estimates on every non-converged shot (decoders.py:179-180, :299-370).
    device_min = 1: NumPy's reliability order computed on the device
    (osd_order_kernel), with no shot left to a host order; device_min = 4096
    (more than a golden batch's OSD shots): every order computed by NumPy on
    the host. Both then run the block elimination on the device."""
    import torch
    from conftest import golden_cases, half_matrix
    from qldpcsim_amd import decoders
    osdpol(device_min=int(device_min))
    n_osd = fallback = 0
    for c, a in golden_cases("_osd50"):
        H = half_matrix(c)
        syn = torch.as_tensor(a["syn"], device="cuda")
        r = decoders.decode_batch(H, syn, c["p_phys"] / 3, c["max_iter"], algo="MS", want_post=True,
                                  layer_ptr=a["layer_ptr"], layer_rows=a["layer_rows"])
        decoders.apply_osd_device(H, syn, r, order)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(r.iters.cpu().numpy(), a["iters"])
        np.testing.assert_array_equal(r.post.cpu().numpy().view(np.uint64), a["post"].view(np.uint64))
        conv = a["conv"] != 0
        np.testing.assert_array_equal(((r.flags.cpu().numpy() & 1) != 0), conv)
        want = np.where(conv[:, None], a["ehat"], a[f"ehat_osd{order}"])
        np.testing.assert_array_equal(r.ehat.cpu().numpy(), want)
        n_osd += int((~conv).sum())
        fallback += getattr(r, "osd_host_order", 0)
    assert n_osd >= 64, n_osd
    if device_min == "1":
        assert fallback == 0, (fallback, n_osd)            # the device order is NumPy's


def test_gpu_osd_large_code_runs_on_device():
    """A 3000 x 6000 H (past the register / LDS OSD kernels, which refused it
    before this round) runs on the device (osd_hbm_kernel) and equals the
    host C++ OSD shot for shot."""
    import torch
    from qldpcsim_amd import _lib, decoders
    rng = np.random.default_rng(8)
    m, n = 3000, 6000
    H = np.zeros((m, n), np.uint8)
    H[rng.integers(0, m, 6 * n), np.repeat(np.arange(n), 6)] = 1
    code = _lib.code_for(H, 0)
    k = 4
    err = (rng.random((k, n)) < 0.02).astype(np.int64)
    syn = ((err @ H.T.astype(np.int64)) % 2).astype(np.uint8)
    post = rng.normal(0, 3, (k, n))
    e0 = (post < 0).astype(np.uint8)
    d = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dt), device="cuda")  # noqa: E731
    s_d, e_d = d(syn, np.uint8), d(e0, np.uint8)
    st = torch.empty(k, dtype=torch.int32, device="cuda")
    perm = d(decoders.osd_perms(post), np.int32)
    _lib.check(_lib.lib.qldpc_osd_device(code.handle, k, s_d.data_ptr(), perm.data_ptr(), 0, e_d.data_ptr(),
                                         st.data_ptr(), None))
    torch.cuda.synchronize()
    want, rc = _host_osd(H, syn, e0, post, 0)
    assert rc == 0 and np.all(st.cpu().numpy() == 0)
    np.testing.assert_array_equal(e_d.cpu().numpy(), want)


def _host_osd(H, syn, e0, post, order):
    from qldpcsim_amd import _lib, decoders
    want = np.ascontiguousarray(e0, np.uint8).copy()
    perms = np.ascontiguousarray(decoders.osd_perms(post), np.int32)
    code_h = _lib.code_for(H)
    rc = _lib.lib.qldpc_osd_decode_batch(code_h.handle, len(e0), _lib.ptr(np.ascontiguousarray(syn, np.uint8)),
                                         _lib.ptr(perms), order, _lib.ptr(want), 0)
    return want, rc


def _random_sparse_code(m, n, row_w, seed):
    rng = np.random.default_rng(seed)
    H = np.zeros((m, n), np.uint8)
    for r in range(m):
        H[r, rng.choice(n, row_w, replace=False)] = 1
    return H


@pytest.mark.parametrize("code", ["steane", "LP04_0", "LP118_2", "bicycle"])
def test_hbm_osd_kernel_matches_default_and_host(code, qopt):
    """osd_hbm_kernel (forced with option osd_hbm on codes the register / LDS
    kernels also take): the same estimates and statuses as the default device
    path and the host C++ OSD, orders 0, 1 and 2, consistent and random
    syndromes."""
    from qldpcsim_amd import codes
    Hx, _ = codes.load_code(code)
    rng = np.random.default_rng(21)
    k = 64
    syn = rng.integers(0, 2, (k, Hx.shape[0])).astype(np.uint8)
    err = (rng.random((k // 2, Hx.shape[1])) < 0.06).astype(np.int64)
    syn[: k // 2] = (err @ Hx.T.astype(np.int64)) % 2
    post = rng.normal(0, 3, (k, Hx.shape[1]))
    e0 = (post < 0).astype(np.uint8)
    for order in (0, 1, 2):
        dflt, sd = _gpu_osd(Hx, syn, e0, post, order)
        qopt(osd_hbm=1)
        hbm, sh = _gpu_osd(Hx, syn, e0, post, order)
        qopt(osd_hbm=0)
        np.testing.assert_array_equal(sh, sd)
        np.testing.assert_array_equal(hbm, dflt)
        ok = sd == 0
        want, _ = _host_osd(Hx[:, :], syn[ok], e0[ok], post[ok], order)
        np.testing.assert_array_equal(hbm[ok], want)


@pytest.mark.parametrize("m,n", [(1100, 2300), (600, 2400), (1200, 1500)])
def test_hbm_osd_codes_past_the_register_kernels(m, n):
    """Codes past the register / LDS OSD kernels (m > 1024 rows or n > 2111
    columns; before, m > 1024 was refused and n > 2111 selected a kernel too
    narrow for the row): the device OSD equals the host C++ OSD shot for
    shot, orders 0 and 1, consistent syndromes and random ones (status 1 where
    the reference raises IndexError). The random codes have all-zero columns
    (~13 % at 600 x 2400): with one first in the order and rank(H) = m, J
    holds m + 1 entries — the reference's assignment fails to broadcast, the
    host and device OSD both write 0 at the extra entry."""
    H = _random_sparse_code(m, n, 8, m + n)
    rng = np.random.default_rng(m * 7 + n)
    k = 24
    syn = rng.integers(0, 2, (k, m)).astype(np.uint8)
    err = (rng.random((k // 2, n)) < 0.03).astype(np.int64)
    syn[: k // 2] = (err @ H.T.astype(np.int64)) % 2
    post = rng.normal(0, 3, (k, n))
    e0 = (post < 0).astype(np.uint8)
    for order in (0, 1):
        got, st = _gpu_osd(H, syn, e0, post, order)
        assert np.all(st[: k // 2] == 0), st
        for i in range(k):
            want, rc = _host_osd(H, syn[i:i + 1], e0[i:i + 1], post[i:i + 1], order)
            if st[i] == 0:
                assert rc == 0
                np.testing.assert_array_equal(got[i], want[0], err_msg=f"shot {i} order {order}")
            else:
                assert st[i] == 1 and rc != 0                      # both: the reference's IndexError
                np.testing.assert_array_equal(got[i], e0[i])      # e_hat left unchanged


@pytest.mark.parametrize("m,n", [(1100, 1800), (700, 2300)])
def test_apply_osd_device_on_codes_past_the_register_kernels(m, n, osdpol):
    """The pipeline's own entry (apply_osd_device: device order where n <=
    2048, NumPy's order on the host past it, then the device elimination) on
    codes past the register / LDS OSD kernels equals the host OSD."""
    import torch
    from qldpcsim_amd import decoders
    H = _random_sparse_code(m, n, 8, 3 * m + n)
    rng = np.random.default_rng(m + 5 * n)
    k = 16
    err = (rng.random((k, n)) < 0.03).astype(np.int64)
    syn = ((err @ H.T.astype(np.int64)) % 2).astype(np.uint8)
    post = rng.normal(0, 3, (k, n))
    e0 = (post < 0).astype(np.uint8)
    want, rc = _host_osd(H, syn, e0, post, 0)
    assert rc == 0
    osdpol(device_min=1)
    d = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dt), device="cuda")  # noqa: E731
    res = decoders.DecodeResult(d(e0, np.uint8), torch.zeros(k, dtype=torch.int32, device="cuda"),
                                d(post, np.float64), torch.zeros(k, dtype=torch.int32, device="cuda"))
    decoders.apply_osd_device(H, d(syn, np.uint8), res, 0)
    np.testing.assert_array_equal(res.ehat.cpu().numpy(), want)
