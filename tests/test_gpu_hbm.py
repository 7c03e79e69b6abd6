"""The HBM-resident decoder (hbm_kernels.hip): codes the LDS-resident kernels
cannot hold (per-half-shot state beyond a CU's LDS, tables past 16 bits)
decode through it automatically, and it equals the oracle bit for bit —
the reference's arithmetic (decoders.py:110-182, :189-290) at any size.
The library option force_hbm routes the bundled codes through it too, so it is also
pinned against the reference's golden vectors."""
import numpy as np
import pytest

from conftest import golden_cases, half_matrix

pytestmark = pytest.mark.gpu


def _regular_code(n, dv, dc, seed):
    """Random (dv, dc)-regular parity-check matrix (socket permutation; repeated
    sockets on one row are dropped, so a few rows / columns fall short)."""
    rng = np.random.default_rng(seed)
    m = n * dv // dc
    sockets = np.repeat(np.arange(n), dv)
    rows = rng.permutation(np.repeat(np.arange(m), dc))
    H = np.zeros((m, n), np.uint8)
    H[rows, sockets] = 1
    return H


def _syndromes(H, B, p, seed):
    rng = np.random.default_rng(seed)
    e = (rng.random((B, H.shape[1])) < p).astype(np.int64)
    return ((e @ H.T.astype(np.int64)) % 2).astype(np.uint8)


def _check(H, syn, algo, prior, max_iter, lp=None, lr=None, bits=False):
    import torch
    from oracle import oracle
    from qldpcsim_amd import decoders
    s = torch.as_tensor(syn, device="cuda")
    if bits:
        s = decoders.pack_bits(s)
    r = decoders.decode_batch(H, s, prior, max_iter, algo=algo, want_post=True, layer_ptr=lp, layer_rows=lr,
                              ehat_bits=bits)
    torch.cuda.synchronize()
    e, it, post, fl = oracle.decode_batch(algo, H, syn, prior, max_iter, lp, lr)
    got_e = decoders.unpack_bits(r.ehat, H.shape[1]) if bits else r.ehat
    np.testing.assert_array_equal(r.iters.cpu().numpy(), it)
    np.testing.assert_array_equal(got_e.cpu().numpy(), e)
    np.testing.assert_array_equal(r.post.cpu().numpy().view(np.uint64), post.view(np.uint64))
    if algo == "MS":                                   # the zero-message leak case, flagged alike
        np.testing.assert_array_equal((r.flags.cpu().numpy() & 2) != 0, (fl & 1) != 0)
    return r


@pytest.mark.parametrize("algo,sched", [("MS", "F"), ("MS", "L"), ("BP", "F"), ("BP", "L")])
def test_large_code_takes_hbm_kernel_and_equals_oracle(algo, sched):
    """n = 12000, (3, 6)-regular: 240 KB of min-sum state per half-shot (LDS
    holds 160 KB), so the decode runs on hbm_decode_kernel; every iteration
    count, hard decision and float64 posterior equals the oracle's, on
    converging and non-converging syndromes, flooding and layered."""
    from qldpcsim_amd import _lib, schedule
    H = _regular_code(12000, 3, 6, 1)
    layers = [np.arange(H.shape[0])] if sched == "F" else schedule.layerize(H)
    lp, lr = schedule.pack_layers(layers, H.shape[0])
    assert _lib.kernel_name(H, lp, lr, algo).startswith("hbm_tile_kernel<")
    syn = np.concatenate([_syndromes(H, 40, 0.03, 2), np.random.default_rng(3).integers(0, 2, (8, H.shape[0]),
                                                                                        dtype=np.uint8)])
    _check(H, syn, algo, 0.03, 12 if algo == "BP" else 25, lp, lr)


def test_code_past_16_bit_tables_decodes():
    """n = 70000 columns and E = 70000 edges (past the LDS kernels' 16-bit
    tables; the reference's load_matrix takes any size): row degree 35,
    bit-packed syndromes and estimates, against the oracle."""
    from qldpcsim_amd import _lib
    rng = np.random.default_rng(4)
    m, n = 2000, 70000
    H = np.zeros((m, n), np.uint8)
    H[rng.permutation(np.repeat(np.arange(m), n // m)), np.arange(n)] = 1
    assert _lib.kernel_name(H, np.array([0, m], np.int32), np.arange(m, dtype=np.int32), "MS") \
        .startswith("hbm_tile_kernel<0, 64, 4>")
    syn = _syndromes(H, 24, 0.002, 5)
    _check(H, syn, "MS", 0.002, 10, bits=True)


@pytest.mark.parametrize("algo", ["MS", "BP"])
def test_forced_hbm_matches_reference_goldens(algo, qopt):
    """Option force_hbm: the bundled codes' golden cases (every schedule,
    the 100-iteration BP set included) through the HBM kernel reproduce the
    reference bit for bit."""
    import torch
    from qldpcsim_amd import _lib, decoders
    qopt(force_hbm=1)
    n = 0
    for c, a in golden_cases():
        if "raises" in c or c["algo"] != algo or c["code"] not in ("LP04_0", "LP118_0", "LP118_2", "steane"):
            continue
        H = half_matrix(c)
        assert _lib.kernel_name(H, a["layer_ptr"], a["layer_rows"], algo).startswith("hbm_tile_kernel<")
        r = decoders.decode_batch(H, torch.as_tensor(a["syn"], device="cuda"), c["p_phys"] / 3, c["max_iter"],
                                  algo=algo, want_post=True, layer_ptr=a["layer_ptr"], layer_rows=a["layer_rows"])
        torch.cuda.synchronize()
        np.testing.assert_array_equal(r.iters.cpu().numpy(), a["iters"], err_msg=str(c))
        np.testing.assert_array_equal(r.post.cpu().numpy().view(np.uint64), a["post"].view(np.uint64))
        if c["osd"] < 0:
            np.testing.assert_array_equal(r.ehat.cpu().numpy(), a["ehat"])
        n += len(a["iters"])
    assert n > 300


def test_forced_hbm_early_stopping_batch_equals_lds_kernels(qopt):
    """Lane recycling over a large batch of decodes of very different lengths
    (p = 0.04 channel + fixed-work syndromes, LP118_0 layered MS): the HBM
    kernel equals the default LDS kernel on every half-shot."""
    import torch
    from qldpcsim_amd import _lib, codes, decoders, schedule
    Hx, Hz = codes.load_code("LP118_0")
    lx, _ = schedule.select_layers(Hx, Hz, "L")
    lp, lr = schedule.pack_layers(lx, Hz.shape[0])
    syn = np.concatenate([_syndromes(Hz, 30000, 0.027, 8),
                          np.random.default_rng(9).integers(0, 2, (3000, Hz.shape[0]), dtype=np.uint8)])
    syn = syn[np.random.default_rng(1).permutation(len(syn))]
    s = torch.as_tensor(syn, device="cuda")
    ref = decoders.decode_batch(Hz, s, 0.04 / 3, 40, algo="MS", want_post=True, layer_ptr=lp, layer_rows=lr)
    qopt(force_hbm=1)
    assert _lib.kernel_name(Hz, lp, lr, "MS") == "hbm_tile_kernel<0, 8, 4>"
    got = decoders.decode_batch(Hz, s, 0.04 / 3, 40, algo="MS", want_post=True, layer_ptr=lp, layer_rows=lr)
    torch.cuda.synchronize()
    assert torch.equal(got.iters, ref.iters) and torch.equal(got.ehat, ref.ehat)
    assert torch.equal(got.flags, ref.flags)
    assert torch.equal(got.post.view(torch.int64), ref.post.view(torch.int64))
    assert 1.0 < ref.iters.float().mean().item() < 20.0


@pytest.mark.parametrize("B", [1, 63, 65, 1000])
def test_forced_hbm_ragged_batches_and_edge_cases(B, qopt):
    """Batches that do not fill a 64-slot tile (1, 63, 65, 1000 half-shots),
    all-zero syndromes (converged after the first iteration), max_iter = 1,
    bit-packed I/O: the HBM kernel equals the LDS kernels on every output."""
    import torch
    from qldpcsim_amd import codes, decoders, schedule
    Hx, Hz = codes.load_code("LP04_0")
    rng = np.random.default_rng(B)
    syn = rng.integers(0, 2, (B, Hz.shape[0]), dtype=np.uint8)
    syn[::3] = 0
    for sched in ("F", "L"):
        lx, _ = schedule.select_layers(Hx, Hz, sched)
        lp, lr = schedule.pack_layers(lx, Hz.shape[0])
        for algo, it in (("MS", 1), ("MS", 30), ("BP", 1), ("BP", 12)):
            s = decoders.pack_bits(torch.as_tensor(syn, device="cuda"))
            qopt(force_hbm=0)
            ref = decoders.decode_batch(Hz, s, 0.03, it, algo=algo, want_post=True, layer_ptr=lp,
                                        layer_rows=lr, ehat_bits=True)
            qopt(force_hbm=1)
            got = decoders.decode_batch(Hz, s, 0.03, it, algo=algo, want_post=True, layer_ptr=lp,
                                        layer_rows=lr, ehat_bits=True)
            torch.cuda.synchronize()
            assert torch.equal(got.iters, ref.iters) and torch.equal(got.ehat, ref.ehat), (sched, algo, it)
            assert torch.equal(got.flags, ref.flags)
            assert torch.equal(got.post.view(torch.int64), ref.post.view(torch.int64))
            assert (got.iters[::3] == 1).all()                    # zero syndromes: converged at once


@pytest.mark.parametrize("algo", ["MS", "BP"])
def test_forced_hbm_non_partition_schedule(algo, qopt):
    """A schedule that is not a partition of the rows (row 5 in two layers,
    row 10 in none): the HBM kernel's state-initialising path (hbm_lazy = 0:
    no first-layer tables) against the oracle and against the LDS kernels,
    max_iter 1 and 20, 200 half-shots (64-slot tiles recycled)."""
    import torch
    from qldpcsim_amd import _lib, codes, decoders, schedule
    Hx, Hz = codes.load_code("LP04_0")
    layers = [np.asarray(l) for l in schedule.layerize(Hx)]
    layers[-1] = np.append(layers[-1], 5)                   # row 5 again in the last layer
    layers = [l[l != 10] for l in layers]                   # row 10 in no layer
    assert any(5 in l for l in layers[:-1]) and not any(10 in l for l in layers)
    lp, lr = schedule.pack_layers(layers, Hz.shape[0])
    syn = np.concatenate([_syndromes(Hz, 150, 0.05, 21),
                          np.random.default_rng(22).integers(0, 2, (50, Hz.shape[0]), dtype=np.uint8)])
    for it in (1, 20):
        qopt(force_hbm=0)
        ref = decoders.decode_batch(Hz, torch.as_tensor(syn, device="cuda"), 0.05 / 3, it, algo=algo,
                                    want_post=True, layer_ptr=lp, layer_rows=lr)
        qopt(force_hbm=1)
        assert _lib.kernel_name(Hz, lp, lr, algo).startswith("hbm_tile_kernel<")
        got = _check(Hz, syn, algo, 0.05 / 3, it, lp, lr)
        assert torch.equal(got.iters, ref.iters) and torch.equal(got.ehat, ref.ehat)
        assert torch.equal(got.post.view(torch.int64), ref.post.view(torch.int64))


@pytest.mark.parametrize("algo,sched", [("MS", "F"), ("MS", "L"), ("BP", "F"), ("BP", "L")])
def test_rows_wider_than_64_edges_decode(algo, sched, qopt):
    """Row degree 100 (the reference's decoders take any H): the HBM kernel's
    two-pass check node for rows past its 64-edge registers (the default for
    MS, whose LDS kernels take rows up to 32 edges; forced for BP, whose
    generic LDS kernel takes any row degree and is checked too), against the
    oracle bit for bit on converging and fixed-work syndromes, 80 half-shots
    (64-slot tiles recycled)."""
    from qldpcsim_amd import _lib, schedule
    H = _regular_code(1200, 5, 100, 7)
    assert H.sum(axis=1).max() > 64
    layers = [np.arange(H.shape[0])] if sched == "F" else schedule.layerize(H)
    lp, lr = schedule.pack_layers(layers, H.shape[0])
    syn = np.concatenate([_syndromes(H, 60, 0.004, 3), np.random.default_rng(4).integers(0, 2, (20, H.shape[0]),
                                                                                         dtype=np.uint8)])
    it = 8 if algo == "BP" else 15
    _check(H, syn, algo, 0.004, it, lp, lr)                 # the default kernel
    qopt(force_hbm=1)
    assert _lib.kernel_name(H, lp, lr, algo) == f"hbm_tile_kernel<{0 if algo == 'MS' else 1}, 64, 4>"
    _check(H, syn, algo, 0.004, it, lp, lr)
