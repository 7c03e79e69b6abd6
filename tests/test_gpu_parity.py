"""GPU parity: the HIP kernels (through the C ABI) against the reference's golden
vectors and the pinned CPU oracle on identical syndromes.

Bar: MS and BP — hard decisions, iteration counts
and float64 posteriors bit-exact against the reference's golden vectors and
the CPU oracle. (BP's tanh / atanh and both decoders' log prior are NumPy's
own, restated in include/qldpc_libm.h; the north-star 1e-5 tolerance is not
needed.)
"""
import numpy as np
import pytest

from conftest import golden_cases, half_matrix

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def dec():
    from qldpcsim_amd import _lib, decoders
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return decoders


CASES = [(c, a) for c, a in golden_cases() if "raises" not in c and c["osd"] < 0 and c["max_iter"] < 100]
BP100 = [(c, a) for c, a in golden_cases("_it100")]    # full-length BP: see test_oracle_golden.py
OSD_CASES = [(c, a) for c, a in golden_cases("_osd") if c["osd"] >= 0]
RAISE_CASES = [(c, a) for c, a in golden_cases() if c.get("raises") == "IndexError"]


def _id(ca):
    c = ca[0]
    return f"{c['algo']}-{c['code']}-{c['half']}-{c['sched']}-{c['kind']}-p{c['p_phys']}-it{c['max_iter']}"


def _assert_post(algo, got, want):
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("ca", CASES, ids=[_id(x) for x in CASES])
def test_kernel_matches_reference_golden(dec, ca):
    c, a = ca
    H = half_matrix(c)
    r = dec.decode_batch(H, a["syn"], c["p_phys"] / 3, c["max_iter"], algo=c["algo"],
                         want_post=True, layer_ptr=a["layer_ptr"], layer_rows=a["layer_rows"])
    np.testing.assert_array_equal(r.iters, a["iters"])
    np.testing.assert_array_equal(r.ehat, a["ehat"])
    _assert_post(c["algo"], r.post, a["post"])
    assert not np.any(r.flags & 2), "min-sum zero-message leak case hit"


@pytest.mark.parametrize("ca", BP100, ids=[_id(x) + f"-{x[0]['id']}" for x in BP100])
def test_bp100_kernel_equals_reference_and_oracle(dec, ca):
    """100-iteration BP (configs[2] / [4]): the GPU equals the reference's
    golden vectors and the CPU oracle bit for bit on every shot, chaotic
    long and non-converging decodes included."""
    from oracle import oracle
    c, a = ca
    H = half_matrix(c)
    r = dec.decode_batch(H, a["syn"], c["p_phys"] / 3, c["max_iter"], algo=c["algo"],
                         want_post=True, layer_ptr=a["layer_ptr"], layer_rows=a["layer_rows"])
    e, it, post, _ = oracle.decode_batch(c["algo"], H, a["syn"], c["p_phys"] / 3, c["max_iter"],
                                         a["layer_ptr"], a["layer_rows"])
    np.testing.assert_array_equal(r.iters, it)
    np.testing.assert_array_equal(r.ehat, e)
    np.testing.assert_array_equal(r.post.view(np.uint64), post.view(np.uint64))
    np.testing.assert_array_equal(r.iters, a["iters"])
    np.testing.assert_array_equal(r.ehat, a["ehat"])
    np.testing.assert_array_equal(r.post.view(np.uint64), a["post"].view(np.uint64))


HEADLINE = golden_cases("_headline")


@pytest.mark.parametrize("ca", HEADLINE, ids=[f"{c['half']}-{c['id']}" for c, _ in HEADLINE])
def test_headline_golden_on_the_bench_path(dec, ca):
    """The exact headline workload from the reference (LP118_0 MS flooding,
    50 iterations, uniform random syndromes; tests/golden/
    ms_LP118_0_headline.npz) through the bench's path: device-resident
    bit-packed syndromes, bit-packed estimates, ms_flood_kernel: iterations,
    hard decisions and posteriors bit-exact."""
    import torch
    from qldpcsim_amd import _lib
    c, a = ca
    H = half_matrix(c)
    assert _lib.kernel_name(H, a["layer_ptr"], a["layer_rows"], "MS", 0).startswith("ms_flood_kernel<8")
    syn = dec.pack_bits(torch.as_tensor(a["syn"], device="cuda"))
    r = dec.decode_batch(H, syn, c["p_phys"] / 3, c["max_iter"], algo="MS", want_post=True,
                         layer_ptr=a["layer_ptr"], layer_rows=a["layer_rows"], ehat_bits=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r.iters.cpu().numpy(), a["iters"])
    np.testing.assert_array_equal(dec.unpack_bits(r.ehat, H.shape[1]).cpu().numpy(), a["ehat"])
    np.testing.assert_array_equal(r.post.cpu().numpy().view(np.uint64), a["post"].view(np.uint64))
    assert np.all(a["iters"] == 50)


@pytest.mark.parametrize("ca", OSD_CASES, ids=[_id(x) + f"-osd{x[0]['osd']}" for x in OSD_CASES])
def test_dropin_shims_with_osd_match_reference(dec, ca):
    c, a = ca
    H = half_matrix(c)
    fn = dec.MS_decoder if c["algo"] == "MS" else dec.BP_decoder
    for k in range(a["syn"].shape[0]):
        lp, lr = a["layer_ptr"], a["layer_rows"]
        layers = [lr[lp[i]:lp[i + 1]] for i in range(len(lp) - 1)]
        e, it = fn(H, a["syn"][k].astype(int), c["p_phys"] / 3, max_iter=c["max_iter"],
                   layers=layers, OSDorder=c["osd"])
        assert it == a["iters"][k]
        np.testing.assert_array_equal(e.astype(np.uint8), a["ehat"][k])
        assert e.dtype == (np.int8 if c["algo"] == "MS" else np.int64)


@pytest.mark.parametrize("ca", RAISE_CASES[:4], ids=[_id(x) for x in RAISE_CASES[:4]])
def test_out_of_range_layers_raise_indexerror(dec, ca):
    c, _ = ca
    from qldpcsim_amd import codes, schedule
    Hx, Hz = codes.load_code(c["code"])
    lx, lz = schedule.select_layers(Hx, Hz, c["sched"])
    H, layers = (Hz, lx) if c["half"] == "X" else (Hx, lz)
    with pytest.raises(IndexError):
        dec.MS_decoder(H, np.ones(H.shape[0], int), 0.01, max_iter=2, layers=layers)


# ---------------------------------------------------------------------------
# larger batches against the oracle (same seeded syndromes)
# ---------------------------------------------------------------------------
def _channel(Hx, Hz, p, B, seed):
    rng = np.random.default_rng(seed)
    n = Hx.shape[1]
    u = rng.random((B, n))
    X, Y, Z = u < p / 3, (u >= p / 3) & (u < 2 * p / 3), (u >= 2 * p / 3) & (u < p)
    ex, ez = (X | Y).astype(np.float32), (Z | Y).astype(np.float32)
    sz = (ex @ Hz.T.astype(np.float32)).astype(np.int64) % 2
    sx = (ez @ Hx.T.astype(np.float32)).astype(np.int64) % 2
    return sz.astype(np.uint8), sx.astype(np.uint8)


@pytest.mark.parametrize("code,sched,algo,p,max_iter,B", [
    ("LP118_0", "F", "MS", None, 50, 4096),      # headline config, random (fixed-work) syndromes
    ("LP118_0", "F", "MS", 0.05, 50, 4096),
    ("LP118_2", "L", "MS", 0.05, 50, 2048),
    ("LP04_0", "S", "MS", 0.08, 20, 1024),
    ("LP04_0", "F", "MS", 0.1, 50, 4096),
    ("LP118_0", "F", "BP", 0.05, 100, 512),
    ("LP118_0", "L", "BP", 0.05, 100, 256),
    ("bicycle", "F", "BP", 0.05, 30, 256),
    ("LP118_0", "F", "BP", None, 5, 512),         # short horizon: every posterior within tolerance
    ("LP118_0", "L", "BP", None, 3, 256),
    ("LP118_0", "L", "MS", 0.05, 50, 2048),
    ("LP118_2", "L", "BP", 0.08, 100, 128),       # BP team kernel, 4-wave teams, global row table
    ("LP118_2", "F", "BP", None, 4, 128),
    ("LP04_0", "F", "BP", 0.1, 100, 512),         # BP team kernel, row degree 7
    ("LP118_0", "S", "MS", 0.05, 3, 256),
    ("T", "F", "MS", 0.05, 50, 1024),
    ("LP118_2", "L", "MS", None, 50, 512),        # layered MS, fixed work (50 iterations)
    ("LP118_0", "L", "MS", None, 50, 512),
    ("LP04_0", "L", "MS", 0.08, 50, 1024),        # layered MS, row degree 7
    ("LP118_2", "S", "MS", 0.05, 4, 256),         # serial schedule: 450 one-row layers
    ("LP118_2", "L", "BP", 0.12, 100, 256),       # many failing decodes: saturated check nodes (|v2c/2| >= 19.5)
    ("LP118_2", "F", "BP", 0.12, 60, 128),
])
def test_kernel_matches_oracle_batches(dec, code, sched, algo, p, max_iter, B):
    from oracle import oracle
    from qldpcsim_amd import codes, schedule
    Hx, Hz = codes.load_code(code)
    lx, lz = schedule.select_layers(Hx, Hz, sched)
    prior = (p if p is not None else 0.05) / 3
    if p is None:
        rng = np.random.default_rng(20251226)
        sz = rng.integers(0, 2, (B, Hz.shape[0]), dtype=np.uint8)
        sx = rng.integers(0, 2, (B, Hx.shape[0]), dtype=np.uint8)
    else:
        sz, sx = _channel(Hx, Hz, p, B, 7)
    for H, layers, syn in ((Hz, lx, sz), (Hx, lz, sx)):
        lp, lr = schedule.pack_layers(layers, H.shape[0])
        r = dec.decode_batch(H, syn, prior, max_iter, algo=algo, want_post=True,
                             layer_ptr=lp, layer_rows=lr)
        e, it, post, fl = oracle.decode_batch(algo, H, syn, prior, max_iter, lp, lr)
        # MS and BP: bit-exact against the oracle on every shot (BP shares the
        # reproducible tanh/atanh of include/qldpc_libm.h with the oracle; the
        # oracle itself is pinned to the reference within 2.2e-8 relative).
        np.testing.assert_array_equal(r.iters, it)
        np.testing.assert_array_equal(r.ehat, e)
        np.testing.assert_array_equal(r.post.view(np.uint64), post.view(np.uint64))
        if algo == "MS":   # the zero-message leak case is flagged identically
            np.testing.assert_array_equal((r.flags & 2) != 0, (fl & 1) != 0)
        if p is not None:
            # property: a converged shot satisfies its syndrome
            conv = r.converged
            Hm = H.astype(np.int64)
            assert np.all(((r.ehat[conv].astype(np.int64) @ Hm.T) % 2) == syn[conv])


def test_full_size_headline_batch_properties(dec):
    """BASELINE config at full size (2^20 shots/half would be the bench; here
    2^18): every fixed-work random syndrome runs exactly 50 iterations, never
    converges (rank(H)=232 < m=240 makes them unsatisfiable w.p. >= 255/256,
    SURVEY.md §8d), a seeded sample matches the oracle bit for bit, and the
    decode is deterministic run to run."""
    import torch
    from oracle import oracle
    from qldpcsim_amd import codes
    Hx, Hz = codes.load_code("LP118_0")
    B = 1 << 18
    g = torch.Generator(device="cuda").manual_seed(1)
    syn = torch.randint(0, 2, (B, Hz.shape[0]), dtype=torch.uint8, device="cuda", generator=g)
    r1 = dec.decode_batch(Hz, syn, 0.05 / 3, 50, algo="MS")
    r2 = dec.decode_batch(Hz, syn, 0.05 / 3, 50, algo="MS")
    torch.cuda.synchronize()
    assert torch.equal(r1.ehat, r2.ehat) and torch.equal(r1.iters, r2.iters)
    conv = ((r1.flags & 1) != 0)
    it = r1.iters
    # converged shots must satisfy the syndrome; all others ran max_iter
    assert bool(torch.all(it[~conv] == 50))
    assert conv.float().mean().item() < 0.02
    idx = np.random.default_rng(3).choice(B, 256, replace=False)
    sub = syn[torch.as_tensor(idx, device="cuda")].cpu().numpy()
    e, its, _, _ = oracle.decode_batch("MS", Hz, sub, 0.05 / 3, 50, want_post=False)
    np.testing.assert_array_equal(r1.ehat[torch.as_tensor(idx, device="cuda")].cpu().numpy(), e)
    np.testing.assert_array_equal(it[torch.as_tensor(idx, device="cuda")].cpu().numpy(), its)


def test_decode_batch_into_preallocated_buffers(dec):
    """decode_batch(out=...) writes the same results into caller buffers (the
    bench's allocation-free steady state) and rejects mismatched buffers."""
    import torch
    from qldpcsim_amd import codes
    Hx, Hz = codes.load_code("LP118_0")
    B, n = 2048, Hz.shape[1]
    g = torch.Generator(device="cuda").manual_seed(5)
    syn = torch.randint(0, 2, (B, Hz.shape[0]), dtype=torch.uint8, device="cuda", generator=g)
    ref = dec.decode_batch(Hz, syn, 0.05 / 3, 50, algo="MS", want_post=True)
    out = dec.DecodeResult(torch.full((B, n), 7, dtype=torch.uint8, device="cuda"),
                           torch.full((B,), -1, dtype=torch.int32, device="cuda"),
                           torch.zeros((B, n), dtype=torch.float64, device="cuda"),
                           torch.full((B,), -1, dtype=torch.int32, device="cuda"))
    r = dec.decode_batch(Hz, syn, 0.05 / 3, 50, algo="MS", want_post=True, out=out)
    torch.cuda.synchronize()
    assert r.ehat.data_ptr() == out.ehat.data_ptr()
    assert torch.equal(r.ehat, ref.ehat) and torch.equal(r.iters, ref.iters)
    assert torch.equal(r.flags, ref.flags) and torch.equal(r.post, ref.post)
    bad = dec.DecodeResult(out.ehat[:, :-1], out.iters, None, out.flags)
    with pytest.raises(ValueError):
        dec.decode_batch(Hz, syn, 0.05 / 3, 50, algo="MS", out=bad)



KERNELS = ["G1", "G2", "G4", "G8", "generic", "default"]


@pytest.mark.parametrize("code", ["LP118_2", "LP118_0", "LP04_0"])
@pytest.mark.parametrize("kernel", KERNELS)
def test_ms_layered_kernels_match_oracle(dec, kernel, code, qopt):
    """Every layered MS kernel shape against the oracle, bit for bit, with
    fixed-work and channel syndromes mixed in one batch: ms_layered_kernel at
    every lanes-per-check width G (option ms_lanes_per_check), the default
    per-layer choice, and the generic decode kernel (option layered_generic).
    Lane mappings never change the arithmetic."""
    from oracle import oracle
    from qldpcsim_amd import _lib, codes, schedule
    Hx, Hz = codes.load_code(code)
    if kernel == "generic":
        qopt(layered_generic=1)
    elif kernel.startswith("G"):
        qopt(ms_lanes_per_check=int(kernel[1:]))
    lx, _ = schedule.select_layers(Hx, Hz, "L")
    lp, lr = schedule.pack_layers(lx, Hz.shape[0])
    rng = np.random.default_rng(11)
    syn = np.concatenate([rng.integers(0, 2, (128, Hz.shape[0]), dtype=np.uint8),
                          _channel(Hx, Hz, 0.06, 256, 5)[0]])
    syn = syn[rng.permutation(len(syn))]
    code_h = _lib.code_for(Hz)
    code_h._sched.clear()                  # launch configs read the env once per schedule
    try:
        r = dec.decode_batch(Hz, syn, 0.06 / 3, 30, algo="MS", want_post=True, layer_ptr=lp, layer_rows=lr)
        if kernel.startswith("G"):
            nm = _lib.kernel_name(Hz, lp, lr, "MS")
            assert nm == f"ms_layered_kernel<{Hz.sum(1).max()}, {kernel[1:]}>", nm
    finally:
        code_h._sched.clear()
    e, it, post, fl = oracle.decode_batch("MS", Hz, syn, 0.06 / 3, 30, lp, lr)
    np.testing.assert_array_equal(r.iters, it)
    np.testing.assert_array_equal(r.ehat, e)
    np.testing.assert_array_equal(r.post.view(np.uint64), post.view(np.uint64))
    np.testing.assert_array_equal((r.flags & 2) != 0, (fl & 1) != 0)


@pytest.mark.parametrize("nlayers", [2, 3, 5])
def test_ms_layered_g1_multi_trip_layers(dec, nlayers, qopt):
    """The one-lane-per-check instance on layers of more than 64 rows (several
    check-node trips per layer, row words from the global table, round 5):
    LP118_2's rows cut into 2-5 contiguous layers of 90-225 rows (one layer of
    every row is flooding and takes the flooding kernel), bit-exact vs the
    oracle."""
    from oracle import oracle
    from qldpcsim_amd import _lib, codes, schedule
    Hx, Hz = codes.load_code("LP118_2")
    m = Hz.shape[0]
    cuts = np.linspace(0, m, nlayers + 1).astype(int)
    layers = [np.arange(cuts[i], cuts[i + 1]) for i in range(nlayers)]
    lp, lr = schedule.pack_layers(layers, m)
    qopt(ms_lanes_per_check=1)
    rng = np.random.default_rng(17)
    syn = np.concatenate([rng.integers(0, 2, (64, m), dtype=np.uint8),
                          _channel(Hx, Hz, 0.05, 192, 9)[0]])
    code_h = _lib.code_for(Hz)
    code_h._sched.clear()
    try:
        r = dec.decode_batch(Hz, syn, 0.05 / 3, 25, algo="MS", want_post=True, layer_ptr=lp, layer_rows=lr)
        nm = _lib.kernel_name(Hz, lp, lr, "MS")
        assert nm == "ms_layered_kernel<8, 1>", nm
    finally:
        code_h._sched.clear()
    e, it, post, fl = oracle.decode_batch("MS", Hz, syn, 0.05 / 3, 25, lp, lr)
    np.testing.assert_array_equal(r.iters, it)
    np.testing.assert_array_equal(r.ehat, e)
    np.testing.assert_array_equal(r.post.view(np.uint64), post.view(np.uint64))


def test_ms_layered_large_mixed_batch(dec):
    """The default layered kernel over a batch large enough that the work
    queue hands out multi-half-shot chunks, with decodes of very different
    lengths: bit-exact vs the oracle."""
    from oracle import oracle
    from qldpcsim_amd import _lib, codes, schedule
    Hx, Hz = codes.load_code("LP118_0")
    _, lz = schedule.select_layers(Hx, Hz, "L")
    lp, lr = schedule.pack_layers(lz, Hx.shape[0])
    rng = np.random.default_rng(3)
    syn = np.concatenate([rng.integers(0, 2, (3000, Hx.shape[0]), dtype=np.uint8),
                          _channel(Hx, Hz, 0.04, 30000, 8)[1]])
    syn = syn[rng.permutation(len(syn))]
    nm = _lib.kernel_name(Hx, lp, lr, "MS")
    assert nm.startswith("ms_layered_kernel<8, 0>"), nm
    r = dec.decode_batch(Hx, syn, 0.04 / 3, 40, algo="MS", want_post=True, layer_ptr=lp, layer_rows=lr)
    e, it, post, fl = oracle.decode_batch("MS", Hx, syn, 0.04 / 3, 40, lp, lr)
    np.testing.assert_array_equal(r.iters, it)
    np.testing.assert_array_equal(r.ehat, e)
    np.testing.assert_array_equal(r.post.view(np.uint64), post.view(np.uint64))


@pytest.mark.parametrize("sched", ["L", "S"])
def test_ms_layered_irregular_columns_match_oracle(dec, sched):
    """Layered / serial MS on a synthetic uniform-row-degree-8 code whose
    column degrees run from 1 to ~20 (bundled codes only have 3-5): exercises
    the layered kernel's generic VN branch (degree bounds outside 3-6), layers
    whose adjacency is not a multiple of 64, and heavy parity toggling."""
    from oracle import oracle
    from qldpcsim_amd import schedule
    rng = np.random.default_rng(21)
    m, n = 96, 200
    H = np.zeros((m, n), np.uint8)
    w = np.ones(n)
    w[:4] = 6.0                                    # a few heavy columns (degree <= 31: fast tables)
    for r in range(m):
        H[r, rng.choice(n, 8, replace=False, p=w / w.sum())] = 1
    H = H[:, H.sum(0) > 0]
    assert H.sum(0).max() >= 9 and H.sum(0).min() <= 2
    layers = schedule.layerize(H) if sched == "L" else [np.array([r]) for r in range(H.shape[0])]
    lp, lr = schedule.pack_layers(layers, H.shape[0])
    syn = np.concatenate([rng.integers(0, 2, (256, H.shape[0]), dtype=np.uint8),
                          ((rng.random((256, H.shape[1])) < 0.03).astype(np.int64) @ H.T.astype(np.int64) % 2)
                          .astype(np.uint8)])
    r = dec.decode_batch(H, syn, 0.05 / 3, 25, algo="MS", want_post=True, layer_ptr=lp, layer_rows=lr)
    e, it, post, fl = oracle.decode_batch("MS", H, syn, 0.05 / 3, 25, lp, lr)
    np.testing.assert_array_equal(r.iters, it)
    np.testing.assert_array_equal(r.ehat, e)
    np.testing.assert_array_equal(r.post.view(np.uint64), post.view(np.uint64))


@pytest.mark.parametrize("code,w,lg", [("LP118_2", "4", "1"), ("LP04_0", "8", "1"), ("LP118_0", "4", "1"),
                                        ("LP118_2", "4", "0"), ("LP118_2", "8", "0"), ("LP04_0", "4", "0"),
                                        ("LP118_0", "8", "0")])
def test_bp_team_layered_kernels_match_oracle(dec, code, w, lg, qopt):
    """Layered BP teams: bp_team_lg_kernel (every graph table in global
    memory, the default) and the all-LDS bp_team_kernel<true, ..> (the
    fallback for schedules without the global image, forced by
    option bp_lg = 0) at both team widths: bit-exact vs the oracle on channel and
    fixed-work syndromes."""
    from oracle import oracle
    from qldpcsim_amd import _lib, codes, schedule
    qopt(bp_lg=int(lg), bp_team_w=int(w))
    Hx, Hz = codes.load_code(code)
    lx, _ = schedule.select_layers(Hx, Hz, "L")
    lp, lr = schedule.pack_layers(lx, Hz.shape[0])
    rng = np.random.default_rng(17)
    syn = np.concatenate([rng.integers(0, 2, (32, Hz.shape[0]), dtype=np.uint8),
                          _channel(Hx, Hz, 0.08, 160, 9)[0]])
    code_h = _lib.code_for(Hz)
    code_h._sched.clear()                  # launch configs read the env once per schedule
    try:
        nm = _lib.kernel_name(Hz, lp, lr, "BP")
        if lg == "1":
            assert nm.startswith("bp_team_lg_kernel<") and nm.endswith(f", {w}>"), nm
        else:
            assert nm.startswith("bp_team_kernel<true") and nm.endswith(f", {w}>"), nm
        r = dec.decode_batch(Hz, syn, 0.08 / 3, 40, algo="BP", want_post=True, layer_ptr=lp, layer_rows=lr)
    finally:
        code_h._sched.clear()
    e, it, post, _ = oracle.decode_batch("BP", Hz, syn, 0.08 / 3, 40, lp, lr)
    np.testing.assert_array_equal(r.iters, it)
    np.testing.assert_array_equal(r.ehat, e)
    np.testing.assert_array_equal(r.post.view(np.uint64), post.view(np.uint64))


@pytest.mark.parametrize("sched", ["F", "L"])
@pytest.mark.parametrize("case", ["L0", "eps0"])
def test_bp_nonfinite_paths_match_oracle(dec, sched, case):
    """BP's rare arithmetic against the oracle, through the team kernels'
    wave-uniform slow paths: p = 0.5 (L = 0: every first v2c is 0, tanh 0,
    P / t = 0 / 0 = NaN, atanh(NaN)) and eps = 0 at p = 1e-20 (L = 46: tanh
    rounds to +-1, th2 = +-1 unclipped, atanh = +-inf, then inf - inf).
    Posteriors compare NaN-aware (NaN payloads are the platform's); every
    shot the oracle flags (tanh = 0) is flagged non-finite on the GPU."""
    from oracle import oracle
    from qldpcsim_amd import _lib, codes, schedule
    Hx, Hz = codes.load_code("LP118_0")
    lp = lr = None
    if sched == "L":
        lx, _ = schedule.select_layers(Hx, Hz, "L")
        lp, lr = schedule.pack_layers(lx, Hz.shape[0])
    rng = np.random.default_rng(5)
    syn = np.concatenate([rng.integers(0, 2, (96, Hz.shape[0]), dtype=np.uint8),
                          _channel(Hx, Hz, 0.05, 96, 3)[0]])
    p, eps = (0.5, 1e-9) if case == "L0" else (1e-20, 0.0)
    r = dec.decode_batch(Hz, syn, p, 12, algo="BP", eps=eps, want_post=True, layer_ptr=lp, layer_rows=lr)
    e, it, post, fl = oracle.decode_batch("BP", Hz, syn, p, 12, lp, lr, eps=eps)
    assert not np.isfinite(post).all()                 # the rare paths ran
    np.testing.assert_array_equal(r.iters, it)
    np.testing.assert_array_equal(r.ehat, e)
    np.testing.assert_array_equal(r.post, post)        # NaN == NaN here
    gpu_nf = (r.flags & _lib.FLAG_NONFINITE) != 0
    assert gpu_nf[(fl & 2) != 0].all()
