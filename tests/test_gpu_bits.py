"""Bit-packed wire format (QLDPC_FMT_BITS): syndromes and hard
decisions as 64-bit words (bit j % 64 of word j / 64) give exactly the
byte-format results in every decode kernel, in the device sampler and in the
outcome counters."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KERNEL_ENVS = {"fast": {}, "generic": {"flood_generic": 1, "layered_generic": 1}}   # library options


@pytest.mark.parametrize("env", sorted(KERNEL_ENVS))
@pytest.mark.parametrize("code,algo,sched", [
    ("LP118_0", "MS", "F"), ("LP118_2", "MS", "L"), ("LP04_0", "MS", "S"), ("steane", "MS", "F"),
    ("LP118_0", "BP", "F"), ("LP118_2", "BP", "L"), ("bicycle", "MS", "L"), ("shor", "BP", "F"),
])
def test_bit_packed_decode_equals_bytes(code, algo, sched, env, qopt):
    import torch
    from qldpcsim_amd import _lib, codes, decoders, schedule
    Hx, Hz = codes.load_code(code)
    qopt(**KERNEL_ENVS[env])
    lx, _ = schedule.select_layers(Hx, Hz, sched)
    lp, lr = schedule.pack_layers(lx, Hz.shape[0])
    _lib.code_for(Hz, 0)._sched.clear()
    g = torch.Generator(device="cuda").manual_seed(5)
    e = (torch.rand((3000, Hz.shape[1]), device="cuda", generator=g) < 0.04).to(torch.float32)
    syn = ((e @ torch.as_tensor(Hz.T, dtype=torch.float32, device="cuda")).remainder(2)).to(torch.uint8)
    syn[:500] = torch.randint(0, 2, syn[:500].shape, dtype=torch.uint8, device="cuda", generator=g)
    try:
        ref = decoders.decode_batch(Hz, syn, 0.04, 25, algo=algo, layer_ptr=lp, layer_rows=lr, want_post=True)
        words = decoders.pack_bits(syn)
        for s_in in (syn, words):
            got = decoders.decode_batch(Hz, s_in, 0.04, 25, algo=algo, layer_ptr=lp, layer_rows=lr,
                                        want_post=True, ehat_bits=True)
            assert got.ehat.dtype == torch.int64 and got.ehat.shape == (3000, (Hz.shape[1] + 63) // 64)
            assert torch.equal(decoders.unpack_bits(got.ehat, Hz.shape[1]), ref.ehat)
            assert torch.equal(got.iters, ref.iters) and torch.equal(got.flags, ref.flags)
            assert torch.equal(got.post, ref.post)
            # bits beyond n stay zero
            assert torch.equal(decoders.pack_bits(ref.ehat), got.ehat)
        got_b = decoders.decode_batch(Hz, words, 0.04, 25, algo=algo, layer_ptr=lp, layer_rows=lr)
        assert torch.equal(got_b.ehat, ref.ehat) and torch.equal(got_b.iters, ref.iters)
    finally:
        _lib.code_for(Hz, 0)._sched.clear()


@pytest.mark.parametrize("code", ["LP118_0", "LP04_0", "steane", "LP118_2"])
def test_bit_packed_sampler_and_counters_equal_bytes(code):
    import torch
    from qldpcsim_amd import codes, decoders, simulator
    Hx, Hz = codes.load_code(code)
    dev = torch.device("cuda", 0)
    a = simulator.DeviceChannel(Hx, Hz, dev, 77, shot0=3)
    b = simulator.DeviceChannel(Hx, Hz, dev, 77, shot0=3)
    sz, sx, ex, ez = a.sample(0.08, 4000)
    wz, wx, fx, fz = b.sample(0.08, 4000, bits=True)
    assert torch.equal(ex, fx) and torch.equal(ez, fz)
    assert torch.equal(decoders.pack_bits(sz), wz) and torch.equal(decoders.pack_bits(sx), wx)
    rX = decoders.decode_batch(Hz, sz, 0.08 / 3, 30)
    rZ = decoders.decode_batch(Hx, sx, 0.08 / 3, 30)
    want = a.count(sz, sx, ex, ez, rX.ehat, rZ.ehat, rX.iters, rZ.iters)
    pX, pZ = decoders.pack_bits(rX.ehat), decoders.pack_bits(rZ.ehat)
    assert a.count(wz, wx, ex, ez, pX, pZ, rX.iters, rZ.iters) == want
    assert a.count(sz, sx, ex, ez, pX, pZ, rX.iters, rZ.iters) == want
    assert a.count(wz, wx, ex, ez, rX.ehat, rZ.ehat, rX.iters, rZ.iters) == want
    assert want["decSuccessExact"] > 0


def test_host_decode_path_pinned_staging_matches_device_path():
    """qldpc_decode_host (pinned staging on its own stream) equals the device
    entry point."""
    import torch
    from qldpcsim_amd import codes, decoders
    Hx, Hz = codes.load_code("LP118_0")
    rng = np.random.default_rng(4)
    syn = rng.integers(0, 2, (777, Hz.shape[0]), dtype=np.uint8)
    h = decoders.decode_batch(Hz, syn, 0.02, 20, want_post=True)
    d = decoders.decode_batch(Hz, torch.as_tensor(syn, device="cuda"), 0.02, 20, want_post=True)
    np.testing.assert_array_equal(h.ehat, d.ehat.cpu().numpy())
    np.testing.assert_array_equal(h.iters, d.iters.cpu().numpy())
    np.testing.assert_array_equal(h.post, d.post.cpu().numpy())
