"""The decoder as a registered PyTorch operator (qldpcsim_amd/ops.py):
registration, shape inference on meta tensors, loud failure on CPU tensors
(no CPU path); on the GPU, equality with decode_batch."""
import numpy as np
import pytest
import torch

from qldpcsim_amd import codes, ops, schedule  # noqa: F401  (registers torch.ops.qldpc)


def _args(code="LP118_0", sched="L"):
    Hx, Hz = codes.load_code(code)
    lx, _ = schedule.select_layers(Hx, Hz, sched)
    lp, lr = schedule.pack_layers(lx, Hz.shape[0])
    return Hz, torch.as_tensor(Hz), torch.as_tensor(lp), torch.as_tensor(lr)


def test_op_is_registered_and_infers_shapes_on_meta():
    # registered from C++ (torch_ops.cpp, TORCH_LIBRARY) by the library built
    # beside the decoder library this process loaded (in-tree by default,
    # QLDPC_LIB's directory for an out-of-tree build)
    import os
    from qldpcsim_amd import _lib
    assert ops.TORCH_OPS_PATH == os.path.join(os.path.dirname(_lib.LIB_PATH), "libqldpc_torch.so")
    if "QLDPC_LIB" not in os.environ:
        assert ops.TORCH_OPS_PATH.endswith(os.path.join("qldpcsim_amd", "_build", "libqldpc_torch.so"))
    sch = str(torch.ops.qldpc.decode.default._schema)
    assert sch.startswith("qldpc::decode(Tensor syndromes, Tensor H, Tensor layer_ptr, Tensor layer_rows")
    Hz, H, lp, lr = _args()
    m, n = Hz.shape
    syn = torch.empty((17, m), dtype=torch.uint8, device="meta")
    e, it, post, fl = torch.ops.qldpc.decode(syn, H, lp, lr, 0.01, 10, "MS", 0.75, 1e-9, True, False)
    assert e.shape == (17, n) and e.dtype == torch.uint8 and it.shape == (17,) and it.dtype == torch.int32
    assert post.shape == (17, n) and post.dtype == torch.float64 and fl.shape == (17,)
    words = torch.empty((5, (m + 63) // 64), dtype=torch.int64, device="meta")
    e, it, post, fl = torch.ops.qldpc.decode(words, H, lp, lr, 0.01, 10, "BP", 0.75, 1e-9, False, True)
    assert e.shape == (5, (n + 63) // 64) and e.dtype == torch.int64 and post.shape == (5, 0)


def test_op_refuses_cpu_tensors():
    Hz, H, lp, lr = _args()
    with pytest.raises(ValueError, match="HIP device"):
        torch.ops.qldpc.decode(torch.zeros((2, Hz.shape[0]), dtype=torch.uint8), H, lp, lr, 0.01, 5)


@pytest.mark.gpu
@pytest.mark.parametrize("code,sched,algo", [("LP118_0", "F", "MS"), ("LP118_2", "L", "MS"), ("LP04_0", "L", "BP")])
def test_op_equals_decode_batch(code, sched, algo):
    from qldpcsim_amd import decoders
    Hz, H, lp, lr = _args(code, sched)
    g = torch.Generator(device="cuda").manual_seed(3)
    syn = torch.randint(0, 2, (2048, Hz.shape[0]), dtype=torch.uint8, device="cuda", generator=g)
    e, it, post, fl = torch.ops.qldpc.decode(syn, H, lp, lr, 0.02, 20, algo, 0.75, 1e-9, True, False)
    ref = decoders.decode_batch(Hz, syn, 0.02, 20, algo=algo, layer_ptr=lp.numpy(), layer_rows=lr.numpy(),
                                want_post=True)
    assert torch.equal(e, ref.ehat) and torch.equal(it, ref.iters) and torch.equal(fl, ref.flags)
    assert torch.equal(post, ref.post)
    eb, itb, _, _ = torch.ops.qldpc.decode(decoders.pack_bits(syn), H, lp, lr, 0.02, 20, algo, 0.75, 1e-9,
                                          False, True)
    assert torch.equal(decoders.unpack_bits(eb, Hz.shape[1]), ref.ehat) and torch.equal(itb, ref.iters)


@pytest.mark.gpu
def test_op_cache_hits_by_content_and_release():
    """The op's graph cache is keyed by H's content (a copy of H hits it, an
    edited H does not) and torch.ops.qldpc.release() frees it; decoding after
    a release rebuilds the graph and gives the same results."""
    from qldpcsim_amd import decoders
    Hz, H, lp, lr = _args("LP04_0", "F")
    g = torch.Generator(device="cuda").manual_seed(4)
    syn = torch.randint(0, 2, (300, Hz.shape[0]), dtype=torch.uint8, device="cuda", generator=g)
    a = torch.ops.qldpc.decode(syn, H, lp, lr, 0.03, 15, "MS", 0.75, 1e-9, True, False)
    b = torch.ops.qldpc.decode(syn, H.clone(), lp, lr, 0.03, 15, "MS", 0.75, 1e-9, True, False)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    H2 = H.clone()
    H2[0, :] = 0                                            # a different matrix: its own graph
    c = torch.ops.qldpc.decode(syn, H2, lp, lr, 0.03, 15, "MS", 0.75, 1e-9, True, False)
    ref2 = decoders.decode_batch(H2.numpy(), syn, 0.03, 15, algo="MS", layer_ptr=lp.numpy(),
                                 layer_rows=lr.numpy(), want_post=True)
    assert torch.equal(c[0], ref2.ehat) and torch.equal(c[1], ref2.iters)
    torch.ops.qldpc.release()
    d = torch.ops.qldpc.decode(syn, H, lp, lr, 0.03, 15, "MS", 0.75, 1e-9, True, False)
    assert all(torch.equal(x, y) for x, y in zip(a, d))
