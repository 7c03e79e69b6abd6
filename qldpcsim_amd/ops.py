"""The batched decoder as a registered PyTorch operator (torch.library).

    torch.ops.qldpc.decode(syndromes, H, layer_ptr, layer_rows, p, max_iter,
                           algo="MS", beta=0.75, eps=1e-9, want_post=False,
                           ehat_bits=False) -> (ehat, iters, post, flags)

The same computation as decoders.decode_batch on a device tensor (the HIP
kernels behind the C ABI, include/qldpc_decoder.h), exposed as a PyTorch-ROCm
operator so that torch code (torch.compile graphs, custom pipelines) can call
the decoder like any other op: it runs on torch's current stream of the
syndromes' device and allocates its outputs through torch's caching
allocator. Replaces, per batch, the reference's per-shot MS_decoder /
BP_decoder calls (qLDPCsim/decoders.py:110-117, :189-195).

Arguments: `syndromes` uint8 [B, m] (one byte per check) or int64
[B, ceil(m/64)] (bit-packed words) on a HIP device; `H` the parity-check
matrix and `layer_ptr` / `layer_rows` the schedule (schedule.pack_layers) as
CPU tensors. Outputs: ehat uint8 [B, n] (int64 [B, ceil(n/64)] with
ehat_bits), iters int32 [B], post float64 [B, n] (or [B, 0] unless
want_post), flags int32 [B]. Errors as decode_batch: ValueError for shapes /
options, RuntimeError for HIP failures; a CPU tensor raises (no CPU path).
"""
import numpy as np
import torch

from . import decoders

__all__ = ["decode"]


def _check_device(syndromes):
    if syndromes.device.type != "cuda":
        raise ValueError("qldpc::decode runs on a HIP device: syndromes must be a device tensor "
                         f"(got {syndromes.device})")


@torch.library.custom_op("qldpc::decode", mutates_args=())
def decode(syndromes: torch.Tensor, H: torch.Tensor, layer_ptr: torch.Tensor, layer_rows: torch.Tensor,
           p: float, max_iter: int, algo: str = "MS", beta: float = 0.75, eps: float = 1e-9,
           want_post: bool = False, ehat_bits: bool = False
           ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    _check_device(syndromes)
    Hn = H.detach().cpu().numpy()
    lp = layer_ptr.detach().cpu().numpy().astype(np.int32)
    lr = layer_rows.detach().cpu().numpy().astype(np.int32)
    with torch.cuda.device(syndromes.device):
        r = decoders.decode_batch(Hn, syndromes, p, max_iter, algo=algo, beta=beta, eps=eps,
                                  want_post=want_post, layer_ptr=lp, layer_rows=lr, ehat_bits=ehat_bits)
    post = r.post if r.post is not None else torch.empty((syndromes.shape[0], 0), dtype=torch.float64,
                                                           device=syndromes.device)
    return r.ehat, r.iters, post, r.flags


@decode.register_fake
def _(syndromes, H, layer_ptr, layer_rows, p, max_iter, algo="MS", beta=0.75, eps=1e-9,
      want_post=False, ehat_bits=False):
    B = syndromes.shape[0]
    n = H.shape[1]
    dev = syndromes.device
    ehat = (syndromes.new_empty((B, (n + 63) // 64), dtype=torch.int64) if ehat_bits
            else syndromes.new_empty((B, n), dtype=torch.uint8))
    post = syndromes.new_empty((B, n if want_post else 0), dtype=torch.float64)
    return (ehat, syndromes.new_empty((B,), dtype=torch.int32), post,
            torch.empty((B,), dtype=torch.int32, device=dev))
