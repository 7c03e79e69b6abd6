"""The batched decoder as a registered PyTorch-ROCm C++ operator (torch.library).

    torch.ops.qldpc.decode(syndromes, H, layer_ptr, layer_rows, p, max_iter,
                           algo="MS", beta=0.75, eps=1e-9, want_post=False,
                           ehat_bits=False) -> (ehat, iters, post, flags)

The same computation as decoders.decode_batch on a device tensor (the HIP
kernels behind the C ABI, include/qldpc_decoder.h), registered from C++
(qldpcsim_amd/csrc/torch_ops.cpp: TORCH_LIBRARY, HIP dispatch key) so that
torch code (torch.compile graphs, custom pipelines) calls the decoder like any
other op without Python in the call path: it runs on torch's current HIP
stream of the syndromes' device, allocates its outputs through torch's
caching allocator, and caches the Tanner graph and schedules per (device, H).
The fake (meta) implementation below gives torch.compile the output shapes.
Replaces, per batch, the reference's per-shot MS_decoder / BP_decoder calls
(qLDPCsim/decoders.py:110-117, :189-195).

Arguments: `syndromes` uint8 [B, m] (one byte per check) or int64
[B, ceil(m/64)] (bit-packed words) on a HIP device; `H` the parity-check
matrix and `layer_ptr` / `layer_rows` the schedule (schedule.pack_layers) as
CPU tensors. Outputs: ehat uint8 [B, n] (int64 [B, ceil(n/64)] with
ehat_bits), iters int32 [B], post float64 [B, n] (or [B, 0] unless
want_post), flags int32 [B]. Errors as decode_batch: ValueError for shapes /
options, RuntimeError for HIP failures; a CPU tensor raises (no CPU path).
"""
import os

import torch

from . import _lib

__all__ = ["decode", "TORCH_OPS_PATH"]

# the C++ operator library (qldpcsim_amd/csrc/torch_ops.cpp, built in-tree by
# __graft_entry__.build / make -C qldpcsim_amd/csrc torch); it links the
# kernels' libqldpc_hip.so. No Python fallback: a missing build fails loudly.
TORCH_OPS_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), "libqldpc_torch.so")
if not os.path.exists(TORCH_OPS_PATH):
    raise ImportError(f"{TORCH_OPS_PATH} is missing: build it with make -C qldpcsim_amd/csrc torch")
torch.ops.load_library(TORCH_OPS_PATH)
decode = torch.ops.qldpc.decode


@torch.library.register_fake("qldpc::decode")
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
