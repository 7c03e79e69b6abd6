"""qldpcsim_amd — MI355X-native batched BP / Min-Sum decoding for qLDPCsim.

Drop-in for the reference's decode hot path (albertogp71/qLDPCsim):
  qldpcsim_amd.decoders   MS_decoder / BP_decoder / OSDdec / decode_batch
  qldpcsim_amd.simulator  load_matrix / simulate_p / simulate / main
  qldpcsim_amd.ops        torch.ops.qldpc.decode (the batched decoder as a PyTorch operator)
The decoders run as hand-written HIP kernels for gfx950 behind the C ABI in
include/qldpc_decoder.h; importing `decoders` or `simulator` fails loudly if
the HIP library has not been built.
"""
__version__ = "0.1.0"
__all__ = ["codes", "schedule", "decoders", "simulator", "ops"]
