// ms_flood_kernels.hip — the flooding min-sum kernel (ms_flood_kernel,
// decoder_kernels.hip; the headline decoder) instantiated in a translation
// unit of its own, built with the AMDGPU max-ILP machine scheduler
// (-mllvm -amdgpu-sched-strategy=max-ilp, Makefile): 46.66 -> 46.04 ms per
// LP118_0 fixed-work launch; the same strategy slows the layered min-sum
// (+1.3 %), BP (+0.4 / +3.6 %) and OSD (+0.2 %) kernels, which keep the
// default. profiles/r06/r06p_ab_sched_strategies.json.
#define QLDPC_TU_FLOOD 1
#include "decoder_kernels.hip"
