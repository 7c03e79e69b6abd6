// bp_team_kernels.hip — the sum-product team kernels (bp_team_kernel,
// bp_team_lg_kernel, decoder_kernels.hip) instantiated in a translation unit
// of their own, built with -fno-slp-vectorize (Makefile): the SLP vectorizer
// packed pairs of their float64 / index operations with register moves
// between, measured 1.4 % slower per LP118_2 BP-L launch and 1.2 % per LP118_0
// BP-F launch; the min-sum kernels keep it (the layered one is 0.3 % faster
// with it). profiles/r06/r06l_ab_noslp.json.
#define QLDPC_TU_BP_TEAM 1
#include "decoder_kernels.hip"
