// hbm_kernels.h — the HBM-resident decoder (codes whose per-half-shot state
// does not fit a CU's LDS, or whose tables overflow the 16-bit LDS formats).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tuning.h"

namespace qldpc {

// One workgroup of kHbmWaves waves = one tile of 64 half-shot slots (lane l =
// slot l); every lane of a wave walks the same check / variable at the same
// time, so graph reads are wave-uniform (scalar loads) and message reads are
// coalesced: tile g's element i of slot l at [g][i][64].
constexpr int kHbmWaves = QLDPC_HBM_WAVES;   // (kernel names in hbm_kernels.hip spell out 4)
struct HbmArgs {
  // graph (relabeled variables, int32, global)
  const int32_t* row_ptr;   // [m+1] CSR
  const int32_t* row_var;   // [E]   relabeled variable of CSR edge e (ascending original variable)
  const int32_t* row_pos;   // [E]   CSC position of CSR edge e
  const int32_t* col_ptr;   // [n+1] CSC over relabeled variables (ascending check inside a column)
  const int32_t* vinv;      // [n]   original column -> relabeled variable
  const uint32_t* wc;       // [m]   stop-test filter word per check
  const uint32_t* avar;     // [n]   filter word per relabeled variable
  uint32_t filt_all;
  // schedule
  const int32_t* lay_ptr;   // [L+1]
  const int32_t* lay_rows;  // [*]
  const int32_t* adj_ptr;   // [L+1]
  const int32_t* adj_vars;  // [*]   relabeled variables adjacent to the layer's rows, ascending
  int n_layers;
  int m, n, E;
  // workspace (tile-major: [tiles][elements][64 slots])
  void* c2v;                // [tiles][E][64]  float (MS) / double (BP)
  void* post;               // [tiles][n][64]  float32 column sum S (MS) / float64 posterior (BP)
  uint8_t* synT;            // [tiles][m][64]
  // batch
  const uint8_t* syn;       // [batch][m] bytes, or uint64 [batch][wm] words
  uint8_t* ehat;            // [batch][n] bytes, or uint64 [batch][wn] words
  int32_t* iters;
  double* out_post;         // [batch][n] original order, or null
  int32_t* flags;
  int syn_bits, eh_bits, wm, wn;
  long long batch;
  uint32_t* queue;          // shot ticket counter (zeroed before the launch)
  double L, beta, eps;
  float L32;
  int max_iter;
};

// dcmax: row degree bound of the instantiation (8, 16, 32 or 64)
const void* select_hbm_kernel(int algo, int dcmax, const char** name);
// fl_var / fl_pos: first layer reaching each variable / CSC position; lazy =
// the layers partition the rows (no state initialisation pass)
hipError_t launch_hbm(const void* kernel, const HbmArgs& a, int tiles, const int32_t* fl_var, const int32_t* fl_pos,
                      int lazy, hipStream_t stream);

}  // namespace qldpc
