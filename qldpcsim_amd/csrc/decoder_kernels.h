// decoder_kernels.h — shared between the HIP kernels and the C-ABI host code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// threads per workgroup the kernels are compiled for (waves per WG <= this/64)
#define QLDPC_MAX_THREADS 768
// max runs of equal column degree the flooding MS kernel handles
#define QLDPC_MAX_RUNS 8
#define QLDPC_FLOOD_HDR 128  // LDS bytes of ms_flood_kernel's runs header (4 * 8 ints)

namespace qldpc {

enum { ALGO_MS = 0, ALGO_BP = 1 };
enum { FLAG_CONVERGED = 1, FLAG_MIN_ZERO = 2, FLAG_NONFINITE = 4 };

// Kernel arguments (by value). Offsets are byte offsets inside the LDS image:
// [blob (graph tables, staged from `blob`)][wave 0 state][wave 1 state]...
struct DecodeArgs {
  const unsigned char* blob;  // device copy of the LDS table image
  int blob_bytes;             // multiple of 16
  int off_cn_tab, off_row_ptr, off_vn_ptr, off_vn_chk;
  int off_lay_ptr, off_lay_rows, off_adj_ptr, off_adj_vars, off_chunk_dmax;
  int wave_bytes;             // per-wave state slice (multiple of 16)
  int off_c2v, off_synw, off_parw;  // inside a wave slice (post f64[n] at 0)
  int off_red;                // bp_team_kernel: team reduction / ticket slots inside the team slice
  int m, n, E, n_layers;
  const uint16_t* vinv;       // [n] original column -> relabeled variable (global)
  const uint8_t* syn;         // [batch][m]
  uint8_t* ehat;              // [batch][n]
  int32_t* iters;             // [batch]
  double* post;               // [batch][n] or null
  int32_t* flags;             // [batch] or null
  long long batch;
  double L;                   // log((1-p)/max(p,eps))
  float L32;                  // float32(L)
  double beta, eps;
  int max_iter;
  uint32_t* queue;            // half-shot work queue (zeroed before the launch), or null = static stride
  // ms_layered_kernel's stop-test filters: 32 random parity
  // checks w_k of H's rows; wc[c] = bit k set if w_k holds row c
  const uint32_t* wc;         // [m]   global
  const uint32_t* rtab;       // [m][8] relabeled variables of each row (global; exact stop test)
  uint32_t filt_all;          // XOR of every variable's filter word (all hard decisions 1)
  const uint32_t* avar;       // [n]   global: filter word per relabeled variable (bp_team_kernel)
  float hd_thresh;            // hard decision of a column sum S: (L + (f64)S < 0) == (S < hd_thresh)
  // bit-packed I/O: syn as uint64 [batch][wm] words, ehat as uint64 [batch][wn]
  // (bit j % 64 of word j / 64) instead of one byte per bit
  int syn_bits, eh_bits;
  int wm, wn;                 // ceil(m / 64), ceil(n / 64)
  int off_libm;               // BP: LDS byte offset of the qldpc_libm_tab image (after every slice)
  int lds_skip;               // ms_layered_kernel (QLDPC_MSL_GT): blob bytes before the LDS image
  // BP saturated check nodes (decoder_kernels.hip, cn_bp_word): c2v magnitude
  // 2 atanh(1 - eps) and the |x| >= 19.5 high-word threshold (0x7ff00000: off)
  double bp_csat;
  uint32_t bp_sat_hi;
};

// `name` (nullable) receives the kernel's name as rocprofv3 reports it
const void* select_kernel(int algo, bool layered, int dc, const char** name);
// flooding MS, uniform row degree: global tables (fblob), LDS = wave state only
const void* select_ms_flood_kernel(int dc, int kc, const char** name);  // nullptr if no instantiation fits
int ms_flood_max_waves(int kc);                      // waves per workgroup it was compiled for
// layered MS, uniform row degree 7/8, G = 1/2/4/8 lanes per check (layer-table blob)
const void* select_ms_layered_kernel(int dc, int g, const char** name);
// layered BP teams, every graph table in global memory (gblob of the schedule)
const void* select_bp_team_lg_kernel(int dc, int w, const char** name);
// BP, uniform row degree 7/8: one team of W waves per half-shot, edge-parallel check nodes
const void* select_bp_team_kernel(bool layered, int dc, int w, const char** name);
hipError_t launch_decode(const void* kernel, const DecodeArgs& args, int grid, int block,
                         int lds_bytes, hipStream_t stream);
hipError_t configure_kernel(const void* kernel, int lds_bytes);

}  // namespace qldpc
