// osd_kernels.h — batched GPU OSD (decoders.py:299-370), shared with capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qldpc {

struct OsdArgs {
  const int32_t* row_ptr;  // [m+1] CSR of H (original columns)
  const int32_t* col_idx;  // [E]
  const int32_t* perm;     // [count][n] reliability order (NumPy argsort, decoders.py:325)
  const uint8_t* syn;      // [count][m]
  uint8_t* ehat;           // [count][n] in/out
  int32_t* status;         // [count] 0 ok, 1 = reference IndexError case, 2 = order left to the host
                           // (3 = internal: osd_block_kernel hands the shot to osd_kernel)
  const int32_t* tiepos;   // [count] or null: osd_order_kernel's verdict; -1 = the order is
                           // left to NumPy on the host: the shot is left untouched (status 2)
  const double* post;      // [count][n] posteriors (spilled for status-2 shots), with tiepos
  int m, n, rank, order;
  // status-2 spill (optional): a shot left to the host also copies its
  // posterior row to spill_post[slot] and its index to spill_idx[slot],
  // slot = atomicAdd(spill_count, 1) (< spill_cap), so the host can fetch
  // exactly those rows with one DMA copy, no gather kernel
  double* spill_post;      // [spill_cap][n]
  int32_t* spill_idx;      // [spill_cap] shot index within the call
  int32_t* spill_count;    // [1]
  long long spill_cap, shot_base;
  unsigned long long* prof; // QLDPC_OSD_TIMING builds only: per-phase cycle sums
  uint32_t* cu_tickets;    // [kOsdCuSlots] per-CU workgroup tickets (engine SIMD choice), or null
  int redo;                // osd_kernel only: process just the shots whose status is 3
                           // (left by osd_block_kernel: syndrome outside H's column space)
};

// Reliability order on the device (decoders.py:320-325): NumPy's exact order
// (osd_order_kernel); tiepos = n, or -1 where the host's NumPy must decide.
struct OrderArgs {
  const double* post;      // [count][n]
  int32_t* perm;           // [count][n]
  int32_t* tiepos;         // [count]
  int n;                   // <= 2048
};
constexpr int kOsdCuSlots = 16 * 256;  // XCC id (4 bits) x HW_ID bits 8-15 (CU, SH, SE)
hipError_t launch_osd_order(const OrderArgs& a, long long count, hipStream_t stream);
size_t osd_order_lds(int n);

// osd_hbm_kernel (any m, n): each shot's working matrix lives in a global
// scratch slice instead of VGPRs / LDS. Per shot, at `scratch + shot *
// stride` (shot = the launch's blockIdx.x): R [nwr][mp] u64 (word-major: word
// q of the row at REF position p at q * mp + p; nwr = ceil((n + 1) / 64), mp =
// m rounded up to 64), then inv_perm [n] i32 at off_inv, the J list [m + 2]
// i32 at off_jl, inJ [n] bytes at off_inj and the CPython set table (order 1)
// at off_table. LDS: the current word of every row [mp] u64 + 3 [nwr] u64 + 160 B.
struct OsdHbmArgs {
  unsigned char* scratch;
  long long stride;
  int nwr, mp, off_inv, off_jl, off_inj, off_table;
};
const void* osd_hbm_kernel_ptr();        // __global__ osd_hbm_kernel(OsdArgs, OsdHbmArgs)
inline size_t osd_hbm_lds(int m, int nwr) { return 8 * (size_t)((m + 63) / 64 * 64) + 24 * (size_t)nwr + 160; }

const void* select_osd_kernel(int nw);  // nw = 64-bit words per row incl. the syndrome column
const void* select_osd_block_kernel(int nw, int m, int* rows_per_thread);  // block elimination (default), same arguments
int osd_nw_of(int nw);

}  // namespace qldpc
