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
  int32_t* status;         // [count] 0 ok, 1 = reference IndexError case
  int m, n, rank, order;
};

const void* select_osd_kernel(int nw);  // nw = 64-bit words per row incl. the syndrome column
int osd_nw_of(int nw);

}  // namespace qldpc
