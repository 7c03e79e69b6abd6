// kargs.h — kernel arguments read afresh from the kernarg segment.
#pragma once
#include <hip/hip_runtime.h>

namespace qldpc {

// The kernel's first argument (a struct T at kernarg offset 0), read afresh
// from the kernarg segment (scalar loads) at the point of use: an argument
// used only before or after a long loop then occupies no SGPRs during it,
// where the compiler would otherwise keep it live and spill other SGPRs to
// VGPR lanes inside the loop.
template <typename T>
__device__ __forceinline__ const T& kargs_fresh() {
  typedef const T __attribute__((address_space(4))) KArgs;
  KArgs* p = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const T*)p;
}

}  // namespace qldpc
