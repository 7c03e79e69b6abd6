// Probe: where does global_load_lds_ubyte put lane i's byte in LDS (base + i, or base + 4 i)?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ void k(const uint8_t* src, uint8_t* out) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[512];
  const int lane = threadIdx.x;
  for (int i = lane; i < 512; i += 64) lds[i] = 0xEE;
  __syncthreads();
  if (lane < 60)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + lane),
                                     (__attribute__((address_space(3))) void*)(lds + 64), 1, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 512; i += 64) out[i] = lds[i];
}
int main() {
  uint8_t h[64], *d, *o, r[512];
  for (int i = 0; i < 64; ++i) h[i] = (uint8_t)(i + 1);
  hipMalloc(&d, 64); hipMalloc(&o, 512);
  hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o);
  hipMemcpy(r, o, 512, hipMemcpyDeviceToHost);
  for (int i = 0; i < 320; ++i) printf("%02x%c", r[i], (i % 32 == 31) ? '\n' : ' ');
  return 0;
}
