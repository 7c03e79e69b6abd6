// Where do the waves of a 4-wave workgroup land? Records HW_ID (SIMD, CU, SE)
// and XCC_ID per wave for a grid shaped like osd_block_kernel's launches
// (256-thread workgroups, enough LDS per workgroup for 4 per CU).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
__global__ void __launch_bounds__(256) probe(uint32_t* out, int spin) {
  extern __shared__ unsigned char lds[];
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
  lds[threadIdx.x] = (unsigned char)threadIdx.x;
  long long t0 = clock64();
  while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
  if ((threadIdx.x & 63) == 0) {
    out[2 * (blockIdx.x * 4 + threadIdx.x / 64)] = hw;
    out[2 * (blockIdx.x * 4 + threadIdx.x / 64) + 1] = xcc;
  }
}
int main() {
  const int nb = 4096;
  uint32_t* d;
  hipMalloc(&d, nb * 4 * 2 * 4);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 36000, 0, d, 200000);
  hipDeviceSynchronize();
  uint32_t* h = (uint32_t*)malloc(nb * 4 * 2 * 4);
  hipMemcpy(h, d, nb * 4 * 2 * 4, hipMemcpyDeviceToHost);
  int hist[4][4] = {{0}};
  int distinct = 0;
  for (int b = 0; b < nb; ++b) {
    int mask = 0;
    for (int w = 0; w < 4; ++w) {
      const uint32_t hw = h[2 * (b * 4 + w)];
      const int simd = (hw >> 4) & 3;
      hist[w][simd]++;
      mask |= 1 << simd;
    }
    distinct += mask == 15;
  }
  for (int w = 0; w < 4; ++w) printf("wave %d simd hist: %d %d %d %d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
  printf("workgroups with 4 distinct SIMDs: %d of %d\n", distinct, nb);
  for (int b = 0; b < 8; ++b) printf("wg %d: hw %08x %08x %08x %08x xcc %x\n", b, h[8 * b], h[8 * b + 2], h[8 * b + 4], h[8 * b + 6], h[8 * b + 1]);
  return 0;
}
