// channel_kernels.h — device depolarizing sampler and outcome counters
// (simulate_p's shot source and counters), shared with capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qldpc {

// CSR of Hx and Hz (original column order), as qldpc_code holds them on the device.
struct PairTabs {
  const int32_t* rp_x;
  const int32_t* ci_x;
  const int32_t* rp_z;
  const int32_t* ci_z;
  int mx, mz, ex, ez;  // rows and edges of Hx / Hz
  int n, W;            // qubits, 64-bit words per packed error vector
  int udeg;            // row degree shared by every row of Hx and Hz, else 0
};

struct SampleArgs {
  PairTabs t;
  uint64_t* errx;  // [batch][W]
  uint64_t* errz;  // [batch][W]
  uint8_t* syz;    // [batch][mz]  Hz errX mod 2 (syn_bits: uint64 [batch][ceil(mz/64)])
  uint8_t* syx;    // [batch][mx]  Hx errZ mod 2
  int syn_bits;
  long long batch;
  uint64_t shot0;
  uint32_t key0, key1;
  uint64_t t1, t2, t3;  // X: u < t1, Y: t1 <= u < t2, Z: t2 <= u < t3 (u a 32-bit draw)
};

struct CountArgs {
  PairTabs t;
  const uint64_t* errx;  // [batch][W]
  const uint64_t* errz;
  const uint8_t* syz;    // [batch][mz]
  const uint8_t* syx;    // [batch][mx]
  const uint8_t* ehx;    // [batch][n] X-half estimate (decodes Hz)
  const uint8_t* ehz;    // [batch][n] Z-half estimate (decodes Hx)
  int syn_bits, eh_bits; // uint64 words instead of bytes (bit j % 64 of word j / 64)
  const int32_t* itx;    // [batch]
  const int32_t* itz;
  unsigned long long* acc;  // [6] accumulated
  long long batch;
};

constexpr int kChannelWaves = 4;  // waves per workgroup (one shot per wave at a time)

// LDS bytes the two kernels need for these tables
int channel_lds_bytes(const PairTabs& t, bool counters);
hipError_t launch_channel_sample(const SampleArgs& a, int grid, hipStream_t stream);
hipError_t launch_count_outcomes(const CountArgs& a, int grid, hipStream_t stream);

}  // namespace qldpc
