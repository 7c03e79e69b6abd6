// channel_kernels.hip — the Monte-Carlo shot source and the outcome counters
// of simulate_p on the device (gfx950), so a simulation batch never leaves HBM.
//
// channel_sample_kernel replaces the Stim sample of the reference circuit
// (simulator.py:196-197: PAULI_CHANNEL_1(p/3,p/3,p/3) on every data qubit,
// :107, then the row slicing :249-252) by its statistical equivalent
// (SURVEY.md App. A.5), drawn from a counter-based generator so any shot of
// the stream can be produced independently:
//     u(shot, j) = Philox4x32-10(key = seed, ctr = (j % 64, (j / 64) / 4,
//                                shot_lo, shot_hi))[(j / 64) % 4]
//     X if u < T1, Y if T1 <= u < T2, Z if T2 <= u < T3, T_k = floor(k·(p/3)·2^32)
//     errX = X | Y, errZ = Z | Y, sy_z = Hz·errX mod 2, sy_x = Hx·errZ mod 2
// Error vectors are written bit-packed (bit j % 64 of word j / 64): they are
// only read again by the counters. Syndromes are written as bytes or, with
// syn_bits, as words of the same layout (the decoder reads either).
// oracle/qldpc_oracle.c restates the same stream.
//
// count_outcomes_kernel forms the reference's per-shot outcomes
// (simulator.py:291-303) and sums them into six int64 counters:
//     exact  errX == eX and errZ == eZ                           (:294-295)
//     degen  not exact, Hz @ (errX ^ eX) == 0 and Hx @ (errZ ^ eZ) == 0 over
//            the integers, no mod 2 (:296-298): with 0/1 entries that is
//            "the difference has no support on a column of nonzero weight"
//     failX  Hz·eX mod 2 != sy_z,  failZ  Hx·eZ mod 2 != sy_x      (:300-303)
//     iteration sums                                              (:291-292)
//
// Both kernels: one wavefront per shot (grid-stride), CSR of Hx / Hz staged
// once per workgroup into LDS as 16-bit column indices; lane l owns bit l of
// every 64-qubit word (ballots assemble the words); checks are lane-parallel.
// HBM-bound byte work, no MFMA: per shot the sampler writes 2·8·W + m_x + m_z
// bytes, the counter reads them back with the 2n estimate bytes.

#include "channel_kernels.h"

namespace qldpc {
namespace {

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Philox4x32-10 (Salmon et al., SC'11), counter (c0..c3), key (k0, k1).
__device__ __forceinline__ uint4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product (hi and lo together)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

struct Tabs {
  const int* rpz;
  const int* rpx;
  const uint16_t* ciz;
  const uint16_t* cix;
  unsigned char* tail;  // 8-byte aligned, after the tables
};

__device__ __forceinline__ int align8(int x) { return (x + 7) & ~7; }

// stage both CSR tables into LDS (whole workgroup; caller syncs)
__device__ Tabs stage_tables(const PairTabs& t, unsigned char* smem) {
  int* rpz = reinterpret_cast<int*>(smem);
  int* rpx = rpz + (t.mz + 1);
  uint16_t* ciz = reinterpret_cast<uint16_t*>(rpx + (t.mx + 1));
  uint16_t* cix = ciz + t.ez;
  const int tail = align8(4 * (t.mz + 1 + t.mx + 1) + 2 * (t.ez + t.ex));
  for (int i = threadIdx.x; i <= t.mz; i += blockDim.x) rpz[i] = t.rp_z[i];
  for (int i = threadIdx.x; i <= t.mx; i += blockDim.x) rpx[i] = t.rp_x[i];
  for (int i = threadIdx.x; i < t.ez; i += blockDim.x) ciz[i] = (uint16_t)t.ci_z[i];
  for (int i = threadIdx.x; i < t.ex; i += blockDim.x) cix[i] = (uint16_t)t.ci_x[i];
  return Tabs{rpz, rpx, ciz, cix, smem + tail};
}

// Parity of row c of a CSR table over the packed vector `w` (LDS, 32-bit
// words: bit j % 32 of word j / 32). DC > 0: every row has DC entries (rows
// start at c·DC; the reads are unrolled and issued together).
template <int DC>
__device__ __forceinline__ uint32_t row_parity(const int* rp, const uint16_t* ci, int c,
                                               const uint32_t* w) {
  uint32_t par = 0;
  if constexpr (DC > 0) {
    uint32_t j[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) j[k] = ci[c * DC + k];
#pragma unroll
    for (int k = 0; k < DC; ++k) par ^= w[j[k] >> 5] >> (j[k] & 31);
  } else {
    const int e1 = rp[c + 1];
    for (int e = rp[c]; e < e1; ++e) {
      const uint32_t j = ci[e];
      par ^= w[j >> 5] >> (j & 31);
    }
  }
  return par & 1u;
}

template <int DC>
__global__ void __launch_bounds__(64 * kChannelWaves) channel_sample_kernel(SampleArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const PairTabs& t = a.t;
  const Tabs tb = stage_tables(t, smem);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int W = t.W;
  uint64_t* wx = reinterpret_cast<uint64_t*>(tb.tail) + wave * 2 * W;  // errX words
  uint64_t* wz = wx + W;                                                // errZ words
  const uint32_t* wx32 = reinterpret_cast<const uint32_t*>(wx);
  const uint32_t* wz32 = reinterpret_cast<const uint32_t*>(wz);
  __syncthreads();
  for (long long b = (long long)blockIdx.x * kChannelWaves + wave; b < a.batch;
       b += (long long)gridDim.x * kChannelWaves) {
    const uint64_t shot = a.shot0 + (uint64_t)b;
    uint64_t myx = 0, myz = 0;
    for (int wq = 0; 4 * wq < W; ++wq) {
      const uint4 r = philox4x32_10((uint32_t)lane, (uint32_t)wq, (uint32_t)shot,
                                    (uint32_t)(shot >> 32), a.key0, a.key1);
      const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int w = 4 * wq + i;
        if (w >= W) break;  // wave-uniform
        const bool v = 64 * w + lane < t.n;
        const uint64_t u = rr[i];
        const uint64_t bx = __ballot(v && u < a.t2);
        const uint64_t bz = __ballot(v && u >= a.t1 && u < a.t3);
        if (lane == w) {
          myx = bx;
          myz = bz;
        }
      }
    }
    if (lane < W) {
      wx[lane] = myx;
      wz[lane] = myz;
      a.errx[b * W + lane] = myx;
      a.errz[b * W + lane] = myz;
    }
    wave_sync();
    if (a.syn_bits) {                           // one 64-bit word per 64 checks (ballot)
      const int wmz = (t.mz + 63) >> 6, wmx = (t.mx + 63) >> 6;
      for (int c0 = 0; c0 < t.mz; c0 += 64) {
        const int c = c0 + lane;
        const uint64_t bits = __ballot(c < t.mz && row_parity<DC>(tb.rpz, tb.ciz, c < t.mz ? c : 0, wx32));
        if (lane == 0) reinterpret_cast<uint64_t*>(a.syz)[b * wmz + (c0 >> 6)] = bits;
      }
      for (int c0 = 0; c0 < t.mx; c0 += 64) {
        const int c = c0 + lane;
        const uint64_t bits = __ballot(c < t.mx && row_parity<DC>(tb.rpx, tb.cix, c < t.mx ? c : 0, wz32));
        if (lane == 0) reinterpret_cast<uint64_t*>(a.syx)[b * wmx + (c0 >> 6)] = bits;
      }
    } else {
      for (int c = lane; c < t.mz; c += 64)
        a.syz[b * t.mz + c] = (uint8_t)row_parity<DC>(tb.rpz, tb.ciz, c, wx32);
      for (int c = lane; c < t.mx; c += 64)
        a.syx[b * t.mx + c] = (uint8_t)row_parity<DC>(tb.rpx, tb.cix, c, wz32);
    }
    wave_sync();  // the next shot overwrites wx / wz
  }
}

// Pack one estimate row (uint8 [n], 0/1) into the per-wave LDS bit vector
// `dst` (bytes; bit j % 8 of byte j / 8), all loads issued up front.
// VEC: n % 4 == 0, so each lane reads 4 estimates with one aligned 32-bit
// load (lane l of chunk k: qubits 256k + 4l .. + 3) and turns them into a
// nibble; lane pairs merge nibbles into a byte. Otherwise byte loads + ballots.
template <bool VEC>
__device__ __forceinline__ void pack_estimate(const uint8_t* row, int n, int W, int lane,
                                              uint8_t* dst) {
  if constexpr (VEC) {
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(row);
    const int chunks = (n + 255) >> 8;
    for (int k = 0; k < chunks; ++k) {
      const int q = 256 * k + 4 * lane;
      const uint32_t x = q < n ? r32[q >> 2] : 0u;
      // bytes b0..b3 (0/1) -> bits 0..3: b_i at bit 8i moves to bit 24 + i
      uint32_t nib = ((x & 0x01010101u) * 0x01020408u) >> 24;
      nib <<= 4 * (lane & 1);
      nib |= __shfl_xor(nib, 1);
      if (!(lane & 1) && (q >> 3) < 8 * W) dst[q >> 3] = (uint8_t)nib;
    }
  } else {
    uint64_t mine = 0;
    for (int w = 0; w < W; ++w) {
      const int j = 64 * w + lane;
      const uint64_t bits = __ballot(j < n && (row[j < n ? j : 0] & 1));
      if (lane == w) mine = bits;
    }
    if (lane < W) reinterpret_cast<uint64_t*>(dst)[lane] = mine;
  }
}

template <int DC, bool VEC>
__global__ void __launch_bounds__(64 * kChannelWaves) count_outcomes_kernel(CountArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const PairTabs& t = a.t;
  const Tabs tb = stage_tables(t, smem);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int W = t.W, n = t.n;
  // columns of nonzero weight in Hz / Hx (the integer "degen" test)
  uint64_t* cmz = reinterpret_cast<uint64_t*>(tb.tail);
  uint64_t* cmx = cmz + W;
  unsigned long long* part = reinterpret_cast<unsigned long long*>(cmx + W);  // [waves][6]
  uint64_t* ex = reinterpret_cast<uint64_t*>(part + 6 * kChannelWaves) + wave * 2 * W;
  uint64_t* ez = ex + W;
  for (int i = threadIdx.x; i < 2 * W; i += blockDim.x) cmz[i] = 0;
  __syncthreads();
  for (int e = threadIdx.x; e < t.ez; e += blockDim.x) {
    const int j = t.ci_z[e];
    atomicOr(reinterpret_cast<unsigned long long*>(&cmz[j >> 6]), 1ull << (j & 63));
  }
  for (int e = threadIdx.x; e < t.ex; e += blockDim.x) {
    const int j = t.ci_x[e];
    atomicOr(reinterpret_cast<unsigned long long*>(&cmx[j >> 6]), 1ull << (j & 63));
  }
  __syncthreads();
  const uint64_t my_cmz = lane < W ? cmz[lane] : 0, my_cmx = lane < W ? cmx[lane] : 0;
  unsigned long long cnt[6] = {0, 0, 0, 0, 0, 0};
  for (long long b = (long long)blockIdx.x * kChannelWaves + wave; b < a.batch;
       b += (long long)gridDim.x * kChannelWaves) {
    // this shot's true errors and iteration counts: loads in flight early
    const uint64_t tx = lane < W ? a.errx[b * W + lane] : 0, tz = lane < W ? a.errz[b * W + lane] : 0;
    const int itx = a.itx[b], itz = a.itz[b];
    if (a.eh_bits) {                            // already words
      if (lane < W) {
        ex[lane] = reinterpret_cast<const uint64_t*>(a.ehx)[b * W + lane];
        ez[lane] = reinterpret_cast<const uint64_t*>(a.ehz)[b * W + lane];
      }
    } else {
      pack_estimate<VEC>(a.ehx + b * n, n, W, lane, reinterpret_cast<uint8_t*>(ex));
      pack_estimate<VEC>(a.ehz + b * n, n, W, lane, reinterpret_cast<uint8_t*>(ez));
    }
    wave_sync();
    bool lane_exact = true, lane_degen = true;
    if (lane < W) {
      const uint64_t dx = tx ^ ex[lane], dz = tz ^ ez[lane];
      lane_exact = (dx | dz) == 0;
      lane_degen = ((dx & my_cmz) | (dz & my_cmx)) == 0;
    }
    const bool exact = __ballot(!lane_exact) == 0;
    const bool degen = !exact && __ballot(!lane_degen) == 0;
    bool fx = false, fz = false;
    const uint32_t* ex32 = reinterpret_cast<const uint32_t*>(ex);
    const uint32_t* ez32 = reinterpret_cast<const uint32_t*>(ez);
    const int wmz = (t.mz + 63) >> 6, wmx = (t.mx + 63) >> 6;
    for (int c = lane; c < t.mz; c += 64) {
      const uint32_t s = a.syn_bits ? (uint32_t)(reinterpret_cast<const uint64_t*>(a.syz)[b * wmz + (c >> 6)] >> (c & 63)) & 1u
                                    : a.syz[b * t.mz + c];
      fx |= row_parity<DC>(tb.rpz, tb.ciz, c, ex32) != s;
    }
    for (int c = lane; c < t.mx; c += 64) {
      const uint32_t s = a.syn_bits ? (uint32_t)(reinterpret_cast<const uint64_t*>(a.syx)[b * wmx + (c >> 6)] >> (c & 63)) & 1u
                                    : a.syx[b * t.mx + c];
      fz |= row_parity<DC>(tb.rpx, tb.cix, c, ez32) != s;
    }
    const bool failx = __ballot(fx) != 0, failz = __ballot(fz) != 0;
    if (lane == 0) {
      cnt[0] += failx;
      cnt[1] += failz;
      cnt[2] += exact;
      cnt[3] += degen;
      cnt[4] += (unsigned long long)(long long)itx;
      cnt[5] += (unsigned long long)(long long)itz;
    }
    wave_sync();  // the next shot overwrites ex / ez
  }
  if (lane == 0)
    for (int k = 0; k < 6; ++k) part[wave * 6 + k] = cnt[k];
  __syncthreads();
  if (threadIdx.x < 6) {
    unsigned long long s = 0;
    for (int w = 0; w < kChannelWaves; ++w) s += part[w * 6 + threadIdx.x];
    if (s) atomicAdd(&a.acc[threadIdx.x], s);
  }
}

// common row degree of Hx and Hz if both are uniform with a specialised
// instantiation, else 0 (generic CSR loop)
int uniform_degree(const PairTabs& t) {
  return (t.udeg == 6 || t.udeg == 7 || t.udeg == 8) ? t.udeg : 0;
}

}  // namespace

int channel_lds_bytes(const PairTabs& t, bool counters) {
  int b = (4 * (t.mz + 1 + t.mx + 1) + 2 * (t.ez + t.ex) + 7) & ~7;
  if (counters) b += 8 * 2 * t.W + 8 * 6 * kChannelWaves;
  return b + kChannelWaves * 2 * t.W * 8;
}

template <typename K>
static hipError_t launch(K kernel, const void* args, size_t size, int grid, int lds, hipStream_t stream) {
  hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  void* params[] = {const_cast<void*>(args)};
  (void)size;
  return hipLaunchKernel((const void*)kernel, dim3(grid), dim3(64 * kChannelWaves), params, (size_t)lds,
                         stream);
}

hipError_t launch_channel_sample(const SampleArgs& a, int grid, hipStream_t stream) {
  const int lds = channel_lds_bytes(a.t, false);
  switch (uniform_degree(a.t)) {
    case 6: return launch(channel_sample_kernel<6>, &a, sizeof a, grid, lds, stream);
    case 7: return launch(channel_sample_kernel<7>, &a, sizeof a, grid, lds, stream);
    case 8: return launch(channel_sample_kernel<8>, &a, sizeof a, grid, lds, stream);
    default: return launch(channel_sample_kernel<0>, &a, sizeof a, grid, lds, stream);
  }
}

hipError_t launch_count_outcomes(const CountArgs& a, int grid, hipStream_t stream) {
  const int lds = channel_lds_bytes(a.t, true);
  // 32-bit estimate loads need every row 4-byte aligned (n % 4 == 0) and a
  // 4-byte aligned base
  const bool vec = (a.t.n % 4 == 0) && ((uintptr_t)a.ehx % 4 == 0) && ((uintptr_t)a.ehz % 4 == 0);
  switch (uniform_degree(a.t) * 2 + (vec ? 1 : 0)) {
    case 13: return launch(count_outcomes_kernel<6, true>, &a, sizeof a, grid, lds, stream);
    case 12: return launch(count_outcomes_kernel<6, false>, &a, sizeof a, grid, lds, stream);
    case 15: return launch(count_outcomes_kernel<7, true>, &a, sizeof a, grid, lds, stream);
    case 14: return launch(count_outcomes_kernel<7, false>, &a, sizeof a, grid, lds, stream);
    case 17: return launch(count_outcomes_kernel<8, true>, &a, sizeof a, grid, lds, stream);
    case 16: return launch(count_outcomes_kernel<8, false>, &a, sizeof a, grid, lds, stream);
    case 1: return launch(count_outcomes_kernel<0, true>, &a, sizeof a, grid, lds, stream);
    default: return launch(count_outcomes_kernel<0, false>, &a, sizeof a, grid, lds, stream);
  }
}

}  // namespace qldpc
