// decoder_kernels.hip — batched BP / normalized Min-Sum decoding on MI355X (gfx950).
//
// Replaces the per-shot message loops of albertogp71/qLDPCsim
//   MS_decoder  qLDPCsim/decoders.py:110-182
//   BP_decoder  qLDPCsim/decoders.py:189-290
// for a batch of syndromes (one "half-shot" = one decode of one syndrome).
//
// Execution model:
//  * One wavefront decodes one half-shot start to finish. All of its message
//    state lives in that wave's slice of LDS:
//        post  f64[n]          posterior LLR per variable  (decoders.py:173 / :276)
//        c2v   f32[E] (MS) or f64[E] (BP), stored in CSC (variable-major) order
//        syn / parity bit-words (layered schedule only)
//    so HBM traffic is the syndrome in (m B), ê out (n B), iterations/flags.
//  * The Tanner graph (CSR check->(var, csc position), CSC pointers, layer
//    lists) is one read-only blob staged into LDS once per workgroup.
//  * Check-node phase: lane owns whole checks; min1/min2/first-argmin/sign
//    product (MS) or the tanh product (BP) are folded in-lane over the
//    check's edges in ascending variable order — no cross-lane traffic.
//  * Variable-node phase: lane owns whole variables; the column sum runs over
//    the contiguous CSC segment in ascending check order — the exact order of
//    NumPy's axis-0 reduction (MS, float32) or np.sum's pairwise rule (BP).
//  * Persistent: each wave strides over half-shots; the grid is sized to the
//    occupancy the LDS budget allows (host side, capi.cpp).
//
// Numerics: MS c2v = fl32(beta * min) formed in float64;
// VN sum float32 sequential; posterior and v2c float64; first layer of the
// first iteration sees float32(L). BP float64; tanh/atanh from
// include/qldpc_libm.h (basic IEEE ops only: identical on GPU and CPU oracle).
// Compiled with -ffp-contract=off: no FMA contraction may change a rounding.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "decoder_kernels.h"
#include "tuning.h"
#include "kargs.h"
#include "../../include/qldpc_libm.h"

namespace qldpc {

// NumPy's tanh / SVML's atanh tables (include/qldpc_libm.h). BP kernels copy
// this image into LDS (DecodeArgs::off_libm) once per workgroup: the lookups
// are per lane (data-dependent intervals), 10-13 per edge and iteration.
static __constant__ qldpc_libm_tab qldpc_libm_dev = QLDPC_LIBM_TAB_INIT;   // one per translation unit

__device__ __forceinline__ const qldpc_libm_tab* stage_libm(unsigned char* lds, int off) {
  const uint4* src = (const uint4*)&qldpc_libm_dev;
  uint4* dst = (uint4*)(lds + off);
  for (int i = threadIdx.x; i < (int)(sizeof(qldpc_libm_tab) / 16); i += blockDim.x) dst[i] = src[i];
  return (const qldpc_libm_tab*)(lds + off);
}

__device__ __forceinline__ void wave_sync() {
  // Lanes of one wave exchange data through LDS between phases. DS
  // instructions of a wave complete in order; the fences only stop the
  // compiler from moving LDS accesses across the phase boundary.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t ballot(int pred) { return __ballot(pred); }
// the same from a bool: the wave's compare mask itself (s_and with exec). The
// int form above materialises the predicate (v_cndmask) and compares it again
// (v_cmp_ne) — two VALU ops per ballot, kept where the code is profiled as is.
__device__ __forceinline__ uint64_t ballot_b(bool pred) { return __builtin_amdgcn_ballot_w64(pred); }

__device__ __forceinline__ const DecodeArgs& kargs_fresh() { return kargs_fresh<DecodeArgs>(); }

// LDS (address space 3) access through a 32-bit byte address held in a VGPR
// (ds_read / ds_write directly; a generic pointer would become flat_load).
#define QLDPC_LDS(T, addr) ((__attribute__((address_space(3))) T*)(uintptr_t)(uint32_t)(addr))
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
}

// NumPy DOUBLE_pairwise_sum over a contiguous LDS segment (np.sum of a 1-D
// float64 array = 0.0 + pairwise(all); decoders.py:269, :276). n <= 128.
__device__ __forceinline__ double np_pairwise_sum(const double* a, int n) {
  if (n < 8) {
    double res = -0.0;
    for (int i = 0; i < n; ++i) res += a[i];
    return 0.0 + res;
  }
  double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
  int i = 8;
  const int nb = n - (n % 8);
  for (; i < nb; i += 8) {
    r0 += a[i + 0]; r1 += a[i + 1]; r2 += a[i + 2]; r3 += a[i + 3];
    r4 += a[i + 4]; r5 += a[i + 5]; r6 += a[i + 6]; r7 += a[i + 7];
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[i];
  return 0.0 + res;
}

// np_pairwise_sum of a BP column (variable node, decoders.py:276): below 8
// terms NumPy adds sequentially from -0.0, so with K >= n terms loaded at
// once (the c2v region is padded by 8 entries) and the terms past n replaced
// by -0.0 — x + -0.0 == x for every x, -0.0 included — the sum is the same
// bit for bit, without a load-wait-add chain per term. K is wave-uniform:
// the smallest of 3 / 5 / 7 covering every active lane's n (ballots); a wave
// holding a column of 8 or more terms takes the general pairwise sum.
template <int K>
__device__ __forceinline__ double np_sum_lt8(const double* a, int n) {
  double x[K];
#pragma unroll
  for (int t = 0; t < K; ++t) x[t] = a[t];
  double res = -0.0;
#pragma unroll
  for (int t = 0; t < K; ++t) res += (t < n) ? x[t] : -0.0;
  return 0.0 + res;
}

// The same when every active lane's n >= 3 (round 6): -0.0 + x0 == x0 for
// every x0, so the sum starts at x0; prefix sums over all K terms, and n
// picks one of the last K - 2 (a compare and a 64-bit select each) instead of
// a compare and select per term — the same float64 additions on the first n
// terms, the same bits
template <int K>
__device__ __forceinline__ double np_sum_lt8_lo3(const double* a, int n) {
  double x[K];
#pragma unroll
  for (int t = 0; t < K; ++t) x[t] = a[t];
  double pre = x[0];
#pragma unroll
  for (int t = 1; t < 3; ++t) pre += x[t];
  double res = pre;                                        // n = 3
#pragma unroll
  for (int t = 3; t < K; ++t) {
    pre += x[t];                                           // (terms past n: discarded below)
    res = n > t ? pre : res;
  }
  return 0.0 + res;
}

// LO3: try the n >= 3 form first (the layered team kernel: -0.7 % per LP118_2
// p = 0.1 launch; the flooding kernel's extra ballot cost +0.7 %, so it keeps
// the plain form, profiles/r06/r06d_ab_msnew_main.json)
template <bool LO3 = false>
__device__ __forceinline__ double np_sum_col(const double* a, int n) {
  if (__builtin_expect(ballot_b(n >= 8) != 0, 0)) return np_pairwise_sum(a, n);
  if (LO3 && ballot_b(n < 3) == 0) {
    if (ballot_b(n > 3) == 0) return np_sum_lt8_lo3<3>(a, n);
    if (ballot_b(n > 5) == 0) return np_sum_lt8_lo3<5>(a, n);
    return np_sum_lt8_lo3<7>(a, n);
  }
  if (ballot_b(n > 3) == 0) return np_sum_lt8<3>(a, n);
  if (ballot_b(n > 5) == 0) return np_sum_lt8<5>(a, n);
  return np_sum_lt8<7>(a, n);
}

// Set bit `c` of a per-wave bit-word array for every lane whose predicate is
// true, for a chunk of 64 consecutive indices starting at c0 (all lanes call).
__device__ __forceinline__ void store_bits64(uint32_t* words, int c0, int pred, int lane) {
  const uint64_t b = ballot(pred);
  if (lane == 0) words[c0 >> 5] = (uint32_t)b;
  if (lane == 1) words[(c0 >> 5) + 1] = (uint32_t)(b >> 32);
}

// Bit-packed I/O (DecodeArgs::syn_bits / eh_bits): syndromes and hard
// decisions as 64-bit words, bit j % 64 of word j / 64 (the error-vector
// layout of the device sampler), instead of one byte per bit.
__device__ __forceinline__ uint32_t syn_bit(const DecodeArgs& a, long long hs, int c) {
  if (a.syn_bits) return (uint32_t)(((const uint64_t*)a.syn)[hs * a.wm + (c >> 6)] >> (c & 63)) & 1u;
  return a.syn[hs * (long long)a.m + c] & 1u;
}
// ê_jo of half-shot hs. Callers visit columns in 64-aligned wave chunks
// (lane l holds column 64 k + l), so with eh_bits the chunk is one ballot and
// lane 0 stores the word.
__device__ __forceinline__ void put_ehat(const DecodeArgs& a, long long hs, int jo, bool bit) {
  if (a.eh_bits) {
    const uint64_t b = ballot(bit);
    if ((jo & 63) == 0) ((uint64_t*)a.ehat)[hs * a.wn + (jo >> 6)] = b;
  } else {
    a.ehat[hs * (long long)a.n + jo] = (uint8_t)bit;
  }
}

// Read-only kernel inputs through the constant address space: with a
// wave-uniform index the compiler issues scalar loads (through a generic
// pointer it must assume the kernel's own stores alias them).
template <typename T>
__device__ __forceinline__ T ld_const(const T* p, long long i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// Syndrome bits of checks lane + 64 i (i < KC) of half-shot hs as bit i of
// the result, every load issued before the first use: bit-packed rows are
// KC wave-uniform words (scalar loads), byte rows KC per-lane loads at
// clamped addresses (a guard around each load made the compiler wait after
// each one).
template <int KC>
__device__ __forceinline__ uint32_t syn_lane_bits(const DecodeArgs& a, long long hs, int lane) {
  const int m = a.m;
  uint32_t r = 0;
  if (a.syn_bits) {
    const uint64_t* row = (const uint64_t*)a.syn + hs * a.wm;
    uint64_t w[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) w[i] = ld_const(row, i < a.wm ? i : a.wm - 1);
#pragma unroll
    for (int i = 0; i < KC; ++i) {                  // (32-bit halves: no 64-bit VGPR shifts)
      const uint32_t h = lane < 32 ? (uint32_t)w[i] : (uint32_t)(w[i] >> 32);
      r |= (((h >> (lane & 31)) & 1u) & (uint32_t)(lane + 64 * i < m)) << i;
    }
  } else {
    const uint8_t* row = a.syn + hs * (long long)m;
    // (opaque lane: the clamped offsets are cheap to form here; hoisted out of
    // the half-shot loop as invariants they cost VGPRs the decode loop needs)
    uint32_t ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    uint32_t b[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) b[i] = row[(int)ln + 64 * i < m ? (int)ln + 64 * i : m - 1];
#pragma unroll
    for (int i = 0; i < KC; ++i) r |= ((b[i] & 1u) & (uint32_t)(lane + 64 * i < m)) << i;
  }
  return r;
}

// ê (and posteriors) of one half-shot: original column jo = ST k + t takes
// post_of(vinv[jo]) (the relabeled variable's posterior); ST = 64 with t the
// lane (one wave per half-shot) or the team size with t the thread index (a
// wave's columns stay one aligned 64-column chunk). Chunks of OC trips: the
// OC vinv loads, then the OC posterior reads, then the outputs — one round
// trip per stage instead of one per trip (a guarded load per trip made the
// compiler wait after each one).
template <int OC, int ST, typename Post>
__device__ __forceinline__ void write_outputs_strided(const DecodeArgs& a, long long hs, int t, Post post_of) {
  const int n = a.n;
  const int cb = t & ~63;                            // this wave's chunk offset within a trip
  double* po = a.post ? a.post + hs * (long long)n : nullptr;
  for (int k0 = 0; ST * k0 < n; k0 += OC) {
    int v[OC];
#pragma unroll
    for (int u = 0; u < OC; ++u) {
      const int jo = ST * (k0 + u) + t;
      v[u] = a.vinv[jo < n ? jo : n - 1];
    }
    double pv[OC];
#pragma unroll
    for (int u = 0; u < OC; ++u) pv[u] = post_of(v[u]);
#pragma unroll
    for (int u = 0; u < OC; ++u) {
      const int jo = ST * (k0 + u) + t;
      if (ST * (k0 + u) + cb < n) {                  // (wave-uniform; columns past n ballot 0)
        if (a.eh_bits) {
          put_ehat(a, hs, jo, jo < n && pv[u] < 0.0);
        } else if (jo < n) {
          put_ehat(a, hs, jo, pv[u] < 0.0);
        }
        if (po && jo < n) po[jo] = pv[u];
      }
    }
  }
}
template <int OC, typename Post>
__device__ __forceinline__ void write_outputs_batched(const DecodeArgs& a, long long hs, int lane, Post post_of) {
  write_outputs_strided<OC, 64>(a, hs, lane, post_of);
}

// syndrome bits of one half-shot into a team's word array: thread t covers
// checks ST k + t, NT trips with their loads in flight together
template <int NT, int ST>
__device__ __forceinline__ void team_syndrome_bits(const DecodeArgs& a, long long hs, uint32_t* synw, int t) {
  const int m = a.m, lane = t & 63, cb = t & ~63;
  for (int k0 = 0; ST * k0 < m; k0 += NT) {
    uint32_t b[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int c = ST * (k0 + u) + t;
      b[u] = syn_bit(a, hs, c < m ? c : m - 1);
    }
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int c0 = ST * (k0 + u) + cb;
      if (c0 < m) store_bits64(synw, c0, (c0 + lane < m) ? (int)b[u] : 0, lane);
    }
  }
}

// Half-shot prologue / epilogue with every global load issued up front (a
// loop of dependent load -> use steps paid one HBM latency per 64 elements).
// The relabeling vinv is per code, so it is read once per kernel into
// registers: VinvRegs holds original column 64k + lane's variable for k < NJ
// (two 16-bit entries per VGPR); n > 64 NJ falls back to global reads.
template <int NJ>
struct VinvRegs {
  uint32_t w[(NJ + 1) / 2];
  __device__ __forceinline__ void load(const uint16_t* vinv, int n, int lane) {
#pragma unroll
    for (int k = 0; k < NJ; k += 2) {
      const int j0 = 64 * k + lane, j1 = j0 + 64;
      const uint32_t v0 = j0 < n ? vinv[j0] : 0u, v1 = j1 < n ? vinv[j1] : 0u;
      w[k / 2] = v0 | (v1 << 16);
    }
  }
  __device__ __forceinline__ int get(int k) const { return (int)((w[k / 2] >> (16 * (k & 1))) & 0xffffu); }
};

// ê (and posteriors) of one half-shot in original column order
template <int NJ>
__device__ __forceinline__ void write_outputs(const DecodeArgs& a, const VinvRegs<NJ>& vr, const double* post,
                                              long long hs, int lane) {
  const int n = a.n;
  double* po = a.post ? a.post + hs * (long long)n : nullptr;
  if (n <= 64 * NJ) {
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const int jo = 64 * k + lane;
      if (64 * k < n && jo < n) {
        const double pv = post[vr.get(k)];
        put_ehat(a, hs, jo, pv < 0.0);
        if (po) po[jo] = pv;
      }
    }
  } else {
    for (int jo = lane; jo < n; jo += 64) {
      const double pv = post[a.vinv[jo]];
      put_ehat(a, hs, jo, pv < 0.0);
      if (po) po[jo] = pv;
    }
  }
}

// syndrome bits of one half-shot into the per-wave word array (m <= 64 NC:
// all byte loads in flight together; larger m loops)
template <int NC>
__device__ __forceinline__ void load_syndrome_bits(const DecodeArgs& a, long long hs, uint32_t* synw, int lane) {
  const int m = a.m;
  if (a.syn_bits) {                                 // already words: copy them
    const uint32_t* src = (const uint32_t*)((const uint64_t*)a.syn + hs * a.wm);
    for (int w = lane; w < 2 * a.wm; w += 64) synw[w] = src[w];
    return;
  }
  const uint8_t* syn = a.syn + hs * (long long)m;
  if (m <= 64 * NC) {
    // every load at a clamped address (a guarded load per chunk made the
    // compiler wait after each one); the opaque lane keeps the offsets from
    // being hoisted out of the half-shot loop into VGPRs
    uint32_t ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    uint32_t b[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = 64 * k + (int)ln;
      b[k] = syn[c < m ? c : m - 1];
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) b[k] = (64 * k + lane < m) ? (b[k] & 1u) : 0u;
#pragma unroll
    for (int k = 0; k < NC; ++k)
      if (64 * k < m) store_bits64(synw, 64 * k, (int)b[k], lane);
  } else {
    for (int c0 = 0; c0 < m; c0 += 64) {
      const int c = c0 + lane;
      store_bits64(synw, c0, c < m ? (syn[c] & 1) : 0, lane);
    }
  }
}

// Persistent half-shot loop. Each wave starts with one static half-shot;
// with a queue, further work comes from a global ticket counter in guided
// chunks (about remaining / (4 * waves) consecutive half-shots, at most 64,
// at least 1), claimed with one atomic when the last half-shot of the current
// chunk starts, so its latency is hidden. Early-terminating decodes (channel
// syndromes: most stop after 1-3 iterations, a few run max_iter) then
// balance across waves instead of leaving a long tail, and the counter sees
// O(waves * log) atomics rather than one per half-shot.
// A wave-uniform 64-bit value the compiler may not prove uniform: pinning it
// to scalar registers keeps the queue state out of VGPRs (the headline kernel
// had spilled it to scratch memory at its 168-VGPR budget).
__device__ __forceinline__ long long uniform64(long long x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (long long)(((uint64_t)hi << 32) | lo);
}

struct HalfShotQueue {
  long long hs, end, stride, batch;
  uint32_t* q;
  uint32_t tk, tlen, seen;
  __device__ __forceinline__ HalfShotQueue(const DecodeArgs& a, int waves, int wid)
      : hs(uniform64((long long)blockIdx.x * waves + wid)), end(0), stride((long long)gridDim.x * waves),
        batch(a.batch), q(a.queue), tk(0), tlen(1), seen(0) {
    end = hs + 1;
  }
  __device__ __forceinline__ void prefetch(int lane) {
    if (q && hs + 1 == end) {                       // last of this chunk: claim the next
      const long long rem = batch - stride - (long long)seen;
      long long len = rem / (4 * stride);
      len = len < 1 ? 1 : (len > 64 ? 64 : len);
      tlen = (uint32_t)len;
      if (lane == 0) tk = atomicAdd(q, tlen);
    }
  }
  __device__ __forceinline__ void advance() {
    if (!q) {
      hs = uniform64(hs + stride);
      return;
    }
    hs = uniform64(hs + 1);
    if (hs < end) return;
    const uint32_t t = __builtin_amdgcn_readfirstlane(tk);
    seen = t + tlen;
    hs = uniform64(stride + (long long)t);
    end = uniform64(hs + tlen);
  }
};

struct LdsView {
  const uint32_t* cn_tab;   // [E] (relabeled var << 16) | csc position, CSR edge order
  const uint16_t* row_ptr;  // [m+1]
  const uint32_t* vn_info;  // [n]   csc start | degree << 16
  const uint8_t* chunk_dmax; // [ceil(n/64)] max degree of relabeled variables 64c..64c+63
  const uint16_t* vn_chk;   // [E]   check of each CSC position (layered)
  const uint16_t* lay_ptr;  // [L+1]
  const uint16_t* lay_rows; // [*]
  const uint16_t* adj_ptr;  // [L+1]
  const uint16_t* adj_vars; // [*]
  const qldpc_libm_tab* lt; // BP: NumPy libm tables (LDS)
};

// Graph table entry formats (capi.cpp builds them):
//  DC == 0 (generic):   cn_tab[row_ptr[c] + k] = (relabeled var << 16) | csc position
//  DC  > 0 (uniform row degree DC, rows padded to 8 entries, 16-byte aligned):
//                       cn_tab[8c + k] = (4 * csc position) << 16 | (8 * relabeled var)
//                       i.e. ready-made LDS byte offsets into c2v (f32) and post (f64).
template <int DC>
__device__ __forceinline__ int tab_var(uint32_t t) { return DC ? (int)((t & 0xffffu) >> 3) : (int)(t >> 16); }
template <int DC>
__device__ __forceinline__ int tab_pos(uint32_t t) { return DC ? (int)(t >> 18) : (int)(t & 0xffffu); }

// Hide a register value's provenance from the optimizer, so that values
// derived from it are not re-derived (or hoisted) where that costs VALU or VGPRs.
__device__ __forceinline__ uint32_t opaque_always(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

// v_min_f64 / v_max_f64 without the canonicalizes LLVM adds around
// minnum/maxnum (operands here are never signalling NaNs).
__device__ __forceinline__ double vmin_f64(double x, double y) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ double vmin_abs_f64(double x, double y) {  // min(|x|, y)
  double r;
  asm("v_min_f64 %0, |%1|, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ double vmax_abs_f64(double x, double y) {  // max(|x|, y)
  double r;
  asm("v_max_f64 %0, |%1|, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}

__device__ __forceinline__ double vmin_abs2_f64(double x, double y) {  // min(|x|, |y|)
  double r;
  asm("v_min_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ double vmax_abs2_f64(double x, double y) {  // max(|x|, |y|)
  double r;
  asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ double vmax_f64(double x, double y) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}

// Smallest and second smallest (with multiplicity) of |v[0..N)| as a
// tournament: pairs, then merges (l1,h1)+(l2,h2) -> (min(l1,l2),
// min(max(l1,l2), min(h1,h2))). Depth ~log2 N instead of a serial chain
// (the check-node step is latency-bound), and fewer ops than the chain.
template <int N>
__device__ __forceinline__ void min12_tree(const double* v, double& lo, double& hi) {
  if constexpr (N == 1) {
    lo = __builtin_fabs(v[0]);
    hi = __builtin_inf();
  } else if constexpr (N == 2) {
    lo = vmin_abs2_f64(v[0], v[1]);
    hi = vmax_abs2_f64(v[0], v[1]);
  } else {
    constexpr int H = (N / 2 + 1) & ~1;   // even split: 3->2+1, 5->2+3, 6->4+2, 7->4+3, 8->4+4
    double l1, h1, l2, h2;
    min12_tree<(H < N ? H : N - 1)>(v, l1, h1);
    min12_tree<N - (H < N ? H : N - 1)>(v + (H < N ? H : N - 1), l2, h2);
    lo = vmin_f64(l1, l2);
    hi = vmin_f64(vmax_f64(l1, l2), vmin_f64(h1, h2));
  }
}

// XOR of N words as a balanced tree (v_xor3_b32-friendly)
__device__ __forceinline__ uint32_t xor3(uint32_t x, uint32_t y, uint32_t z) {
  uint32_t r;
  // gfx950 has no v_xor3_b32; v_bitop3_b32 truth table 0x96 = S0 ^ S1 ^ S2
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}
template <int N>
__device__ __forceinline__ uint32_t xor_tree(const uint32_t* w) {
  if constexpr (N == 1) return w[0];
  else if constexpr (N == 2) return w[0] ^ w[1];
  else if constexpr (N == 3) return xor3(w[0], w[1], w[2]);
  else if constexpr (N == 4) return xor3(w[0], w[1], w[2]) ^ w[3];
  else if constexpr (N == 5) return xor3(xor3(w[0], w[1], w[2]), w[3], w[4]);
  else return xor3(xor_tree<N - 2>(w), w[N - 2], w[N - 1]);
}

__device__ __forceinline__ uint32_t hi_word(double d) { return (uint32_t)(__builtin_bit_cast(uint64_t, d) >> 32); }

// ---------------------------------------------------------------------------
// Min-sum check-node update for a uniform-degree code (DC = 7 or 8), the hot
// loop of the headline workload (decoders.py:155-169 for one row):
//   v_e   = post_j - c2v_e  (float64; FIRST: float32(L), :148-149)
//   min1 / first argmin / min2 of |v_e|, sign product with the syndrome sign
//   c2v_e = fl32(beta * (e == argmin ? min2 : min1)) with sign syn*prod*sign_e
// Signs and the parity of the hard decisions are folded from the high words
// (v_e is never -0.0 and post never -0.0 or NaN for finite L: DESIGN.md §4).
// Returns the check's "unsatisfied" bit for the posteriors it read.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_row8(const uint32_t* tab, uint32_t (&t)[8]) {
  const uint4 t0 = *(const uint4*)tab;
  const uint4 t1 = *(const uint4*)(tab + 4);
  t[0] = t0.x; t[1] = t0.y; t[2] = t0.z; t[3] = t0.w;
  t[4] = t1.x; t[5] = t1.y; t[6] = t1.z; t[7] = t1.w;
}

// Min-sum check-node update of one uniform-degree check (decoders.py:155-169)
// whose edges are given as absolute LDS byte addresses (pa: post f64, ca: c2v
// f32). `live` = 0 for a pad check (its writes land in the pad; flags masked).
template <int DC>
struct CnLoad {
  double pj[DC];
  float cv[DC];
};

template <int DC>
__device__ __forceinline__ void cn_ms_load(CnLoad<DC>& L, const uint32_t* pa, const uint32_t* ca) {
#pragma unroll
  for (int k = 0; k < DC; ++k) {
    L.pj[k] = *QLDPC_LDS(const double, pa[k]);
    L.cv[k] = *QLDPC_LDS(const float, ca[k]);
  }
}

template <int DC>
__device__ __forceinline__ uint32_t cn_ms_compute(const DecodeArgs& a, const CnLoad<DC>& L, const uint32_t* ca,
                                                  uint32_t synb, uint32_t live, int& fl) {
  double v[DC];
  uint32_t hv[DC], hp[DC];
#pragma unroll
  for (int k = 0; k < DC; ++k) {
    v[k] = L.pj[k] - (double)L.cv[k];                     // v2c = post - c2v (:177)
    hv[k] = hi_word(v[k]);
    hp[k] = hi_word(L.pj[k]);
  }
  double min1, min2;                                      // first min / min of the rest (:160-164)
  min12_tree<DC>(v, min1, min2);
  const uint32_t ph = xor_tree<DC>(hp);                   // hard-decision parity (:174)
  const uint32_t sh = xor_tree<DC>(hv);                   // np.sign product (:157-159)
  double m1 = min1, m2 = min2;
  // Rare cases behind one wave-uniform test: an infinite min (min2 = inf
  // whenever min1 is) and a zero min (min1 = 0, App. A.1.6 leak case, flagged).
  if (__builtin_expect(ballot((min1 == 0.0) | (min2 == __builtin_inf())) != 0, 0)) {
    m1 = __builtin_isinf(min1) ? 0.0 : min1;              // (:165)
    m2 = __builtin_isinf(min2) ? 0.0 : min2;              // (:166)
    if (m1 == 0.0 && live) fl |= FLAG_MIN_ZERO;
  }
  const uint32_t npm = ((sh >> 31) ^ synb) << 31;
  // c2v_e = fl32(beta * (|v_e| == min1 ? min2 : min1)), sign syn * prod *
  // sign_e (:167-168). The reference gives min2 to the first argmin only;
  // "every edge equal to min1" is the same thing: with a tie min2 == min1.
  const uint32_t c1n = opaque_always(__builtin_bit_cast(uint32_t, (float)(a.beta * m1)) ^ npm);
  const uint32_t c2n = opaque_always(__builtin_bit_cast(uint32_t, (float)(a.beta * m2)) ^ npm);
#pragma unroll
  for (int k = 0; k < DC; ++k) {
    const uint32_t c = (__builtin_fabs(v[k]) == min1) ? c2n : c1n;
    *QLDPC_LDS(uint32_t, ca[k]) = c ^ (hv[k] & 0x80000000u);
  }
  return ((ph >> 31) ^ synb) & live;
}

template <int DC>
__device__ __forceinline__ uint32_t cn_ms_abs(const DecodeArgs& a, const uint32_t* pa, const uint32_t* ca,
                                              uint32_t synb, uint32_t live, int& fl) {
  CnLoad<DC> L;
  cn_ms_load<DC>(L, pa, ca);
  return cn_ms_compute<DC>(a, L, ca, synb, live, fl);
}

// NC independent checks per call: every LDS read of all NC checks is issued
// before any arithmetic. `t[q]` holds check q's 8 table words (registers).
template <int DC, bool FIRST, int NC>
__device__ __forceinline__ uint32_t cn_ms_uniform(const DecodeArgs& a, const uint32_t (*t)[8],
                                                  const uint32_t* synb, const bool* live,
                                                  const unsigned char* post_b,
                                                  unsigned char* c2v_b, int& fl) {
  static_assert(DC >= 2 && DC <= 8, "uniform fast path handles row degrees 2..8");
  if constexpr (FIRST) {
    // every v_e = float32(L): min1 = min2 = |L32|, argmin 0, sign_e = L32 < 0
    const double vf = (double)a.L32;
    const double av = __builtin_fabs(vf);
    const float c = (float)(a.beta * av);
    const uint32_t neg = (uint32_t)(vf < 0.0);
    if (av == 0.0) fl |= FLAG_MIN_ZERO;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const uint32_t negprod = ((neg * DC) ^ synb[q]) & 1u;
      const float val = (neg ^ negprod) ? -c : c;
      if (live[q]) {
#pragma unroll
        for (int k = 0; k < DC; ++k) *(float*)(c2v_b + (t[q][k] >> 16)) = val;
      }
    }
    return 0;
  } else {
    // the flooding kernel's check node (cn_ms_load / cn_ms_compute) on
    // addresses formed from the packed table words
    uint32_t unsat = 0;
    const uint32_t pb = lds_addr(post_b), cb = lds_addr(c2v_b);
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      uint32_t pa[8], ca[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        pa[k] = pb + (t[q][k] & 0xffffu);
        ca[k] = cb + (t[q][k] >> 16);
      }
      if (live[q]) {
        CnLoad<DC> L;
        cn_ms_load<DC>(L, pa, ca);
        unsat |= cn_ms_compute<DC>(a, L, ca, synb[q], 1u, fl);
      }
    }
    return unsat;
  }
}

// Check-node update of one check `c` (lane-local), any degree.
//   MS: decoders.py:155-169.  BP: decoders.py:249-262.
// Returns the check's current parity XOR syndrome bit ("unsatisfied"),
// computed from the hard decisions of the posteriors it reads (only
// meaningful when !first).
// ---------------------------------------------------------------------------
template <int ALGO, int DC>
__device__ __forceinline__ uint32_t cn_update(const DecodeArgs& a, const LdsView& g, int c,
                                              uint32_t synb, bool first, const double* post,
                                              void* c2v_raw, int& fl) {
  if constexpr (ALGO == ALGO_MS && DC > 0) {
    uint32_t t[1][8];
    load_row8(g.cn_tab + c * 8, t[0]);
    const uint32_t sb[1] = {synb};
    const bool live[1] = {true};
    if (first) return cn_ms_uniform<DC, true, 1>(a, t, sb, live, (const unsigned char*)post, (unsigned char*)c2v_raw, fl);
    return cn_ms_uniform<DC, false, 1>(a, t, sb, live, (const unsigned char*)post, (unsigned char*)c2v_raw, fl);
  }
  const int e0 = DC ? c * 8 : (int)g.row_ptr[c];
  const int deg = DC ? DC : (int)g.row_ptr[c + 1] - e0;
  uint32_t par = 0;
  if constexpr (ALGO == ALGO_MS) {
    float* c2v = (float*)c2v_raw;
    double min1 = __builtin_inf(), min2 = __builtin_inf();
    int idx = 0;
    uint32_t negm = 0;
    const double vfirst = (double)a.L32;
    for (int k = 0; k < deg; ++k) {
      const uint32_t t = g.cn_tab[e0 + k];
      const int j = tab_var<DC>(t), pos = tab_pos<DC>(t);
      double v;
      if (first) {
        v = vfirst;                                   // float32(L) (:148-149)
      } else {
        const double pj = post[j];
        par ^= (uint32_t)(pj < 0.0);                  // hard decision (:174)
        v = pj - (double)c2v[pos];                    // v2c = post - c2v (:177)
      }
      negm |= (uint32_t)(v < 0.0) << k;              // np.sign, 0 -> +1 (:157-158)
      const double av = __builtin_fabs(v);
      idx = (av < min1) ? k : idx;                   // first argmin (:161)
      min2 = __builtin_fmin(min2, __builtin_fmax(min1, av));  // min of the rest (:162-164)
      min1 = __builtin_fmin(min1, av);
    }
    if (deg == 0) return synb;                       // no edges: c2v stays 0
    if (__builtin_isinf(min1)) min1 = 0.0;           // (:165)
    if (__builtin_isinf(min2)) min2 = 0.0;           // (:166)
    if (min1 == 0.0) fl |= FLAG_MIN_ZERO;            // App. A.1.6 leak case (flagged, not emulated)
    const uint32_t negprod = (uint32_t)(__builtin_popcount(negm) & 1) ^ synb;
    // c2v_e = fl32(beta * syn * prod * min_e / sign_e): magnitude rounded from
    // the float64 product once, sign = syn * prod * sign_e (:167-168).
    const float c1 = (float)(a.beta * min1), c2 = (float)(a.beta * min2);
    for (int k = 0; k < deg; ++k) {
      const int pos = tab_pos<DC>(g.cn_tab[e0 + k]);
      const float mag = (k == idx) ? c2 : c1;
      c2v[pos] = (((negm >> k) & 1u) ^ negprod) ? -mag : mag;
    }
  } else {
    double* c2v = (double*)c2v_raw;
    if (deg == 0) return synb;                       // `continue` (:251-252)
    double prod = 1.0;
#pragma unroll
    for (int k = 0; k < (DC ? DC : 32); ++k) {
      if (!DC && k >= deg) break;
      const uint32_t t = g.cn_tab[e0 + k];
      const int j = tab_var<DC>(t), pos = tab_pos<DC>(t);
      const double pj = post[j];
      par ^= (uint32_t)(pj < 0.0);
      const double v = pj - c2v[pos];                // v2c (:269)
      const double th = qldpc_tanh_t(v / 2.0, g.lt->tanh_c);   // (:254) np.tanh
      prod *= th;                                    // np.prod: sequential fold
      c2v[pos] = th;                                 // scratch: own edge, rewritten below
    }
    if (!DC && deg > 32) {
      // generic degrees > 32: second half of the fold (rare; bicycle = 18)
      for (int k = 32; k < deg; ++k) {
        const uint32_t t = g.cn_tab[e0 + k];
        const int j = tab_var<DC>(t), pos = tab_pos<DC>(t);
        const double pj = post[j];
        par ^= (uint32_t)(pj < 0.0);
        const double th = qldpc_tanh_t((pj - c2v[pos]) / 2.0, g.lt->tanh_c);
        prod *= th;
        c2v[pos] = th;
      }
    }
    const double lim = 1.0 - a.eps;
    for (int k = 0; k < deg; ++k) {
      const int pos = tab_pos<DC>(g.cn_tab[e0 + k]);
      const double th = c2v[pos];
      if (th == 0.0) fl |= FLAG_NONFINITE;
      double th2 = prod / th;                        // (:256)
      if (__builtin_fabs(th2) >= lim)                // (:257-258)
        th2 = th2 - a.eps * (th2 > 0.0 ? 1.0 : (th2 < 0.0 ? -1.0 : 0.0));
      double val = 2.0 * qldpc_atanh_t(th2, g.lt->atanh_hl, g.lt->atanh_rcp);   // (:259) np.arctanh
      if (synb) val = -val;                          // (:260-261)
      if (!__builtin_isfinite(val)) fl |= FLAG_NONFINITE;
      c2v[pos] = val;
    }
  }
  return par ^ synb;
}

// Variable-node update of relabeled variable j: column sum in ascending check
// order. MS: float32 sequential (np.sum axis=0, decoders.py:172), post = L +
// (f64)S (:173). BP: np.sum pairwise rule, post = L0 + S (:269, :276).
// vn_info[j] = csc start | degree << 16.
template <int K>
__device__ __forceinline__ float ms_colsum(const float* c, int d) {
  // K unconditional loads (the c2v region is padded by 8 floats, so reading
  // past a short column stays inside this wave's slice), then the sequential
  // sum with the missing terms replaced by +0.0f — exact, since the running
  // sum starts at +0.0f and is never -0.0f.
  float x[K];
#pragma unroll
  for (int t = 0; t < K; ++t) x[t] = c[t];
  float s = 0.0f;
#pragma unroll
  for (int t = 0; t < K; ++t) s += (t < d) ? x[t] : 0.0f;
  return s;
}

// VN column sum with a wave-uniform degree bound dmax (unrolled loads).
__device__ __forceinline__ float ms_colsum_sw(const float* c, int d, int dmax) {
  switch (dmax) {
    case 0: return 0.0f;
    case 1: return ms_colsum<1>(c, d);
    case 2: return ms_colsum<2>(c, d);
    case 3: return ms_colsum<3>(c, d);
    case 4: return ms_colsum<4>(c, d);
    case 5: return ms_colsum<5>(c, d);
    case 6: return ms_colsum<6>(c, d);
    case 7: return ms_colsum<7>(c, d);
    case 8: return ms_colsum<8>(c, d);
    default: {
      float s = 0.0f;
      for (int t = 0; t < d; ++t) s += c[t];
      return s;
    }
  }
}

// dmax: wave-uniform upper bound of the degrees of the variables this pass
// covers (per 64-variable chunk, from the host), so the loads are unrolled.
template <int ALGO>
__device__ __forceinline__ double vn_post(const DecodeArgs& a, const LdsView& g, int j,
                                          const void* c2v_raw, int dmax) {
  const uint32_t info = g.vn_info[j];
  const int p0 = (int)(info & 0xffffu), d = (int)(info >> 16);
  if constexpr (ALGO == ALGO_MS) {
    const float* c = (const float*)c2v_raw + p0;
    float s;
    switch (dmax) {
      case 0: s = 0.0f; break;
      case 1: s = ms_colsum<1>(c, d); break;
      case 2: s = ms_colsum<2>(c, d); break;
      case 3: s = ms_colsum<3>(c, d); break;
      case 4: s = ms_colsum<4>(c, d); break;
      case 5: s = ms_colsum<5>(c, d); break;
      case 6: s = ms_colsum<6>(c, d); break;
      case 7: s = ms_colsum<7>(c, d); break;
      case 8: s = ms_colsum<8>(c, d); break;
      default:
        s = 0.0f;
        for (int t = 0; t < d; ++t) s += c[t];
    }
    return a.L + (double)s;
  } else {
    const double* c2v = (const double*)c2v_raw;
    const double t = np_sum_col(c2v + p0, d);
    return d == 0 ? a.L : a.L + t;                   // L_post[j] = L0 (:277-278)
  }
}

template <int ALGO, bool LAYERED, int DC>
__global__ void __launch_bounds__(QLDPC_MAX_THREADS) decode_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

  // Stage the read-only graph blob into LDS (16-byte vector copies).
  {
    const uint4* src = (const uint4*)a.blob;
    uint4* dst = (uint4*)lds;
    const int nvec = a.blob_bytes >> 4;
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();

  LdsView g;
  g.cn_tab = (const uint32_t*)(lds + a.off_cn_tab);
  g.row_ptr = (const uint16_t*)(lds + a.off_row_ptr);
  g.vn_info = (const uint32_t*)(lds + a.off_vn_ptr);
  g.chunk_dmax = (const uint8_t*)(lds + a.off_chunk_dmax);
  g.vn_chk = (const uint16_t*)(lds + a.off_vn_chk);
  g.lay_ptr = (const uint16_t*)(lds + a.off_lay_ptr);
  g.lay_rows = (const uint16_t*)(lds + a.off_lay_rows);
  g.adj_ptr = (const uint16_t*)(lds + a.off_adj_ptr);
  g.adj_vars = (const uint16_t*)(lds + a.off_adj_vars);
  g.lt = nullptr;
  if constexpr (ALGO == ALGO_BP) {
    g.lt = stage_libm(lds, a.off_libm);
    __syncthreads();
  }

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int waves = blockDim.x >> 6;
  unsigned char* ws = lds + a.blob_bytes + wid * a.wave_bytes;
  double* post = (double*)ws;
  void* c2v = (void*)(ws + a.off_c2v);
  uint32_t* synw = (uint32_t*)(ws + a.off_synw);
  uint32_t* parw = (uint32_t*)(ws + a.off_parw);

  const int m = a.m, n = a.n;
  const int nwords = (m + 31) >> 5;

  for (HalfShotQueue Q(a, waves, wid); Q.hs < a.batch; Q.advance()) {
    const long long hs = Q.hs;
    Q.prefetch(threadIdx.x & 63);
    int fl = 0;
    int iters = a.max_iter;
    bool conv = false;

    if constexpr (!LAYERED) {
      // ---------------- flooding: one layer holding every check ------------
      uint32_t synreg = 0;  // bit i = syndrome of check lane + 64 i
      for (int i = 0, c = lane; c < m; ++i, c += 64) synreg |= syn_bit(a, hs, c) << i;
      if constexpr (ALGO == ALGO_BP) {
        // BP's first check-node pass reads v2c = L0 (decoders.py:235):
        // post = L0, c2v = 0. (MS's first pass reads float32(L) directly.)
        for (int j = lane; j < n; j += 64) post[j] = a.L;
        double* cz = (double*)c2v;
        for (int p = lane; p < a.E; p += 64) cz[p] = 0.0;
        wave_sync();
      }
      for (int it = 0;; ++it) {
        // CN over all checks; its parity pass is the stop test of iteration it-1
        // (decoders.py:175-176 — checks read the posteriors the last VN wrote).
        uint32_t unsat = 0;
        if constexpr (QLDPC_ABLATE == 2) {
          unsat = 1;
        } else if constexpr (ALGO == ALGO_MS && DC > 0) {
          for (int i = 0, c = lane; c < m; ++i, c += 64) {
            uint32_t t[1][8];
            load_row8(g.cn_tab + c * 8, t[0]);
            const uint32_t sb[1] = {(synreg >> i) & 1u};
            const bool live[1] = {true};
            if (it == 0)
              (void)cn_ms_uniform<DC, true, 1>(a, t, sb, live, (const unsigned char*)post, (unsigned char*)c2v, fl);
            else
              unsat |= cn_ms_uniform<DC, false, 1>(a, t, sb, live, (const unsigned char*)post, (unsigned char*)c2v, fl);
          }
        } else if (it == 0) {
          for (int i = 0, c = lane; c < m; ++i, c += 64)
            (void)cn_update<ALGO, DC>(a, g, c, (synreg >> i) & 1u, true, post, c2v, fl);
        } else {
          for (int i = 0, c = lane; c < m; ++i, c += 64)
            unsat |= cn_update<ALGO, DC>(a, g, c, (synreg >> i) & 1u, false, post, c2v, fl);
        }
        if (it > 0 && ballot(unsat != 0) == 0) {
          iters = it;
          conv = true;
          break;
        }
        wave_sync();
        if constexpr (QLDPC_ABLATE != 1) {
          for (int j0 = 0; j0 < n; j0 += 64) {
            const int dmax = __builtin_amdgcn_readfirstlane((int)g.chunk_dmax[j0 >> 6]);
            const int j = j0 + lane;
            if (j < n) post[j] = vn_post<ALGO>(a, g, j, c2v, dmax);
          }
        }
        wave_sync();
        if (it + 1 == a.max_iter) {
          // final stop test after the last VN (its result only sets the flag:
          // both branches of the reference return max_iter, :176 / :182)
          uint32_t un = 0;
          for (int i = 0, c = lane; c < m; ++i, c += 64) {
            const int e0 = DC ? c * 8 : (int)g.row_ptr[c];
            const int deg = DC ? DC : (int)g.row_ptr[c + 1] - e0;
            uint32_t par = 0;
            for (int k = 0; k < deg; ++k) par ^= (uint32_t)(post[tab_var<DC>(g.cn_tab[e0 + k])] < 0.0);
            un |= par ^ ((synreg >> i) & 1u);
          }
          conv = ballot(un != 0) == 0;
          break;
        }
      }
    } else {
      // ---------------- layered / serial: explicit row lists ----------------
      // State starts at c2v = 0, post = L (msg_v2c = L, :148-149 / :235).
      const double L = a.L;
      for (int j = lane; j < n; j += 64) post[j] = L;
      if constexpr (ALGO == ALGO_MS) {
        float* c = (float*)c2v;
        for (int p = lane; p < a.E; p += 64) c[p] = 0.0f;
      } else {
        double* c = (double*)c2v;
        for (int p = lane; p < a.E; p += 64) c[p] = 0.0;
      }
      // syndrome bits and the parity of the initial hard decisions (all = L<0)
      for (int c0 = 0; c0 < m; c0 += 64) {
        const int c = c0 + lane;
        const int in = c < m;
        store_bits64(synw, c0, in ? (int)syn_bit(a, hs, c) : 0, lane);
        int deg = 0;
        if (in) deg = DC ? DC : (int)g.row_ptr[c + 1] - (int)g.row_ptr[c];
        store_bits64(parw, c0, in && (L < 0.0) && (deg & 1), lane);
      }
      wave_sync();
      bool first = true;
      for (int it = 0; it < a.max_iter && !conv; ++it) {
        for (int l = 0; l < a.n_layers; ++l) {
          // CN over the layer's rows (Jacobi: all read the same posteriors)
          const int q0 = g.lay_ptr[l], q1 = g.lay_ptr[l + 1];
          for (int q = q0 + lane; q < q1; q += 64) {
            const int c = g.lay_rows[q];
            const uint32_t sb = (synw[c >> 5] >> (c & 31)) & 1u;
            (void)cn_update<ALGO, DC>(a, g, c, sb, first, post, c2v, fl);
          }
          first = false;
          wave_sync();
          // VN over the variables adjacent to the layer (others are unchanged,
          // so recomputing every column as decoders.py:172 / :265 does is
          // bit-identical); hard-decision flips toggle check parities.
          const int v0 = g.adj_ptr[l], v1 = g.adj_ptr[l + 1];
          for (int q = v0 + lane; q < v1; q += 64) {
            const int j = g.adj_vars[q];
            const double old = post[j];
            const double nw = vn_post<ALGO>(a, g, j, c2v, -1);
            post[j] = nw;
            if ((old < 0.0) != (nw < 0.0)) {
              const uint32_t info = g.vn_info[j];
              for (int p = (int)(info & 0xffffu), pe = p + (int)(info >> 16); p < pe; ++p) {
                const int c = g.vn_chk[p];
                atomicXor(&parw[c >> 5], 1u << (c & 31));
              }
            }
          }
          wave_sync();
          // stop test after every layer (:175-176 / :283-285)
          uint32_t un = 0;
          for (int w = lane; w < nwords; w += 64) un |= parw[w] ^ synw[w];
          if (ballot(un != 0) == 0) {
            iters = it + 1;
            conv = true;
            break;
          }
        }
      }
    }

    // ---------------- outputs (original column order) ----------------------
    double* po = a.post ? a.post + hs * (long long)n : nullptr;
    for (int jo = lane; jo < n; jo += 64) {
      const double pv = post[a.vinv[jo]];
      put_ehat(a, hs, jo, pv < 0.0);                  // e_hat = post < 0 (:174 / :280)
      if (po) po[jo] = pv;
    }
    // OR the lane-local flags across the wave
    uint32_t fall = 0;
    {
      const uint64_t b1 = ballot((fl & FLAG_MIN_ZERO) != 0);
      const uint64_t b2 = ballot((fl & FLAG_NONFINITE) != 0);
      fall = (b1 ? FLAG_MIN_ZERO : 0) | (b2 ? FLAG_NONFINITE : 0) | (conv ? FLAG_CONVERGED : 0);
    }
    if (lane == 0) {
      a.iters[hs] = iters;
      if (a.flags) a.flags[hs] = (int32_t)fall;
    }
    wave_sync();  // the next half-shot reuses this wave's LDS slice
  }
}

// ---------------------------------------------------------------------------
// Flooding min-sum for uniform row degree DC <= 8 — the headline kernel.
//
// Differences from decode_kernel<MS, false, DC> (same arithmetic, same
// results, bit for bit):
//  * No graph tables in LDS. Each lane's static graph data comes once from
//    HBM ("fblob", capi.cpp) and lives in VGPRs as ready-made LDS byte
//    addresses: pa[i][k] = &post[var], ca[i][k] = &c2v[csc position] of edge
//    k of check c = lane + 64 i. The check-node step then spends no VALU on
//    addressing. Pad checks (c >= m) read post[0] and write the 8-float pad
//    behind c2v; `livem` masks their flags.
//  * Variable nodes are visited by runs of equal column degree K (variables
//    are relabeled by degree, so the CSC start of variable start + o is
//    p0 + o * K): no per-variable table, no masking, a compile-time K.
// The LDS then holds only wave state: post f64[n] | c2v f32[E + 8].
// ---------------------------------------------------------------------------
// Per-lane edge addresses of the KC checks a lane owns: absolute LDS byte
// addresses, 16 VGPRs per check, no VALU per use.
template <int KC>
struct FloodTab {
  uint32_t pa[KC][8], ca[KC][8];
  __device__ __forceinline__ void init(const uint32_t* ftab, int lane, uint32_t pbase, uint32_t cbase) {
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      uint32_t t[8];
      load_row8(ftab + (size_t)(lane + 64 * i) * 8, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        pa[i][k] = pbase + (t[k] & 0xffffu);
        ca[i][k] = cbase + (t[k] >> 16);
        // opaque: otherwise the compiler keeps the packed words and re-forms
        // one of the two addresses with a VALU add at every use
        asm volatile("" : "+v"(pa[i][k]), "+v"(ca[i][k]));
      }
    }
  }
  __device__ __forceinline__ void get(int i, uint32_t (&p)[8], uint32_t (&c)[8]) const {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      p[k] = pa[i][k];
      c[k] = ca[i][k];
    }
  }
};
struct FloodRuns {  // fblob header: runs of equal column degree (capi.cpp)
  int n_runs;
  int start[QLDPC_MAX_RUNS], count[QLDPC_MAX_RUNS], deg[QLDPC_MAX_RUNS], p0[QLDPC_MAX_RUNS];
};

// Sequential float32 sum in ascending check order (np.sum axis=0). It starts
// from the first term instead of 0.0f + x0: the two differ only in the sign of
// an all-zero sum, and post = L + S is the same for S = +0 and S = -0 (L is
// never -0), so the posteriors are bit-identical.
template <int K>
__device__ __forceinline__ float vn_sum(const float* c) {
  if constexpr (K == 0) {
    return 0.0f;
  } else {
    float x[K];
#pragma unroll
    for (int t = 0; t < K; ++t) x[t] = c[t];
    float s = x[0];
#pragma unroll
    for (int t = 1; t < K; ++t) s += x[t];               // float32, ascending check
    return s;
  }
}

template <int K>
__device__ __forceinline__ void vn_run(const DecodeArgs& a, double* post, const float* c2v,
                                       int start, int count, int p0, int lane) {
  // post[start + o] = L + (f64) sum_t c2v[p0 + o K + t]   (decoders.py:172-173)
  // Full 64-variable chunks two at a time (two independent add chains in
  // flight), then the masked tail.
  const float* c = c2v + p0 + lane * K;
  double* po = post + start + lane;
  int o0 = 0;
  if constexpr (QLDPC_VN_PAIR != 0) {
    for (; o0 + 128 <= count; o0 += 128) {
      const float s0 = vn_sum<K>(c + o0 * K);
      const float s1 = vn_sum<K>(c + (o0 + 64) * K);
      po[o0] = a.L + (double)s0;
      po[o0 + 64] = a.L + (double)s1;
    }
  }
  for (; o0 + 64 <= count; o0 += 64) po[o0] = a.L + (double)vn_sum<K>(c + o0 * K);
  if (o0 + lane < count) po[o0] = a.L + (double)vn_sum<K>(c + o0 * K);
}

__device__ __forceinline__ void vn_run_any(const DecodeArgs& a, double* post, const float* c2v,
                                           int start, int count, int K, int p0, int lane) {
  for (int o = lane; o < count; o += 64) {
    const float* c = c2v + p0 + o * K;
    float s = 0.0f;
    for (int t = 0; t < K; ++t) s += c[t];
    post[start + o] = a.L + (double)s;
  }
}

template <int KC>
constexpr int ms_flood_max_threads() { return KC >= 8 ? 512 : 256; }
template <int KC>
constexpr int ms_flood_wpe() { return KC >= 8 ? 2 : QLDPC_FLOOD_WPE; }

template <int DC, int KC>
__global__ void __launch_bounds__(ms_flood_max_threads<KC>()) __attribute__((amdgpu_waves_per_eu(ms_flood_wpe<KC>())))
ms_flood_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  static_assert(DC >= 2 && DC <= 8, "row degree 2..8");
  const FloodRuns* runs = (const FloodRuns*)a.blob;                     // global, uniform
  const uint32_t* ftab = (const uint32_t*)(a.blob + a.off_cn_tab);      // global
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int waves = blockDim.x >> 6;
  unsigned char* ws = lds + QLDPC_FLOOD_HDR + wid * a.wave_bytes;
  double* post = (double*)ws;
  unsigned char* c2v_b = ws + a.off_c2v;
  const float* c2v_f = (const float*)c2v_b;
  const int m = a.m, n = a.n;

  // static per-lane graph data (VGPRs for the kernel)
  FloodTab<KC> tab;
  tab.init(ftab, lane, lds_addr(ws), lds_addr(ws) + (uint32_t)a.off_c2v);
  uint32_t livem = 0;
#pragma unroll
  for (int i = 0; i < KC; ++i)
    if (lane + 64 * i < m) livem |= 1u << i;
  // the runs header lives in LDS (the first QLDPC_FLOOD_HDR bytes): one
  // broadcast read per field per iteration, no global latency in the loop
  const int n_runs = __builtin_amdgcn_readfirstlane(runs->n_runs);
  if (threadIdx.x < 4 * QLDPC_MAX_RUNS) ((int*)lds)[threadIdx.x] = (&runs->start[0])[threadIdx.x];
  __syncthreads();
  const int* hdr = (const int*)lds;

  for (HalfShotQueue Q(a, waves, wid); Q.hs < a.batch; Q.advance()) {
    const long long hs = Q.hs;
    Q.prefetch(threadIdx.x & 63);
    int fl = 0;
    int iters = a.max_iter;
    bool conv = false;
    uint32_t synreg = 0;
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const int c = lane + 64 * i;
      if (c < m) synreg |= syn_bit(a, hs, c) << i;
    }
    for (int it = 0;; ++it) {
      uint32_t unsat = 0;
      if (it == 0) {
        // every v2c = float32(L) (decoders.py:148-149): one value per check
        const double vf = (double)a.L32;
        const double av = __builtin_fabs(vf);
        const uint32_t cb = __builtin_bit_cast(uint32_t, (float)(a.beta * av));
        const uint32_t neg = (uint32_t)(vf < 0.0);
        if (av == 0.0) fl |= FLAG_MIN_ZERO;
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          const uint32_t negprod = ((neg * DC) ^ (synreg >> i)) & 1u;
          const uint32_t val = cb | ((neg ^ negprod) << 31);
          uint32_t pa[8], ca[8];
          tab.get(i, pa, ca);
#pragma unroll
          for (int k = 0; k < DC; ++k) *QLDPC_LDS(uint32_t, ca[k]) = val;
        }
      } else {
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          uint32_t pa[8], ca[8];
          tab.get(i, pa, ca);
          unsat |= cn_ms_abs<DC>(a, pa, ca, (synreg >> i) & 1u, (livem >> i) & 1u, fl);
          __builtin_amdgcn_sched_barrier(0);         // one check's working set at a time
        }
        // stop test of iteration it-1 (decoders.py:175-176)
        if (ballot(unsat != 0) == 0) {
          iters = it;
          conv = true;
          break;
        }
      }
      wave_sync();
      for (int r = 0; r < n_runs; ++r) {
        const int st = __builtin_amdgcn_readfirstlane(hdr[r]);
        const int cnt = __builtin_amdgcn_readfirstlane(hdr[QLDPC_MAX_RUNS + r]);
        const int K = __builtin_amdgcn_readfirstlane(hdr[2 * QLDPC_MAX_RUNS + r]);
        const int p0 = __builtin_amdgcn_readfirstlane(hdr[3 * QLDPC_MAX_RUNS + r]);
        switch (K) {
          case 0: vn_run<0>(a, post, c2v_f, st, cnt, p0, lane); break;
          case 1: vn_run<1>(a, post, c2v_f, st, cnt, p0, lane); break;
          case 2: vn_run<2>(a, post, c2v_f, st, cnt, p0, lane); break;
          case 3: vn_run<3>(a, post, c2v_f, st, cnt, p0, lane); break;
          case 4: vn_run<4>(a, post, c2v_f, st, cnt, p0, lane); break;
          case 5: vn_run<5>(a, post, c2v_f, st, cnt, p0, lane); break;
          case 6: vn_run<6>(a, post, c2v_f, st, cnt, p0, lane); break;
          default: vn_run_any(a, post, c2v_f, st, cnt, K, p0, lane); break;
        }
      }
      wave_sync();
      if (it + 1 == a.max_iter) {
        uint32_t un = 0;
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          uint32_t ph = 0;
          uint32_t pa[8], ca[8];
          tab.get(i, pa, ca);
#pragma unroll
          for (int k = 0; k < DC; ++k) ph ^= hi_word(*QLDPC_LDS(const double, pa[k]));
          un |= (((ph >> 31) ^ (synreg >> i)) & (livem >> i)) & 1u;
        }
        conv = ballot(un != 0) == 0;
        break;
      }
    }
    double* po = a.post ? a.post + hs * (long long)n : nullptr;
    for (int jo = lane; jo < n; jo += 64) {
      const double pv = post[a.vinv[jo]];
      put_ehat(a, hs, jo, pv < 0.0);
      if (po) po[jo] = pv;
    }
    const uint64_t b1 = ballot((fl & FLAG_MIN_ZERO) != 0);
    if (lane == 0) {
      a.iters[hs] = iters;
      if (a.flags) a.flags[hs] = (int32_t)((b1 ? FLAG_MIN_ZERO : 0) | (conv ? FLAG_CONVERGED : 0));
    }
    wave_sync();
  }
}

// ---------------------------------------------------------------------------
// Check node of the layered kernel with G lanes per check (G = 1, 2, 4, 8):
// lane `sub` of a group owns the EPL = 8 / G consecutive edges sub*EPL ..
// of its check. Layers are short (LP118_2: 30 rows, LP118_0: 16, serial: 1),
// so one lane per check left most of the wave idle while it walked all DC
// edges; with G lanes the per-lane chain is EPL edges long and a wave covers
// 64 / G checks per pass. Per lane: min1/min2 of its |v| by the tournament,
// then merged across the group with DPP lane swaps (quad xor 1, quad xor 2,
// half-row mirror) by (l1,h1)+(l2,h2) -> (min(l1,l2), min(max(l1,l2),
// min(h1,h2))); min / max are exact, so the group ends with the reference's
// two values (decoders.py:160-166) whatever the order. The sign product is
// the XOR of the group's sign words over the same swaps. Missing edges (k >=
// DC) read post[0], count as |v| = inf and write nothing.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  return __builtin_bit_cast(double, ((uint64_t)dpp_u32<CTRL>((uint32_t)(u >> 32)) << 32) | dpp_u32<CTRL>((uint32_t)u));
}
constexpr int kDppQuadXor1 = 0xB1;     // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;     // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // row_half_mirror: lane i <-> 7-i within 8

template <int CTRL>
__device__ __forceinline__ void group_merge(double& lo, double& hi, uint32_t& sh) {
  const double olo = dpp_f64<CTRL>(lo), ohi = dpp_f64<CTRL>(hi);
  sh ^= dpp_u32<CTRL>(sh);
  const double nlo = vmin_f64(lo, olo);
  hi = vmin_f64(vmax_f64(lo, olo), vmin_f64(hi, ohi));
  lo = nlo;
}

// Two lanes per check, every lane live (row degree 8: four edges per lane):
// the one-lane-per-check instance's layers of at most 32 rows (round 6).
// Lanes past the layer's last check repeat the trip's first check — the same
// reads, the same values stored — so nothing is masked (as cn_layer's UNI).
__device__ __forceinline__ void cn_ms_pair_uni(const DecodeArgs& a, const uint32_t* trow, int sub, uint32_t synb,
                                               bool first, uint32_t post_b, uint32_t c2v_b, int& fl) {
  const uint4 w = *(const uint4*)(trow + 4 * sub);
  const uint32_t t[4] = {w.x, w.y, w.z, w.w};
  double v[4];
  uint32_t hv[4];
  if (first) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (double)a.L32;            // (:148-149)
  } else {
    // the eight reads in one block, one wait: with the branch inside the edge
    // loop the compiler gave each edge its own block and LDS round trip
    float pf[4], cf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pf[i] = *QLDPC_LDS(const float, post_b + (t[i] & 0xffffu));
      cf[i] = *QLDPC_LDS(const float, c2v_b + (t[i] >> 16));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (a.L + (double)pf[i]) - (double)cf[i];   // (:173, :177)
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) hv[i] = hi_word(v[i]);
  double lo, hi;
  min12_tree<4>(v, lo, hi);
  uint32_t sh = xor_tree<4>(hv);                                  // (:157-159)
  group_merge<kDppQuadXor1>(lo, hi, sh);
  double m1 = lo, m2 = hi;
  if (__builtin_expect(ballot((lo == 0.0) | (hi == __builtin_inf())) != 0, 0)) {
    m1 = __builtin_isinf(lo) ? 0.0 : lo;                          // (:165)
    m2 = __builtin_isinf(hi) ? 0.0 : hi;                          // (:166)
    if (m1 == 0.0) fl |= FLAG_MIN_ZERO;
  }
  const uint32_t npm = ((sh >> 31) ^ synb) << 31;
  const uint32_t c1n = __builtin_bit_cast(uint32_t, (float)(a.beta * m1)) ^ npm;
  const uint32_t c2n = __builtin_bit_cast(uint32_t, (float)(a.beta * m2)) ^ npm;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t c = (__builtin_fabs(v[i]) == lo) ? c2n : c1n;   // (:167-168)
    *QLDPC_LDS(uint32_t, c2v_b + (t[i] >> 16)) = c ^ (hv[i] & 0x80000000u);
  }
}

template <int DC, int G>
__device__ __forceinline__ void cn_ms_split(const DecodeArgs& a, const uint32_t* trow, int sub, bool live,
                                            uint32_t synb, bool first, uint32_t post_b, uint32_t c2v_b,
                                            int& fl) {
  constexpr int EPL = 8 / G;
  uint32_t t[EPL];
  if constexpr (EPL == 8) {
    load_row8(trow, t);
  } else if constexpr (EPL == 4) {
    const uint4 w = *(const uint4*)(trow + 4 * sub);
    t[0] = w.x; t[1] = w.y; t[2] = w.z; t[3] = w.w;
  } else if constexpr (EPL == 2) {
    const uint2 w = *(const uint2*)(trow + 2 * sub);
    t[0] = w.x; t[1] = w.y;
  } else {
    t[0] = trow[sub];
  }
  bool ek[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) ek[i] = live && (DC == 8 || EPL * sub + i < DC);
  double v[EPL];
  uint32_t hv[EPL];
  if (first) {
#pragma unroll
    for (int i = 0; i < EPL; ++i) v[i] = (double)a.L32;          // (:148-149)
  } else {
    // all reads in one block, one wait (as cn_ms_pair_uni)
    float pf[EPL], cf[EPL];
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      pf[i] = *QLDPC_LDS(const float, post_b + (t[i] & 0xffffu));
      cf[i] = *QLDPC_LDS(const float, c2v_b + (t[i] >> 16));
    }
    // post_j = L + (f64)S_j rebuilt from the float32 column sum (exact: the
    // value the reference stores, decoders.py:173); v2c = post - c2v (:177)
#pragma unroll
    for (int i = 0; i < EPL; ++i) v[i] = (a.L + (double)pf[i]) - (double)cf[i];
  }
#pragma unroll
  for (int i = 0; i < EPL; ++i) hv[i] = ek[i] ? hi_word(v[i]) : 0u;
  double av[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) av[i] = ek[i] ? v[i] : __builtin_inf();
  double lo, hi;
  min12_tree<EPL>(av, lo, hi);
  uint32_t sh = xor_tree<EPL>(hv);                                // np.sign product (:157-159)
  if constexpr (G >= 2) group_merge<kDppQuadXor1>(lo, hi, sh);
  if constexpr (G >= 4) group_merge<kDppQuadXor2>(lo, hi, sh);
  if constexpr (G >= 8) group_merge<kDppHalfMirror>(lo, hi, sh);
  double m1 = lo, m2 = hi;
  if (__builtin_expect(ballot(live && ((lo == 0.0) | (hi == __builtin_inf()))) != 0, 0)) {
    m1 = __builtin_isinf(lo) ? 0.0 : lo;                          // (:165)
    m2 = __builtin_isinf(hi) ? 0.0 : hi;                          // (:166)
    if (m1 == 0.0 && live) fl |= FLAG_MIN_ZERO;
  }
  const uint32_t npm = ((sh >> 31) ^ synb) << 31;
  const uint32_t c1n = __builtin_bit_cast(uint32_t, (float)(a.beta * m1)) ^ npm;
  const uint32_t c2n = __builtin_bit_cast(uint32_t, (float)(a.beta * m2)) ^ npm;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const uint32_t c = (__builtin_fabs(v[i]) == lo) ? c2n : c1n;   // (:167-168)
    if (ek[i]) *QLDPC_LDS(uint32_t, c2v_b + (t[i] >> 16)) = c ^ (hv[i] & 0x80000000u);
  }
}


// ---------------------------------------------------------------------------
// Layered / serial min-sum for uniform-degree codes (decoders.py:153-177 with
// an explicit layer list). Per layer: CN over the layer's rows (Jacobi, the
// fast uniform path), VN over the variables adjacent to the layer, parity
// toggles for flipped hard decisions, stop test. The blob holds the layer
// rows' table words in layer order (ltab) and each adjacency slot's
// (variable, csc start | degree) so every phase is one dependent LDS hop
// shorter than decode_kernel<MS, true, DC>.
// ---------------------------------------------------------------------------
// XOR of a 32-bit value over the 64 lanes (all lanes active): DPP within each
// row of 16 lanes, then the four row results.
constexpr int kDppRowMirror = 0x140;   // row_mirror: lane i <-> 15-i within 16
__device__ __forceinline__ uint32_t wave_xor(uint32_t x) {
  x ^= dpp_u32<kDppQuadXor1>(x);
  x ^= dpp_u32<kDppQuadXor2>(x);
  x ^= dpp_u32<kDppHalfMirror>(x);
  x ^= dpp_u32<kDppRowMirror>(x);
  // rows 1 / 3 take lane 15 of rows 0 / 2 (row_bcast:15), then rows 2-3 take
  // lane 31 (row_bcast:31): lane 63 holds the wave's XOR, one readlane instead
  // of four plus three scalar XORs (layered MS -0.7 %, layered BP -0.5 % per
  // launch, profiles/r06/r06w_ab_wave_xor_bcast.json)
  x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// Variable-node pass of one layer (decoders.py:172-174 over the layer's
// adjacent variables) for a wave-uniform degree bound K: two 64-variable
// chunks per trip with every LDS read of both issued before the sums (the
// chunks' variables are distinct, so their colS writes never alias the other
// chunk's reads). Hard decisions are compared in the float32 domain
// (S < hd_thresh is exactly L + (f64)S < 0). Each flipped hard decision
// contributes its variable's filter word (stop test, ms_layered_kernel); the
// lane-local XOR is returned.
// Variables per lane per pass: layers of more than 128 adjacent variables take
// QLDPC_VN_H (4: LP118_2's 240 / 480 in one / two passes instead of two / four,
// -6.5 % per launch), smaller ones 2 (a 4-wide pass over <= 128 variables
// idles half its lanes: LP118_0 +4 %)
// LO (round 6): every variable of the layer has degree >= LO (host flag, bit
// 7 of the layer's degree byte): the sum is formed as prefix sums over all K
// slots and the degree picks one of the last K - LO + 1 of them, instead of a
// compare and select per slot — the same float32 operations on the first d
// terms, so the same bits (s never is -0.0: it starts as 0 + x0)
// TWO (round 6): every degree is LO or K (bit 8; LP118_2's 3 / 5): one select
// of the two prefix sums (32.42 -> 31.71 ms per LP118_2 p = 0.1 launch,
// profiles/r06/r06h_ab_msl_two_min.json)
// one IEEE float32 add (round to nearest, the same v_add_f32 the compiler
// emits) that the SLP vectorizer cannot pair into v_pk_add_f32: the paired
// prefix sums of two variables needed a register move per pair to line up
// their operands (-0.8 % per LP118_2 p = 0.1 launch,
// profiles/r06/r06aa_ab_vn_asm_add.json)
__device__ __forceinline__ float vadd_f32(float a, float b) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int K, int H, int LO = 1, bool TWO = false>
__device__ __forceinline__ uint32_t vn_layer(const uint32_t* adj_info, const uint32_t* avar, float* colS,
                                             const float* c2v, int v0, int v1, int lane, float thr) {
  uint32_t acc = 0;
  auto trip = [&](int qb, const uint32_t (&info)[H]) {
    bool in[H];
#pragma unroll
    for (int h = 0; h < H; ++h) in[h] = qb + 64 * h + lane < v1;
    float old[H];
    uint32_t av[H];
    float x[H][K];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      old[h] = colS[info[h] >> 21];                         // column sum before this layer
      av[h] = avar[info[h] >> 21];
      const float* c = c2v + (info[h] & 0xffffu);
#pragma unroll
      for (int t = 0; t < K; ++t) x[h][t] = c[t];          // c2v padded by 8 floats
    }
    // every read issued before any sum: left alone, the compiler turned a
    // read whose value only feeds a select into an exec-masked read issued
    // after all the others, behind a wait for everything in flight
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int t = 0; t < K; ++t) asm volatile("" : "+v"(x[h][t]));
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int d = (int)((info[h] >> 16) & 31u);
      float s = 0.0f;                                       // sequential, ascending check (:172)
      if constexpr (LO > 1) {
        float pre = vadd_f32(0.0f, x[h][0]);
#pragma unroll
        for (int t = 1; t < LO; ++t) pre = vadd_f32(pre, x[h][t]);
        s = pre;                                            // d = LO
#pragma unroll
        for (int t = LO; t < K; ++t) {
          pre = vadd_f32(pre, x[h][t]);                     // (slots past d: discarded below)
          if constexpr (!TWO) s = d > t ? pre : s;
        }
        if constexpr (TWO) s = d > LO ? pre : s;            // every degree is LO or K
      } else {
#pragma unroll
        for (int t = 0; t < K; ++t) s += (t < d) ? x[h][t] : 0.0f;
      }
      // every lane stores: a pad lane (past v1) holds variable v1 - 1's word
      // and computes exactly the value that variable's lane stored (same reads — the
      // c2v entries do not change in the VN — same sum), so no exec mask is
      // needed around the store (-4.1 % per LP118_2 p = 0.1 launch,
      // -4.9 % LP118_0, profiles/r04ax/)
      colS[info[h] >> 21] = s;
      const bool flip = in[h] && ((old[h] < thr) != (s < thr));   // hard decision flipped (:173-174)
      acc ^= flip ? av[h] : 0u;
    }
  };
  for (int qb = v0; qb < v1; qb += 64 * H) {
    uint32_t info[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int q = qb + 64 * h + lane;
      info[h] = adj_info[min(q, v1 - 1)];
    }
    trip(qb, info);
  }
  return acc;
}

// Exact stop test (decoders.py:175-176): every row's parity of the current
// hard decisions against its syndrome bit. Runs only when the filters pass.
template <int DC>
__device__ __forceinline__ bool layered_full_check(const DecodeArgs& a, const float* colS, const uint32_t* synw,
                                                   int lane, float thr) {
  uint32_t un = 0;
  for (int c = lane; c < a.m; c += 64) {
    const uint4 t0 = *(const uint4*)(a.rtab + 8 * (size_t)c);
    const uint4 t1 = *(const uint4*)(a.rtab + 8 * (size_t)c + 4);
    const uint32_t t[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    uint32_t par = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) par ^= (uint32_t)(colS[t[k]] < thr);
    un |= par ^ ((synw[c >> 5] >> (c & 31)) & 1u);
  }
  return ballot(un != 0) == 0;
}

// Check nodes of one layer (rows q0..q1 of the layer-ordered table) with GG
// lanes per check: GG = 1 walks a row's DC edges in one lane (cn_ms_compute),
// GG > 1 splits them over a lane group (cn_ms_split). All rows read the same
// snapshot of the column sums (Jacobi within the layer, decoders.py:155-169).
// SYNL: the syndrome bit by layer position (synl[q]), else by check index
// (lrow[q], then synw) — see the synl build in ms_layered_kernel
template <int DC, int GG, bool UNI = false, bool SYNL = false>
__device__ __forceinline__ void cn_layer(const DecodeArgs& a, const uint32_t* ltab, const uint16_t* lrow,
                                         const uint32_t* synw, const uint32_t* synl, int q0, int q1, int lane,
                                         bool first,
                                         const float* colS, unsigned char* c2v_b, uint32_t post_b,
                                         uint32_t c2v_a, int& fl) {
  if constexpr (GG == 1) {
    // UNI (the one-lane-per-check kernel instance): a wave-uniform loop —
    // lanes past the layer's last check repeat that check (one v_min; the
    // same reads, all issued before any store, so they store exactly its
    // values) instead of sitting out under an exec mask: -0.9 % per LP118_2
    // p = 0.1 launch, but +2.1 % inside the per-layer switch of LP118_0's
    // instance, which keeps the masked loop (profiles/r04ay/)
    for (int qi = UNI ? q0 : q0 + lane; qi < q1; qi += 64) {
      const int q = !UNI ? qi : min(qi + lane, q1 - 1);
      uint32_t t[1][8];
      load_row8(ltab + q * 8, t[0]);
      const int c = SYNL ? q : lrow[q];
      const uint32_t* sw_base = SYNL ? synl : synw;
      // The row words and the check index go out in one LDS round trip, and
      // the syndrome word with the messages: left alone, the compiler waited
      // for the index before issuing the row reads and hoisted the syndrome
      // read above the branch with a wait of its own (-1.4 % per launch on
      // LP118_2 p = 0.1, profiles/r04aq/)
      __builtin_amdgcn_sched_barrier(0);
      const bool live[1] = {true};
      if (first) {
        const uint32_t sb[1] = {(sw_base[c >> 5] >> (c & 31)) & 1u};
        (void)cn_ms_uniform<DC, true, 1>(a, t, sb, live, (const unsigned char*)colS, c2v_b, fl);
      } else {
        CnLoad<DC> Ld;
        uint32_t ca[8];
        float pf[8];
#pragma unroll
        for (int k = 0; k < DC; ++k) {
          ca[k] = c2v_a + (t[0][k] >> 16);
          pf[k] = *QLDPC_LDS(const float, post_b + (t[0][k] & 0xffffu));
          Ld.cv[k] = *QLDPC_LDS(const float, ca[k]);
        }
        // every read issued before any arithmetic (left alone, the scheduler
        // split the 16 reads over three round trips)
        uint32_t sw = sw_base[c >> 5];
#pragma unroll
        for (int k = 0; k < DC; ++k) asm volatile("" : "+v"(pf[k]), "+v"(Ld.cv[k]));
        asm volatile("" : "+v"(sw));
#pragma unroll
        for (int k = 0; k < DC; ++k) Ld.pj[k] = a.L + (double)pf[k];   // (:173)
        (void)cn_ms_compute<DC>(a, Ld, ca, (sw >> (c & 31)) & 1u, 1u, fl);
      }
    }
  } else {
    // 64 / GG checks per pass; every lane takes part in the group swaps, so
    // the loop runs wave-uniformly
    for (int qb = q0; qb < q1; qb += 64 / GG) {
      const int q = qb + lane / GG;
      const bool live = q < q1;
      const int qs = live ? q : q0;
      const int c = SYNL ? qs : lrow[qs];
      const uint32_t sb = ((SYNL ? synl : synw)[c >> 5] >> (c & 31)) & 1u;
      cn_ms_split<DC, GG>(a, ltab + qs * 8, lane & (GG - 1), live, sb, first, post_b, c2v_a, fl);
    }
  }
}

// Stop test without per-check parity state: 32 fixed random parity checks
// w_k of H's rows. If H e = s then w_k H e = w_k s for every k, so the layer
// can only have converged when the 32 filter parities of the hard decisions
// (F, updated by the flipped variables' words a_j = bit k of w_k H) equal those
// of the syndrome (B); then the exact row-by-row test decides. A state with
// H e != s passes all 32 filters with probability 2^-32, so the exact test
// runs about once per decode, and the per-flip parity toggles (LDS atomics,
// one per edge of every flipped variable) are gone.
template <int DC, int G>
__global__ void __launch_bounds__(QLDPC_MAX_THREADS) ms_layered_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  // QLDPC_MSL_GT (the one-lane-per-check instance): the row table [Q][8] and
  // the filter words stay in global memory (L1/L2-resident; the LDS image
  // starts a.lds_skip bytes in, after the row table, and ends before the
  // filter words), so a CU holds 8 waves' state instead of 7 (LP118_2: 39.9
  // -> 36.5 ms per p = 0.1 launch; loading the next layer's row words a layer
  // ahead measured slower, profiles/r05/msl_global_tables_ab.json)
  constexpr int GT = G == 1 ? QLDPC_MSL_GT : 0;
  const int sk = GT ? a.lds_skip : 0;
  {
    const uint4* src = (const uint4*)(a.blob + sk);
    uint4* dst = (uint4*)lds;
    const int nvec = a.blob_bytes >> 4;
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const uint32_t* ltab_l = (const uint32_t*)(lds + a.off_cn_tab);    // [Q][8]
  const uint32_t* ltab_g = (const uint32_t*)(a.blob + a.off_cn_tab); // [Q][8] global (GT)
  const uint32_t* ltab = [&]() {
    if constexpr (GT != 0) return ltab_g;
    else return ltab_l;
  }();
  const uint16_t* lrow = (const uint16_t*)(lds + a.off_lay_rows - sk);    // [Q]
  const uint16_t* lay_ptr = (const uint16_t*)(lds + a.off_lay_ptr - sk);  // [L+1]
  const uint16_t* adj_ptr = (const uint16_t*)(lds + a.off_adj_ptr - sk);  // [L+1]
  const uint32_t* adj_info = (const uint32_t*)(lds + a.off_row_ptr - sk); // [A] var<<21 | deg<<16 | csc start
  const uint16_t* adj_dmax = (const uint16_t*)(lds + a.off_chunk_dmax - sk);// [L] max degree per layer
  const uint32_t* avar = [&]() {                                         // [n] filter word per variable
    if constexpr (GT != 0) return a.avar;
    else return (const uint32_t*)(lds + a.off_vn_chk - sk);
  }();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int waves = blockDim.x >> 6;
  unsigned char* ws = lds + a.blob_bytes + wid * a.wave_bytes;
  // the slice keeps the float32 column sums S (post = L + (f64)S is rebuilt
  // where it is read): 4 n bytes instead of 8 n, so a CU holds more waves
  float* colS = (float*)ws;
  unsigned char* c2v_b = ws + a.off_c2v;
  float* c2v = (float*)c2v_b;
  uint32_t* synw = (uint32_t*)(ws + a.off_synw);
  uint32_t* synl = (uint32_t*)(ws + a.off_parw);                      // syndrome bits by layer position
  const uint32_t post_b = lds_addr(colS), c2v_a = lds_addr(c2v_b);
  const int m = a.m, n = a.n;
  const float thr = a.hd_thresh;

  // Layer bounds in registers (round 6): lane l holds layer l's row range,
  // adjacency range and degree byte, read at each layer head by v_readlane
  // instead of an LDS round trip (-3.5 % per LP118_2 p = 0.1 launch,
  // profiles/r06/r06c_msl_lreg_ab.json); schedules of more than 64 layers
  // (serial ones) keep the LDS reads (a uniform branch the compiler hoists)
  const bool lreg = a.n_layers <= 64;
  uint32_t lq_r = 0, lv_r = 0;
  int ld_r = 0;
  {
    if (lane < a.n_layers) {
      lq_r = (uint32_t)lay_ptr[lane] | ((uint32_t)lay_ptr[lane + 1] << 16);
      lv_r = (uint32_t)adj_ptr[lane] | ((uint32_t)adj_ptr[lane + 1] << 16);
      ld_r = (int)adj_dmax[lane];
    }
  }
  for (HalfShotQueue Q(a, waves, wid); Q.hs < a.batch; Q.advance()) {
    const long long hs = Q.hs;
    Q.prefetch(threadIdx.x & 63);
    int fl = 0;
    int iters = a.max_iter;
    bool conv = false;
    const double L = a.L;
    {
      const DecodeArgs& ak = QLDPC_MSL_KARGS ? kargs_fresh() : a;
      load_syndrome_bits<8>(ak, hs, synw, lane);
      // 16-byte stores (both regions are 16-byte aligned and padded to a
      // multiple of 4 floats: colS align16(4 n), c2v E + 8): a quarter of the
      // store instructions of the per-half-shot reset — LP118_2 p = 0.01
      // (1.16 iterations per half-shot) 10.86 -> 10.21 ms per launch, p = 0.05
      // -2.7 % (profiles/r06/r06ag_ab_zero4.json)
      const uint4 z = {0u, 0u, 0u, 0u};
      for (int j = 4 * lane; j < n; j += 256) *(uint4*)(colS + j) = z;   // post = L, c2v = 0 (:148-150)
      for (int p = 4 * lane; p < ak.E; p += 256) *(uint4*)(c2v + p) = z;
    }
    wave_sync();
    if constexpr (G == 0) {
      // the syndrome bits in layer order, once per half-shot (the per-layer
      // lane-group instance): each check node reads its bit by layer
      // position (synl) instead of the check index and then the syndrome
      // word: LP118_0 layered 55.08 -> 54.27 ms per launch; the one-lane
      // instance measured slower with it (LP118_2 p = 0.1 +0.9 %, p = 0.05
      // +2.3 %: the index read hides under the row words' global load, the
      // per-half-shot build does not), profiles/r06/r06y_ab_synl.json
      const int nq = lay_ptr[a.n_layers];
      for (int qb = 0; qb < nq; qb += 64) {
        const int q = qb + lane;
        const int c = q < nq ? lrow[q] : 0;
        const uint64_t bl = ballot(q < nq && ((synw[c >> 5] >> (c & 31)) & 1u));
        if (lane == 0) {
          synl[qb >> 5] = (uint32_t)bl;
          synl[(qb >> 5) + 1] = (uint32_t)(bl >> 32);
        }
      }
    }
    wave_sync();
    // filter parities of the syndrome (B) and of the hard decisions (F: all
    // variables start at post = L, so all ones iff L < 0)
    uint32_t bl = 0;
    uint32_t F;
    {
      const DecodeArgs& ak = QLDPC_MSL_KARGS ? kargs_fresh() : a;
      for (int c = lane; c < m; c += 64) bl ^= ((synw[c >> 5] >> (c & 31)) & 1u) ? ak.wc[c] : 0u;
      F = (L < 0.0) ? ak.filt_all : 0u;
    }
    const uint32_t B = wave_xor(bl);
    bool first = true;
    for (int it = 0; it < a.max_iter && !conv; ++it) {
      for (int l = 0; l < a.n_layers; ++l) {
        uint32_t dq, dv;
        int dsel;
        if (lreg) {
          dq = (uint32_t)__builtin_amdgcn_readlane((int)lq_r, l);
          dv = (uint32_t)__builtin_amdgcn_readlane((int)lv_r, l);
          dsel = __builtin_amdgcn_readlane(ld_r, l);
        } else {
          dq = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)lay_ptr[l] | ((uint32_t)lay_ptr[l + 1] << 16)));
          dv = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)adj_ptr[l] | ((uint32_t)adj_ptr[l + 1] << 16)));
          dsel = __builtin_amdgcn_readfirstlane((int)adj_dmax[l]);
        }
        const int q0 = (int)(dq & 0xffffu), q1 = (int)(dq >> 16);
        if constexpr ((QLDPC_ABLATE_L & 1) != 0) {
        } else if constexpr (G != 0) {
          if constexpr (QLDPC_MSL_PRIO == 1) __builtin_amdgcn_s_setprio(1);
          if constexpr (QLDPC_MSL_PRIO == 2) __builtin_amdgcn_s_setprio(0);
          if (G == 1 && DC == 8 && q1 - q0 <= 32) {
            // a layer of at most 32 rows: two lanes per check (four edges
            // each, one DPP merge) instead of half the wave repeating the
            // first check: 33.40 -> 32.77 ms per LP118_2 p = 0.1 launch
            // (profiles/r06/r06f_ab_g2s.json; the generic split check node
            // instead: 34.25 ms)
            for (int qb = q0; qb < q1; qb += 32) {
              const int q = qb + (lane >> 1);
              const int qs = min(q, q1 - 1);
              const int c = lrow[qs];
              const uint32_t sb = (synw[c >> 5] >> (c & 31)) & 1u;
              cn_ms_pair_uni(a, ltab + qs * 8, lane & 1, sb, first, post_b, c2v_a, fl);
            }
          } else
            cn_layer<DC, G, G == 1>(a, ltab, lrow, synw, synl, q0, q1, lane, first, colS, c2v_b, post_b, c2v_a, fl);
          if constexpr (QLDPC_MSL_PRIO == 1) __builtin_amdgcn_s_setprio(0);
          if constexpr (QLDPC_MSL_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        } else {
          // lanes per check chosen per layer by the host (bits 5-6 of adj_dmax)
          switch ((dsel >> 5) & 3) {
            case 0: cn_layer<DC, 1, false, true>(a, ltab, lrow, synw, synl, q0, q1, lane, first, colS, c2v_b, post_b, c2v_a, fl); break;
            case 1: cn_layer<DC, 2, false, true>(a, ltab, lrow, synw, synl, q0, q1, lane, first, colS, c2v_b, post_b, c2v_a, fl); break;
            case 2: cn_layer<DC, 4, false, true>(a, ltab, lrow, synw, synl, q0, q1, lane, first, colS, c2v_b, post_b, c2v_a, fl); break;
            default: cn_layer<DC, 8, false, true>(a, ltab, lrow, synw, synl, q0, q1, lane, first, colS, c2v_b, post_b, c2v_a, fl); break;
          }
        }
        first = false;
        wave_sync();
        // VN over the layer's adjacent variables (decoders.py:172-174: the
        // other columns are unchanged, so this equals the full recompute)
        const int v0 = (int)(dv & 0xffffu), v1 = (int)(dv >> 16);
        const int dmax = dsel & 31;
        const bool lo3 = (dsel & 0x80) != 0;                // every adjacent variable of degree >= 3
        const bool two = (dsel & 0x100) != 0;               // ... and of degree 3 or dmax
        uint32_t acc = 0;
        switch ((QLDPC_ABLATE_L & 2) ? -1 : dmax) {
          case -1: break;
#define QLDPC_VN_CASE(K)                                                                              \
  case K:                                                                                             \
    if (K >= 5 && two)                                                                                \
      acc = v1 - v0 > 128 ? vn_layer<K, QLDPC_VN_H, 3, K >= 5>(adj_info, avar, colS, c2v, v0, v1, lane, thr) \
                          : vn_layer<K, 2, 3, K >= 5>(adj_info, avar, colS, c2v, v0, v1, lane, thr);  \
    else if (lo3)                                                                                     \
      acc = v1 - v0 > 128 ? vn_layer<K, QLDPC_VN_H, 3>(adj_info, avar, colS, c2v, v0, v1, lane, thr)  \
                          : vn_layer<K, 2, 3>(adj_info, avar, colS, c2v, v0, v1, lane, thr);          \
    else                                                                                              \
      acc = v1 - v0 > 128 ? vn_layer<K, QLDPC_VN_H>(adj_info, avar, colS, c2v, v0, v1, lane, thr)     \
                          : vn_layer<K, 2>(adj_info, avar, colS, c2v, v0, v1, lane, thr);             \
    break;
          QLDPC_VN_CASE(3) QLDPC_VN_CASE(4) QLDPC_VN_CASE(5) QLDPC_VN_CASE(6)
#undef QLDPC_VN_CASE
          default:
            for (int q = v0 + lane; q < v1; q += 64) {
              const uint32_t info = adj_info[q];
              const int j = (int)(info >> 21), d = (int)((info >> 16) & 31u);
              const float old = colS[j];
              const float s = ms_colsum_sw(c2v + (info & 0xffffu), d, dmax);
              colS[j] = s;
              if ((old < thr) != (s < thr)) acc ^= avar[j];       // hard decision flipped
            }
        }
        if constexpr ((QLDPC_ABLATE_L & 4) == 0) F ^= wave_xor(acc);
        wave_sync();
        // stop test (:175-176): filters first, the exact test only if they pass
        if (F == B && layered_full_check<DC>(QLDPC_MSL_KARGS ? kargs_fresh() : a, colS, synw, lane, thr)) {
          iters = it + 1;
          conv = true;
          break;
        }
      }
    }
    // ê, posteriors in original order (post = L + (f64)S, decoders.py:173-174)
    {
      const DecodeArgs& ak = QLDPC_MSL_KARGS ? kargs_fresh() : a;
      write_outputs_batched<4>(ak, hs, lane, [&](int v) { return L + (double)colS[v]; });
      const uint64_t b1 = ballot((fl & FLAG_MIN_ZERO) != 0);
      if (lane == 0) {
        ak.iters[hs] = iters;
        if (ak.flags) ak.flags[hs] = (int32_t)((b1 ? FLAG_MIN_ZERO : 0) | (conv ? FLAG_CONVERGED : 0));
      }
    }
    wave_sync();
  }
}

// ---------------------------------------------------------------------------
// Sum-product BP for uniform row degree DC (7 or 8): one TEAM of W wavefronts
// (one workgroup) decodes one half-shot, with the check-node update spread
// over the edges — 8 lanes per check, lane k owns edge k — instead of a lane
// per check. Same arithmetic, same results as decode_kernel<BP, …, DC>, bit
// for bit (decoders.py:249-262 per check):
//   t_k  = tanh(v_k / 2)                 one lane per edge
//   P    = ((t_0 t_1) t_2) ... t_{d-1}   np.prod's sequential fold, carried
//                                        lane to lane by d-1 shuffles
//   c2v_k = ±2 atanh(clip(P / t_k))       one lane per edge
// Why: BP's float64 state is large (LP118_2: 37 KB per half-shot), so a
// one-wave-per-half-shot kernel runs 3-7 waves per CU and stalls on the long
// dependent tanh / atanh chains (30-60 % VALU busy). A team puts 4-8x the
// lanes on one half-shot's state: more waves per CU for the same LDS, and a
// layered layer (30-60 checks) becomes one pass of 8-lane groups.
// Variable nodes: one lane per variable (np.sum pairwise rule), as before.
// Team-wide stop tests go through LDS slots (double-buffered, one barrier);
// layered: parity filters posted per wave (see the layered branch).
// ---------------------------------------------------------------------------
// Saturated check nodes. NumPy's tanh is +-1.0 exactly for |x| >= 19.5: the
// interval [16, 24) evaluates 1 + y r(y) with |y r(y)| ~ 2 exp(-2|x|) <=
// 2.3e-17, below half an ulp of 1 (2^-54), and [24, inf) has the constant
// polynomial 1 (include/qldpc_numpy_tables.h; checked on the host restatement
// and against NumPy, tests/test_libm.py). When every edge of a check has
// |v2c / 2| >= 19.5, all its t_k are +-1, np.prod is +-1, th2 = P / t_k is
// +-1 and clips to +-(1 - eps) (decoders.py:256-258), so c2v_k = +-2
// atanh(1 - eps): one constant, DecodeArgs::bp_csat (capi.cpp, the same
// restated atanh). A finite |x| is >= 19.5 iff its high word (sign cleared)
// is >= 0x40338000 (19.5's low word is 0): DecodeArgs::bp_sat_hi, or
// 0x7ff00000 (never) when the constant is not finite (eps <= 0: atanh(1)).

// edge k of a check whose table word t (row table entry 8c + k) is given;
// SAT: with the saturated-check fast path
template <int DC, bool SAT>
__device__ __forceinline__ uint32_t cn_bp_word(const DecodeArgs& a, const qldpc_libm_tab* lt, uint32_t t, bool valid,
                                               int k, int lane, uint32_t synb, const double* post, double* c2v,
                                               int& fl) {
  const bool ek = valid && k < DC;
  // a wave with no check of this pass skips it (uniform); inside, every lane
  // loads and computes (t = 0 for a pad edge / check: variable 0, position
  // 0, in bounds) and the pad lanes' values are replaced by selects — no
  // exec-masked branches around the loads and the tanh
  if (ballot_b(valid) == 0) return 0u;
  constexpr int CP = SAT ? QLDPC_BP_CNPRIO : QLDPC_BP_FCNPRIO;   // check-node phase priorities
  if constexpr (CP == 1 || CP == 2) __builtin_amdgcn_s_setprio(1);
  const int j = (int)((t & 0xffffu) >> 3), p = (int)(t >> 18);
  const double pjr = post[j];
  const double x = (pjr - c2v[p]) / 2.0;                      // v2c (:269)
  // saturated (finite, |x| >= 19.5): the high word (sign cleared) in
  // [bp_sat_hi, 0x7ff00000), one unsigned compare after the subtraction
  const uint32_t xh = (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32) & 0x7fffffffu;
  const uint32_t shi = a.bp_sat_hi;
  const bool unsat = xh - shi >= 0x7ff00000u - shi;
  if (SAT && ballot_b(ek & unsat) == 0) {
    // every edge of the wave's checks saturated: t_k = sign(x_k), P = the
    // product of the group's signs (pad edges: +1), the message's sign =
    // sign(P / t_k), then the syndrome's (:260-261)
    const double csat = kargs_fresh<DecodeArgs>().bp_csat;
    const uint64_t nb = ballot_b(ek && x < 0.0);
    const uint32_t gs = (uint32_t)(nb >> (lane & 56)) & 0xffu;
    const uint32_t neg = ((uint32_t)__builtin_popcount(gs) ^ (gs >> (lane & 7)) ^ synb) & 1u;
    if (ek) c2v[p] = neg ? -csat : csat;
    const uint64_t hb = ballot_b(ek && pjr < 0.0);
    const uint32_t par = (uint32_t)__builtin_popcount((uint32_t)(hb >> (lane & 56)) & 0xffu) & 1u;
    if constexpr (CP == 1 || CP == 2) __builtin_amdgcn_s_setprio(0);
    return valid ? (par ^ synb) : 0u;
  }
  double th;                                                  // np.tanh (:254)
  if (__builtin_expect(ballot_b(!(__builtin_fabs(x) < 0x1p1023)) != 0, 0))
    th = qldpc_tanh_x(x, lt->tanh_c, 0);                      // a NaN / huge argument in the wave
  else
    th = qldpc_tanh_x(x, lt->tanh_c, 1);
  th = ek ? th : 1.0;
  if constexpr (CP == 1) __builtin_amdgcn_s_setprio(0);
  const double pj = ek ? pjr : 0.0;
  // np.prod: sequential left fold over the check's edges in ascending variable
  // order, ((t_0 t_1) t_2) ..., formed redundantly by every lane of the group
  // from the group's t values (one permute each): same rounding as a
  // lane-to-lane prefix chain, without its per-step index arithmetic, selects
  // and final broadcast (BP flooding is VALU-bound)
  const int base = lane & ~7;
  // (the permutes issued together before the fold, each waited for in turn
  // now: +1 % per BP-L launch through register spills, r06k_ab_cn_reads_bp_shfl.json)
  double P = __shfl(th, base, 64);
#pragma unroll
  for (int s = 1; s < DC; ++s) P = P * __shfl(th, base + s, 64);
  // parity of the hard decisions of the posteriors this check read (:283-285)
  const uint64_t hb = ballot_b(ek && pj < 0.0);
  const uint32_t par = (uint32_t)__builtin_popcount((uint32_t)(hb >> (lane & 56)) & 0xffu) & 1u;
  // Every lane computes (a pad lane: th = 1, its results discarded); only
  // the message store is guarded.
  // P / th (:256). QLDPC_DIV is IEEE division for nonzero operands in the
  // normal range (|th| <= 1 and |P| <= |th| here); a wave holding a zero
  // (a -0 product keeps its sign only through v_div_fixup), tiny or
  // non-finite one divides the general way.
  double th2;
  if (__builtin_expect(ballot_b(ek && !(__builtin_fabs(th) > 1e-150 && __builtin_fabs(P) > 1e-150)) != 0, 0))
    th2 = P / th;
  else
    th2 = QLDPC_DIV(P, th);
  // (:257-258): |th2| >= 1 - eps implies th2 != 0, so th2 - eps sign(th2)
  // is copysign(|th2| - eps, th2) (round-to-nearest is symmetric in sign;
  // a NaN compares false and stays)
  th2 = (__builtin_fabs(th2) >= 1.0 - a.eps) ? __builtin_copysign(__builtin_fabs(th2) - a.eps, th2) : th2;
  if constexpr (CP == 2) __builtin_amdgcn_s_setprio(0);
  if constexpr (CP == 3) __builtin_amdgcn_s_setprio(1);
  // np.arctanh (:259); SVML's rare path (|th2| >= 1, NaN) only when a lane
  // of the wave needs it
  double at;
  if (__builtin_expect(ballot_b(ek && !(__builtin_fabs(th2) < 1.0)) != 0, 0))
    at = qldpc_atanh_x(th2, lt->atanh_hl, lt->atanh_rcp, 0);
  else
    at = qldpc_atanh_x(th2, lt->atanh_hl, lt->atanh_rcp, 1);
  double val = 2.0 * at;
  if (synb) val = -val;                                   // (:260-261)
  if (ek && (th == 0.0 || !__builtin_isfinite(val))) fl |= FLAG_NONFINITE;
  if (ek) c2v[p] = val;
  if constexpr (CP == 3) __builtin_amdgcn_s_setprio(0);
  return valid ? (par ^ synb) : 0u;
}

template <int DC, bool SAT>
__device__ __forceinline__ uint32_t cn_bp_group(const DecodeArgs& a, const LdsView& g, int c, bool valid,
                                                int k, int lane, uint32_t synb, const double* post,
                                                double* c2v, int& fl) {
  const uint32_t tw = g.cn_tab[8 * c + k];                     // (c = 0 for a pad check)
  const uint32_t t = (valid && k < DC) ? tw : 0u;
  return cn_bp_word<DC, SAT>(a, g.lt, t, valid, k, lane, synb, post, c2v, fl);
}

// Every graph table in LDS: the flooding BP kernel (VALU-bound), and the
// layered fallback when the schedule has no global layer image (n > 2048 or a
// column degree > 31, capi.cpp); bp_team_lg_kernel is the layered default.
template <bool LAYERED, int DC, int W>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4))) bp_team_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  {
    const uint4* src = (const uint4*)a.blob;
    uint4* dst = (uint4*)lds;
    const int nvec = a.blob_bytes >> 4;
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) dst[i] = src[i];
  }
  LdsView g;
  g.lt = stage_libm(lds, a.off_libm);
  __syncthreads();
  g.cn_tab = (const uint32_t*)(lds + a.off_cn_tab);
  g.row_ptr = (const uint16_t*)(lds + a.off_row_ptr);
  g.vn_info = (const uint32_t*)(lds + a.off_vn_ptr);
  g.chunk_dmax = (const uint8_t*)(lds + a.off_chunk_dmax);
  g.vn_chk = (const uint16_t*)(lds + a.off_vn_chk);
  g.lay_ptr = (const uint16_t*)(lds + a.off_lay_ptr);
  g.lay_rows = (const uint16_t*)(lds + a.off_lay_rows);
  g.adj_ptr = (const uint16_t*)(lds + a.off_adj_ptr);
  g.adj_vars = (const uint16_t*)(lds + a.off_adj_vars);

  constexpr int TS = 64 * W;        // threads per team
  constexpr int GP = 8 * W;         // 8-lane check groups per pass
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int grp = tid >> 3, k = tid & 7;
  unsigned char* ws = lds + a.blob_bytes;
  double* post = (double*)ws;
  double* c2v = (double*)(ws + a.off_c2v);
  uint32_t* synw = (uint32_t*)(ws + a.off_synw);
  uint32_t* red = (uint32_t*)(ws + a.off_red);          // [2][W] any-slots, [2][2] tickets
  const int m = a.m, n = a.n;
  const double L = a.L;

  int rphase = 0;
  auto team_any = [&](bool pred) -> bool {              // one barrier
    const uint64_t b = ballot(pred);
    if (lane == 0) red[rphase * W + wid] = b != 0;
    __syncthreads();
    bool r = false;
#pragma unroll
    for (int w = 0; w < W; ++w) r |= red[rphase * W + w] != 0;
    rphase ^= 1;
    return r;
  };

  // team-level guided work queue (HalfShotQueue's policy, one ticket per team)
  long long hs = blockIdx.x, end = hs + 1;
  const long long stride = gridDim.x;
  uint32_t seen = 0, tlen = 1, tk = 0;
  int tphase = 0;
  while (hs < a.batch) {
    bool claimed = false;
    if (a.queue && hs + 1 == end) {
      const long long rem = a.batch - stride - (long long)seen;
      long long len = rem / (4 * stride);
      len = len < 1 ? 1 : (len > 64 ? 64 : len);
      tlen = (uint32_t)len;
      claimed = true;
      if (tid == 0) tk = atomicAdd(a.queue, tlen);
    }
    int fl = 0;
    int iters = a.max_iter;
    bool conv = false;

    // state: post = L, c2v = 0 (decoders.py:235-236); syndrome (and, layered,
    // initial parity) bit-words
    for (int j = tid; j < n; j += TS) post[j] = L;
    for (int p = tid; p < a.E; p += TS) c2v[p] = 0.0;
    team_syndrome_bits<2, TS>(a, hs, synw, tid);
    __syncthreads();

    if constexpr (!LAYERED) {
      for (int it = 0;; ++it) {
        uint32_t unsat = 0;
        for (int c0 = 0; c0 < m; c0 += GP) {
          const int c = c0 + grp;
          const bool valid = c < m;
          const uint32_t sb = valid ? (synw[c >> 5] >> (c & 31)) & 1u : 0u;
          unsat |= cn_bp_group<DC, false>(a, g, valid ? c : 0, valid, k, lane, sb, post, c2v, fl);
        }
        // the parity pass is the stop test of iteration it-1 (:283-285); its
        // team barrier also orders these c2v writes before the VN reads them
        if (it > 0) {
          if (!team_any(unsat != 0)) {
            iters = it;
            conv = true;
            break;
          }
        } else {
          __syncthreads();
        }
        for (int j = tid; j < n; j += TS) post[j] = vn_post<ALGO_BP>(a, g, j, c2v, -1);
        __syncthreads();
        if (it + 1 == a.max_iter) {
          uint32_t un = 0;
          for (int c = tid; c < m; c += TS) {
            uint32_t par = 0;
#pragma unroll
            for (int q = 0; q < DC; ++q) par ^= (uint32_t)(post[tab_var<DC>(g.cn_tab[8 * c + q])] < 0.0);
            un |= par ^ ((synw[c >> 5] >> (c & 31)) & 1u);
          }
          conv = !team_any(un != 0);
          break;
        }
      }
    } else {
      // Stop test after every layer (:283-285) by ms_layered_kernel's 32
      // parity filters: B = the syndrome's filter parities, F
      // = the hard decisions', kept current with the filter word of every
      // variable the VN flips; only F == B (convergence, or a 2^-32 false
      // match) runs the exact row check. Each wave posts its flips' XOR in a
      // slot read after the VN barrier, so a layer costs two team barriers,
      // not three, and no parity atomics.
      uint32_t bl = 0;
      for (int c = lane; c < m; c += 64) bl ^= ((synw[c >> 5] >> (c & 31)) & 1u) ? a.wc[c] : 0u;
      const uint32_t B = wave_xor(bl);
      uint32_t F = (L < 0.0) ? a.filt_all : 0u;           // every post starts at L
      uint32_t* fsl = red + 2 * W + 4;                    // [W] filter words of this layer's flips
      for (int it = 0; it < a.max_iter && !conv; ++it) {
        for (int l = 0; l < a.n_layers; ++l) {
          const int q0 = g.lay_ptr[l], q1 = g.lay_ptr[l + 1];
          for (int qb = q0; qb < q1; qb += GP) {
            const int q = qb + grp;
            const bool valid = q < q1;
            const int c = valid ? (int)g.lay_rows[q] : 0;
            const uint32_t sb = valid ? (synw[c >> 5] >> (c & 31)) & 1u : 0u;
            (void)cn_bp_group<DC, QLDPC_BP_SAT>(a, g, c, valid, k, lane, sb, post, c2v, fl);
          }
          __syncthreads();
          // VN over the layer's adjacent variables
          const int v0 = g.adj_ptr[l], v1 = g.adj_ptr[l + 1];
          uint32_t acc = 0;
          for (int q = v0 + tid; q < v1; q += TS) {
            const int j = g.adj_vars[q];
            const double old = post[j];
            const double nw = vn_post<ALGO_BP>(a, g, j, c2v, -1);
            post[j] = nw;
            if ((old < 0.0) != (nw < 0.0)) acc ^= a.avar[j];   // hard decision flipped
          }
          const uint32_t wacc = wave_xor(acc);
          if (lane == 0) fsl[wid] = wacc;
          __syncthreads();
#pragma unroll
          for (int w = 0; w < W; ++w) F ^= fsl[w];
          if (F == B) {                                   // team-uniform
            uint32_t un = 0;
            for (int c = tid; c < m; c += TS) {
              uint32_t par = 0;
#pragma unroll
              for (int q = 0; q < DC; ++q) par ^= (uint32_t)(post[tab_var<DC>(g.cn_tab[8 * c + q])] < 0.0);
              un |= par ^ ((synw[c >> 5] >> (c & 31)) & 1u);
            }
            if (!team_any(un != 0)) {
              iters = it + 1;
              conv = true;
              break;
            }
          }
        }
      }
    }
    write_outputs_strided<4, TS>(a, hs, tid, [&](int v) { return post[v]; });   // (:280)
    const bool nonfin = team_any((fl & FLAG_NONFINITE) != 0);
    if (tid == 0) {
      a.iters[hs] = iters;
      if (a.flags) a.flags[hs] = (int32_t)((nonfin ? FLAG_NONFINITE : 0) | (conv ? FLAG_CONVERGED : 0));
      if (claimed) {
        red[2 * W + 2 * tphase] = tk;
        red[2 * W + 2 * tphase + 1] = tlen;
      }
    }
    __syncthreads();                                      // slice reuse; ticket visible
    if (!a.queue) {
      hs += stride;
    } else if (++hs >= end) {
      const uint32_t t0 = red[2 * W + 2 * tphase], l0 = red[2 * W + 2 * tphase + 1];
      tphase ^= 1;
      seen = t0 + l0;
      hs = stride + (long long)t0;
      end = hs + l0;
    }
  }
}

// ---------------------------------------------------------------------------
// Layered BP teams with every graph table in global memory (L1/L2-resident):
// the rows in layer order (8 table words each) and their check indices, and
// per adjacency slot of a layer its (variable, degree, CSC start) word. LDS
// then holds only the team's float64 state (LP118_2: 37 KB), so a CU holds
// 4 four-wave teams (the VGPR cap) instead of 3 with the row table alone in
// global memory or 2 with every table in LDS. The table reads are issued a
// phase ahead: this layer's adjacency words while its check nodes run, the
// next layer's row words while this layer's variable nodes run. Same
// arithmetic as bp_team_kernel<true, DC, W>, bit for bit.
// ---------------------------------------------------------------------------
template <int DC, int W>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4))) bp_team_lg_kernel(DecodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  {
    const uint4* src = (const uint4*)a.blob;                    // LDS part: layer pointers
    uint4* dst = (uint4*)lds;
    const int nvec = a.blob_bytes >> 4;
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) dst[i] = src[i];
  }
  const qldpc_libm_tab* lt = stage_libm(lds, a.off_libm);
  __syncthreads();
  const uint32_t* ltab_g = (const uint32_t*)(a.blob + a.off_cn_tab);      // [Q][8] rows, layer order
  const uint16_t* lrow_g = (const uint16_t*)(a.blob + a.off_lay_rows);    // [Q]    their checks
  const uint32_t* adj_g = (const uint32_t*)(a.blob + a.off_row_ptr);      // [A]    var<<21 | deg<<16 | start
  const uint16_t* lay_ptr = (const uint16_t*)(lds + a.off_lay_ptr);
  const uint16_t* adj_ptr = (const uint16_t*)(lds + a.off_adj_ptr);

  constexpr int TS = 64 * W;        // threads per team
  constexpr int GP = 8 * W;         // 8-lane check groups per pass
  constexpr int NPF = 2;            // CN passes prefetched per layer
  constexpr int NAF = 2;            // VN slots prefetched per thread
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int grp = tid >> 3, k = tid & 7;
  unsigned char* ws = lds + a.blob_bytes;
  double* post = (double*)ws;
  double* c2v = (double*)(ws + a.off_c2v);
  uint32_t* synw = (uint32_t*)(ws + a.off_synw);
  uint32_t* red = (uint32_t*)(ws + a.off_red);
  const int m = a.m, n = a.n, nl = a.n_layers;
  const double L = a.L;

  int rphase = 0;
  auto team_any = [&](bool pred) -> bool {              // one barrier
    const uint64_t b = ballot(pred);
    if (lane == 0) red[rphase * W + wid] = b != 0;
    __syncthreads();
    bool r = false;
#pragma unroll
    for (int w = 0; w < W; ++w) r |= red[rphase * W + w] != 0;
    rphase ^= 1;
    return r;
  };
  uint32_t pt[NPF], pc[NPF];                            // prefetched row words / checks
  auto rows_pf = [&](int l) {
    const int q0 = lay_ptr[l], q1 = lay_ptr[l + 1];
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int q = q0 + GP * i + grp;
      const bool v = q < q1;
      pt[i] = (v && k < DC) ? ltab_g[8 * q + k] : 0u;
      pc[i] = v ? lrow_g[q] : 0u;
    }
  };

  long long hs = blockIdx.x, end = hs + 1;
  const long long stride = gridDim.x;
  uint32_t seen = 0, tlen = 1, tk = 0;
  int tphase = 0;
  while (hs < a.batch) {
    bool claimed = false;
    if (a.queue && hs + 1 == end) {
      const long long rem = a.batch - stride - (long long)seen;
      long long len = rem / (4 * stride);
      len = len < 1 ? 1 : (len > 64 ? 64 : len);
      tlen = (uint32_t)len;
      claimed = true;
      if (tid == 0) tk = atomicAdd(a.queue, tlen);
    }
    int fl = 0;
    int iters = a.max_iter;
    bool conv = false;
    rows_pf(0);
    for (int j = tid; j < n; j += TS) post[j] = L;      // (decoders.py:235-236)
    for (int p = tid; p < a.E; p += TS) c2v[p] = 0.0;
    team_syndrome_bits<2, TS>(a, hs, synw, tid);
    __syncthreads();
    // stop test after every layer by the parity filters (bp_team_kernel)
    uint32_t bl = 0;
    for (int c = lane; c < m; c += 64) bl ^= ((synw[c >> 5] >> (c & 31)) & 1u) ? a.wc[c] : 0u;
    const uint32_t B = wave_xor(bl);
    uint32_t F = (L < 0.0) ? a.filt_all : 0u;
    uint32_t* fsl = red + 2 * W + 4;
    for (int it = 0; it < a.max_iter && !conv; ++it) {
      for (int l = 0; l < nl; ++l) {
        const int q0 = lay_ptr[l], q1 = lay_ptr[l + 1];
        const int v0 = adj_ptr[l], v1 = adj_ptr[l + 1];
        uint32_t pa[NAF];                                 // this layer's adjacency, in flight during the CN
#pragma unroll
        for (int i = 0; i < NAF; ++i) {
          const int q = v0 + TS * i + tid;
          pa[i] = q < v1 ? adj_g[q] : 0u;
        }
#pragma unroll
        for (int i = 0; i < NPF; ++i) {
          if (q0 + GP * i < q1) {
            const bool valid = q0 + GP * i + grp < q1;
            const int c = (int)pc[i];
            // (c = 0 for a pad check: an unmasked in-bounds read)
            const uint32_t sb = (valid ? synw[c >> 5] >> (c & 31) : 0u) & 1u;
            (void)cn_bp_word<DC, QLDPC_BP_SAT>(a, lt, pt[i], valid, k, lane, sb, post, c2v, fl);
          }
        }
        for (int qb = q0 + GP * NPF; qb < q1; qb += GP) {  // layers of more than NPF passes
          const int q = qb + grp;
          const bool valid = q < q1;
          const int c = valid ? (int)lrow_g[q] : 0;
          const uint32_t t = (valid && k < DC) ? ltab_g[8 * q + k] : 0u;
          const uint32_t sb = valid ? (synw[c >> 5] >> (c & 31)) & 1u : 0u;
          (void)cn_bp_word<DC, QLDPC_BP_SAT>(a, lt, t, valid, k, lane, sb, post, c2v, fl);
        }
        rows_pf(l + 1 < nl ? l + 1 : 0);                  // in flight during the VN
        // the team's variable nodes ahead of other teams' check nodes on the
        // SIMD: a layer's VN is short and every wave of the team waits for it
        // at the next barrier
        if constexpr (QLDPC_BP_VNPRIO != 0) __builtin_amdgcn_s_setprio(QLDPC_BP_VNPRIO);
        __syncthreads();
        uint32_t acc = 0;                                 // VN over the layer's adjacent variables
        auto vn = [&](uint32_t info) {
          const int j = (int)(info >> 21), d = (int)((info >> 16) & 31u);
          const double old = post[j];
          const double sc = np_sum_col<true>(c2v + (info & 0xffffu), d);
          const double nw = d == 0 ? L : L + sc;            // (:276-278)
          post[j] = nw;
          if ((old < 0.0) != (nw < 0.0)) acc ^= a.avar[j];
        };
#pragma unroll
        for (int i = 0; i < NAF; ++i)
          if (v0 + TS * i + tid < v1) vn(pa[i]);
        for (int q = v0 + TS * NAF + tid; q < v1; q += TS) vn(adj_g[q]);
        const uint32_t wacc = wave_xor(acc);
        if (lane == 0) fsl[wid] = wacc;
        __syncthreads();
        if constexpr (QLDPC_BP_VNPRIO != 0) __builtin_amdgcn_s_setprio(QLDPC_BP_LHPRIO);
#pragma unroll
        for (int w = 0; w < W; ++w) F ^= fsl[w];
        if (F == B) {                                     // team-uniform
          uint32_t un = 0;
          for (int c = tid; c < m; c += TS) {
            const uint4 t0 = *(const uint4*)(a.rtab + 8 * (size_t)c);
            const uint4 t1 = *(const uint4*)(a.rtab + 8 * (size_t)c + 4);
            const uint32_t rv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
            uint32_t par = 0;
#pragma unroll
            for (int q = 0; q < DC; ++q) par ^= (uint32_t)(post[rv[q]] < 0.0);
            un |= par ^ ((synw[c >> 5] >> (c & 31)) & 1u);
          }
          if (!team_any(un != 0)) {
            iters = it + 1;
            conv = true;
            break;
          }
        }
      }
    }
    write_outputs_strided<4, TS>(a, hs, tid, [&](int v) { return post[v]; });   // (:280)
    const bool nonfin = team_any((fl & FLAG_NONFINITE) != 0);
    if (tid == 0) {
      a.iters[hs] = iters;
      if (a.flags) a.flags[hs] = (int32_t)((nonfin ? FLAG_NONFINITE : 0) | (conv ? FLAG_CONVERGED : 0));
      if (claimed) {
        red[2 * W + 2 * tphase] = tk;
        red[2 * W + 2 * tphase + 1] = tlen;
      }
    }
    __syncthreads();                                      // slice reuse; ticket visible
    if (!a.queue) {
      hs += stride;
    } else if (++hs >= end) {
      const uint32_t t0 = red[2 * W + 2 * tphase], l0 = red[2 * W + 2 * tphase + 1];
      tphase ^= 1;
      seen = t0 + l0;
      hs = stride + (long long)t0;
      end = hs + l0;
    }
  }
}

// ---------------------------------------------------------------------------
// Host-side launch helpers (called from capi.cpp)
// ---------------------------------------------------------------------------
// The BP team kernels and the flooding min-sum kernel are instantiated in
// translation units of their own (bp_team_kernels.hip, built without SLP
// vectorization; ms_flood_kernels.hip, built with the max-ILP machine
// scheduler); every other kernel here.
#if !defined(QLDPC_TU_BP_TEAM) && !defined(QLDPC_TU_FLOOD)
template <int ALGO, bool LAYERED, int DC>
static const void* kernel_ptr() {
  return (const void*)&decode_kernel<ALGO, LAYERED, DC>;
}

int ms_flood_max_waves(int kc) { return (kc >= 8 ? 512 : 256) / 64; }

// Kernel names as rocprofv3 reports them (bench.py matches profiles by name).
#define QLDPC_NAMED(ptr, str) do { if (name) *name = str; return (const void*)ptr; } while (0)

const void* select_ms_layered_kernel(int dc, int g, const char** name) {
#define QLDPC_MSL(D, Gn) if (dc == D && g == Gn) QLDPC_NAMED((&ms_layered_kernel<D, Gn>), "ms_layered_kernel<" #D ", " #Gn ">");
  QLDPC_MSL(7, 0) QLDPC_MSL(8, 0) QLDPC_MSL(7, 1) QLDPC_MSL(8, 1) QLDPC_MSL(7, 2) QLDPC_MSL(8, 2)
  QLDPC_MSL(7, 4) QLDPC_MSL(8, 4) QLDPC_MSL(7, 8) QLDPC_MSL(8, 8)
#undef QLDPC_MSL
  return nullptr;
}

const void* select_kernel(int algo, bool layered, int dc, const char** name) {
  static const char* names[2][2][3] = {
      {{"decode_kernel<0, false, 0>", "decode_kernel<0, false, 7>", "decode_kernel<0, false, 8>"},
       {"decode_kernel<0, true, 0>", "decode_kernel<0, true, 7>", "decode_kernel<0, true, 8>"}},
      {{"decode_kernel<1, false, 0>", "decode_kernel<1, false, 7>", "decode_kernel<1, false, 8>"},
       {"decode_kernel<1, true, 0>", "decode_kernel<1, true, 7>", "decode_kernel<1, true, 8>"}}};
  if (name) *name = names[algo == ALGO_MS ? 0 : 1][layered ? 1 : 0][dc == 7 ? 1 : (dc == 8 ? 2 : 0)];
#define QLDPC_PICK(ALG)                                                                 \
  switch (dc) {                                                                         \
    case 7: return layered ? kernel_ptr<ALG, true, 7>() : kernel_ptr<ALG, false, 7>();  \
    case 8: return layered ? kernel_ptr<ALG, true, 8>() : kernel_ptr<ALG, false, 8>();  \
    default: return layered ? kernel_ptr<ALG, true, 0>() : kernel_ptr<ALG, false, 0>(); \
  }
  if (algo == ALGO_MS) {
    QLDPC_PICK(ALGO_MS)
  } else {
    QLDPC_PICK(ALGO_BP)
  }
#undef QLDPC_PICK
}

hipError_t launch_decode(const void* kernel, const DecodeArgs& args, int grid, int block,
                         int lds_bytes, hipStream_t stream) {
  void* params[] = {(void*)&args};
  return hipLaunchKernel(kernel, dim3(grid), dim3(block), params, (size_t)lds_bytes, stream);
}

hipError_t configure_kernel(const void* kernel, int lds_bytes) {
  return hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
}

#elif defined(QLDPC_TU_FLOOD)

#define QLDPC_NAMED(ptr, str) do { if (name) *name = str; return (const void*)ptr; } while (0)

const void* select_ms_flood_kernel(int dc, int kc, const char** name) {
  // instantiated (DC, KC) shapes; the host passes ceil(m/64) checks per lane
  if (dc == 7 && kc <= 2) QLDPC_NAMED((&ms_flood_kernel<7, 2>), "ms_flood_kernel<7, 2>");
  if (dc == 8 && kc <= 2) QLDPC_NAMED((&ms_flood_kernel<8, 2>), "ms_flood_kernel<8, 2>");
  if (dc == 7 && kc <= 4) QLDPC_NAMED((&ms_flood_kernel<7, 4>), "ms_flood_kernel<7, 4>");
  if (dc == 8 && kc <= 4) QLDPC_NAMED((&ms_flood_kernel<8, 4>), "ms_flood_kernel<8, 4>");
  if (dc == 7 && kc <= 8) QLDPC_NAMED((&ms_flood_kernel<7, 8>), "ms_flood_kernel<7, 8>");
  if (dc == 8 && kc <= 8) QLDPC_NAMED((&ms_flood_kernel<8, 8>), "ms_flood_kernel<8, 8>");
  return nullptr;
}

#else  // QLDPC_TU_BP_TEAM

#define QLDPC_NAMED(ptr, str) do { if (name) *name = str; return (const void*)ptr; } while (0)

const void* select_bp_team_kernel(bool layered, int dc, int w, const char** name) {
#define QLDPC_BPT(L, D, Wn) \
  if (layered == L && dc == D && w == Wn) QLDPC_NAMED((&bp_team_kernel<L, D, Wn>), "bp_team_kernel<" #L ", " #D ", " #Wn ">");
  QLDPC_BPT(false, 7, 4) QLDPC_BPT(false, 8, 4) QLDPC_BPT(true, 7, 4) QLDPC_BPT(true, 8, 4)
  QLDPC_BPT(false, 7, 8) QLDPC_BPT(false, 8, 8) QLDPC_BPT(true, 7, 8) QLDPC_BPT(true, 8, 8)
#undef QLDPC_BPT
  return nullptr;
}

const void* select_bp_team_lg_kernel(int dc, int w, const char** name) {
  if (dc == 7 && w == 4) QLDPC_NAMED((&bp_team_lg_kernel<7, 4>), "bp_team_lg_kernel<7, 4>");
  if (dc == 8 && w == 4) QLDPC_NAMED((&bp_team_lg_kernel<8, 4>), "bp_team_lg_kernel<8, 4>");
  if (dc == 7 && w == 8) QLDPC_NAMED((&bp_team_lg_kernel<7, 8>), "bp_team_lg_kernel<7, 8>");
  if (dc == 8 && w == 8) QLDPC_NAMED((&bp_team_lg_kernel<8, 8>), "bp_team_lg_kernel<8, 8>");
  return nullptr;
}

#endif  // translation units

}  // namespace qldpc
