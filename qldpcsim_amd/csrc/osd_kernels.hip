// osd_kernels.hip — batched OSD post-decoding on MI355X (gfx950).
//
// Replaces OSDdec (qLDPCsim/decoders.py:299-370) with its gf2math.rank /
// gf2math.REF calls (gf2math.py:91-187) for a batch of non-converged shots.
// One workgroup = one shot; thread t owns row t of the column-permuted matrix
// Hp = H[:, perm] (perm = the reliability order, computed by the caller with
// NumPy exactly as decoders.py:320-325), held bit-packed in VGPRs, with the
// syndrome as an augmented column.
//
// Equivalences used (OSD):
//  * Gaussian elimination over the columns of Hp in order, pivot = first row at
//    or below the current pivot row holding a 1 (gf2math.REF's rule), finds a
//    pivot exactly in the columns that raise the rank — the greedy
//    complementary information set J of decoders.py:329-342 (plus column 0,
//    which the reference takes unconditionally).
//  * Non-pivot columns cause no row operation, so the row operations equal
//    those of REF(Hp[:, J], reduced=True); applied to the augmented syndrome
//    they give T @ s. With R = T @ Hp: T @ sJ = T @ s + R[:, I] @ e_I (mod 2),
//    so e_J = (T @ sJ)[:|J|] (decoders.py:352-358) needs one elimination.
//  * Order semantics with the reference's aliasing: order 1
//    flips e_perm[infoSet[0]] (CPython set order, emulated), order >= 2 is
//    order 0.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "osd_kernels.h"
#include "tuning.h"
#include "../../include/qldpc_libm.h"

namespace qldpc {

__device__ int first_setdiff(int n, const unsigned char* inJ, int nJ, int* table);

// a status-2 shot's posterior row into the spill buffer (OsdArgs), whole
// workgroup; `slot` is an LDS int the block may overwrite
__device__ __forceinline__ void spill_shot(const OsdArgs& a, long long shot, int n, int* slot) {
  if (!a.spill_count) return;
  if (threadIdx.x == 0) *slot = atomicAdd(a.spill_count, 1);
  __syncthreads();
  const long long q = *slot;
  if (q >= a.spill_cap) return;
  const double* src = a.post + shot * (long long)n;
  double* dst = a.spill_post + q * (long long)n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
  if (threadIdx.x == 0) a.spill_idx[q] = (int32_t)(a.shot_base + shot);
}

// Shots whose reliability order the device leaves to NumPy on the host
// (osd_order_kernel's tiepos -1: a NaN posterior, or x86-simd-sort's
// std::sort fallback): status 2, posteriors spilled, before any elimination.
__device__ __forceinline__ bool osd_host_shot(const OsdArgs& a, long long shot, int n, int* slot) {
  if (!a.tiepos || a.tiepos[shot] >= 0) return false;        // uniform per workgroup
  if (threadIdx.x == 0) a.status[shot] = 2;
  spill_shot(a, shot, n, slot);
  return true;
}

// s_getreg immediates: (size - 1) << 11 | offset << 6 | register id
constexpr int kHwRegHwId = (31 << 11) | 4;    // HW_ID: SIMD bits 4-5, CU 8-11, SH 12, SE 13-15
constexpr int kHwRegXccId = (31 << 11) | 20;  // XCC_ID: bits 0-3

template <int NW>
__global__ void __launch_bounds__(1024) osd_kernel(OsdArgs a) {
  // LDS: inv_perm[n] | J list [m+2] | inJ bytes [n] | emask [NW] u64 |
  //      candidate rows [2][16][NW] | xrow rows [2][NW] | candidate ids [2][16] |
  //      misc [4] | set table
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int m = a.m, n = a.n;
  int* inv = (int*)lds;
  int* Jl = inv + n;
  unsigned char* inJ = (unsigned char*)(Jl + m + 2);
  // offsets from `lds` itself (a cast through an integer would turn every
  // access below into a generic flat access instead of ds_read / ds_write)
  uint64_t* emask = (uint64_t*)(lds + ((4 * (n + m + 2) + n + 15) & ~15));
  uint64_t* cbuf = emask + NW;                     // [2][16][NW]
  uint64_t* xbuf = cbuf + 2 * 16 * NW;             // [2][NW]
  int* slots = (int*)(xbuf + 2 * NW);              // [2][16]
  int* misc = slots + 32;                          // [0]=|J| [1]=status [2]=first info index
  int* table = misc + 4;                           // CPython set emulation (order 1)

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6, nwaves = blockDim.x >> 6;
  const long long shot = blockIdx.x;
  if (a.redo && a.status[shot] != 3) return;       // second pass after osd_block_kernel
  if (!a.redo && osd_host_shot(a, shot, n, slots)) return;
  const int32_t* perm = a.perm + shot * (long long)n;
  const uint8_t* syn = a.syn + shot * (long long)m;
  uint8_t* ehat = a.ehat + shot * (long long)n;

  for (int i = t; i < n; i += blockDim.x) {
    inv[perm[i]] = i;
    inJ[i] = 0;
  }
  __syncthreads();

  // my row of Hp (+ syndrome bit at column n); thread t holds the row at
  // position t of REF's current row order (rows move by REF's swaps)
  uint64_t R[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) R[w] = 0;
  const bool own = t < m;
  if (own) {
    for (int e = a.row_ptr[t]; e < a.row_ptr[t + 1]; ++e) {
      const int i = inv[a.col_idx[e]];
#pragma unroll
      for (int w = 0; w < NW; ++w)
        if ((i >> 6) == w) R[w] |= 1ull << (i & 63);
    }
    if (syn[t] & 1) {
#pragma unroll
      for (int w = 0; w < NW; ++w)
        if ((n >> 6) == w) R[w] |= 1ull << (n & 63);
    }
  }

  int xrow = 0, rank = 0, nJ = 0, step = 0;
  bool done = a.rank == 0;                          // rank(H) = 0: IndexError below
  if (t == 0) {
    Jl[0] = 0;                                      // column 0 always (decoders.py:329)
    inJ[0] = 1;
  }
  nJ = 1;
  // One workgroup barrier per column. Before it, each wave's first candidate
  // row (a 1 in column i at a position >= xrow) and the row at position xrow
  // publish their words >= w; after it, every thread knows the pivot (the
  // smallest candidate position: REF's "first row at or below") and reads its
  // row from the winning wave's slot. Rows at positions >= xrow are zero in
  // every column < i (a nonzero there would have been a pivot), so words < w
  // never need to move. Two slot sets alternate: a wave writing set s at
  // column k+2 has passed column k+1's barrier, which every reader of column
  // k's set s had reached after its reads.
  // Fully unrolled over the NW words, so every R[w] / R[q] index is a
  // compile-time constant and the row stays in VGPRs (a runtime word index
  // would put R in scratch memory: one global access per touch).
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (done || 64 * w >= n) continue;
    for (int b = 0; b < 64; ++b) {
      const int i = 64 * w + b;
      if (i >= n || done) break;
      const bool has = own && ((R[w] >> b) & 1ull);
      const uint64_t bal = __ballot(has && t >= xrow);
      const int set = step & 1;
      uint64_t* cb = cbuf + (set * 16 + wave) * NW;
      uint64_t* xb = xbuf + set * NW;
      int* sl = slots + 16 * set;
      if (bal) {
        if (lane == __builtin_ctzll(bal)) {
#pragma unroll
          for (int q = w; q < NW; ++q) cb[q] = R[q];
          sl[wave] = t;
        }
      } else if (lane == 0) {
        sl[wave] = 0x7fffffff;
      }
      if (t == xrow) {
#pragma unroll
        for (int q = w; q < NW; ++q) xb[q] = R[q];
      }
      __syncthreads();
      int piv = 0x7fffffff;
      for (int q = 0; q < nwaves; ++q) piv = min(piv, sl[q]);
      ++step;
      if (piv == 0x7fffffff) continue;              // dependent column: not in J
      // pivot row `piv` moves to position xrow (REF's row swap), then every
      // other row holding a 1 in column i is XOR-ed with it (below and above)
      const uint64_t* pr = cbuf + (set * 16 + (piv >> 6)) * NW;
      if (t == piv && piv != xrow) {
#pragma unroll
        for (int q = w; q < NW; ++q) R[q] = xb[q];   // old row xrow: 0 in column i
      } else if (t == xrow) {
#pragma unroll
        for (int q = w; q < NW; ++q) R[q] = pr[q];
      } else if (has) {
#pragma unroll
        for (int q = w; q < NW; ++q) R[q] ^= pr[q];  // pivot row is 0 left of column i
      }
      if (i != 0) {
        if (t == 0) {
          Jl[nJ] = i;
          inJ[i] = 1;
        }
        ++nJ;
      }
      ++xrow;
      ++rank;
      if (rank >= a.rank || xrow >= m) done = true;
      if (i == 0 && done) rank = -1;                // column 0 alone reaches rank(H): the
    }                                               // greedy loop never breaks (:333-342)
  }
  if (rank < a.rank) {                              // greedy loop runs past column n-1
    if (t == 0) a.status[shot] = 1;                 // (the reference raises IndexError)
    return;
  }
  __syncthreads();
  // information-set values e_I (e_perm = e_hat[perm], decoders.py:345):
  // one column per thread, words assembled by ballots (all loads in flight)
  for (int i0w = 64 * wave; i0w < 64 * NW; i0w += blockDim.x) {
    const int i = i0w + lane;
    const bool bit = i < n && !inJ[i] && (ehat[perm[i]] & 1);
    const uint64_t bits = __ballot(bit);
    if (lane == 0) emask[i0w >> 6] = bits;
  }
  if (t == 0) {
    int i0 = -1;
    if (a.order == 1 && nJ < n) {
      // first element of CPython's set(range(n)) - set(J) (decoders.py:344)
      i0 = first_setdiff(n, inJ, nJ, table);
    }
    misc[2] = i0;
  }
  __syncthreads();
  const int i0 = misc[2];
  if (t == 0 && i0 >= 0) emask[i0 >> 6] ^= 1ull << (i0 & 63);  // order-1 flip (:349-350)
  __syncthreads();
  // e_J = (T sJ)[:|J|], T sJ = T s + R[:, I] e_I (mod 2)   (decoders.py:352-358)
  if (own && t < nJ) {
    uint64_t acc = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      if (w == (n >> 6)) acc ^= (R[w] >> (n & 63)) & 1ull;      // T s (augmented column)
      acc ^= (uint64_t)(__builtin_popcountll(R[w] & emask[w]) & 1);
    }
    ehat[perm[Jl[t]]] = (uint8_t)(acc & 1ull);                // e_hat[perm] = ... (:368)
  }
  if (t == 0)                                                  // (J past T sJ's m rows: 0, as
    for (int p = m; p < nJ; ++p) ehat[perm[Jl[p]]] = 0;        // the host OSD; osd_hbm_kernel)
  if (t == 0 && i0 >= 0) ehat[perm[i0]] ^= 1;
  if (t == 0) a.status[shot] = 0;
}

// ---------------------------------------------------------------------------
// Block elimination (the default GPU OSD): one workgroup barrier per 64-column
// word instead of one per column (osd_kernel spends most of its instructions
// on that per-column protocol). Thread t owns row t of Hp (+ syndrome).
//
// Pivot rows are chosen by row index (the first unused row holding a 1), not
// by REF's row order. That changes T but not what OSD reads from it: the
// pivot columns J are the columns independent of their predecessors (a
// property of Hp), and the fully reduced pivot row of column j_k gives the
// k-th entry of e_J = the unique solution of H_J x = s + H_I e_I (DESIGN.md
// §3, OSD). Two cases need REF's own order and go to osd_kernel instead: an
// all-zero column 0 (the host never selects this kernel for an H with a zero
// column) and a syndrome outside the column space of H (status 3 here, then
// osd_kernel redoes those shots in the same stream).
//
// Per word w:
//   A  every row publishes its word w
//   B  wave 0 runs the elimination over the 64 columns of word w alone on
//      that copy (row 64 s + lane in slot s): word value, and C = the set of
//      this block's pivot rows (by block-start value) XOR-ed into it so far.
//      Column i: pivot = first unused row with a 1 (ballots), every other row
//      with a 1 is XOR-ed with it: word ^= pivot word, C ^= C_pivot ^ {pivot}.
//      Columns no unused row holds are skipped unseen: XORs among unused rows
//      never set a bit that none of them held.
//   C  the block's pivot rows publish their words w.. (still block-start values)
//   D  every row applies its C to words w..: each update added a current
//      pivot row = its block-start value + earlier pivot rows of the block.
// ---------------------------------------------------------------------------
// x with lane `l` replaced by the wave-uniform v (v_writelane_b32)
__device__ __forceinline__ uint32_t write_lane(uint32_t x, uint32_t v, int l) {
  asm("v_writelane_b32 %0, %1, m0" : "+v"(x) : "s"(v), "{m0}"(l));   // (gfx9: one SGPR operand, lane in M0)
  return x;
}

__device__ __forceinline__ uint32_t wave_or32(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xf, 0xf, false);  // row_half_mirror
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xf, 0xf, false);  // row_mirror
  return (uint32_t)(__builtin_amdgcn_readlane((int)x, 0) | __builtin_amdgcn_readlane((int)x, 16) |
                    __builtin_amdgcn_readlane((int)x, 32) | __builtin_amdgcn_readlane((int)x, 48));
}

// Phase B over the columns `cols` of one half-word (HI: bits 32..63, read
// from hi[]) on the first SF compact slots, straight-line per column: one
// ballot per slot masked by the slot's still-free rows (fm[s], a wave-uniform
// lane mask in SGPRs); the slot that hits reads the pivot's values (readlane
// under its compile-time slot index: no dispatch on the slot afterwards) and
// clears the pivot's own column bit in the pivot row, so the elimination
// needs no per-slot exclusion of the pivot row: within the block the row's
// bits at this or earlier columns are never read again, and the engine's
// lo/hi words are dropped at the block end (only cl/ch leave it).
// Pivot k's compact position and column bit go to pk[k]; returns the pivot
// count K.
template <int SL, int SF, bool HI>
__device__ __forceinline__ int block_half(uint32_t (&lo)[SL], uint32_t (&hi)[SL], uint32_t (&cl)[SL],
                                          uint32_t (&ch)[SL], uint64_t (&fm)[SL], uint32_t cols, int K,
                                          int w, int lane, int& rank, int& nJ, bool& done, uint64_t& pivm,
                                          int rankH, int m, int& pkv) {
  while (cols && !done) {
    // loop-carried scalars re-asserted wave-uniform: otherwise the compiler
    // keeps them per lane and turns the loop into an exec-masked one
    cols = (uint32_t)__builtin_amdgcn_readfirstlane((int)cols);
    K = __builtin_amdgcn_readfirstlane(K);
    rank = __builtin_amdgcn_readfirstlane(rank);
    nJ = __builtin_amdgcn_readfirstlane(nJ);
    pivm = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pivm >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pivm);
    // next column with a pivot: slots scanned in ascending order, the scan
    // stops at the first hit (uniform branches) — once rows fill up, slot 0
    // almost always holds the pivot. Dependent columns (no free row holds
    // them) are skipped without touching the state; they are not in J.
    int f = -1, bit = 0;
    uint32_t plo = 0, phi = 0, pcl = 0, pch = 0;
    while (cols && f < 0) {
      bit = (int)__builtin_ctz(cols);
      cols &= cols - 1;
      const uint32_t bm = 1u << bit;
#pragma unroll
      for (int s = 0; s < SF; ++s) {
        const uint64_t c = __ballot(((HI ? hi[s] : lo[s]) & bm) != 0) & fm[s];
        if (c) {
          const int fl = (int)__builtin_ctzll(c);
          f = 64 * s + fl;
          plo = __builtin_amdgcn_readlane((int)lo[s], fl);
          phi = __builtin_amdgcn_readlane((int)hi[s], fl);
          pcl = __builtin_amdgcn_readlane((int)cl[s], fl);
          if (HI) pch = __builtin_amdgcn_readlane((int)ch[s], fl);
          fm[s] &= ~(1ull << fl);                     // no longer free
          if (HI) hi[s] = write_lane(hi[s], phi & ~bm, fl);
          else lo[s] = write_lane(lo[s], plo & ~bm, fl);
          break;
        }
      }
      f = __builtin_amdgcn_readfirstlane(f);
    }
    if (f < 0) break;                               // (dependent columns: not in J)
    // (+ the pivot itself; the 64-bit form, (pch:pcl) ^ (1ull << K), was
    // miscompiled in the 128-VGPR spilling instance: wrong eliminations,
    // correct at 3 waves per SIMD without spills — tools/osd_check.py)
    if (HI) {
      const uint32_t kb = 1u << (K & 31);
      pcl ^= K < 32 ? kb : 0u;
      pch ^= K < 32 ? 0u : kb;
    } else {
      pcl ^= 1u << K;                               // (low half: K < 32)
    }
    // Rows holding a 1 (above and below) take the pivot: x ^= p & mask with
    // mask = 0 / ~0 from the column bit (one bit-field extract) — branch-free
    // (v_bitop3), no exec-mask round trip from a VALU compare through SALU
    // per slot. The low half is done in HI. In the low half the block has
    // fewer than 32 pivots, so every C word's high half is still zero (no
    // ch update).
#pragma unroll
    for (int s = 0; s < SF; ++s) {
      const uint32_t mk = (uint32_t)__builtin_amdgcn_sbfe((int)(HI ? hi[s] : lo[s]), bit, 1);   // 0 / -1
      if (!HI) lo[s] ^= plo & mk;
      hi[s] ^= phi & mk;
      cl[s] ^= pcl & mk;
      if (HI) ch[s] ^= pch & mk;
    }
    const int wb = (HI ? 32 : 0) + bit;
    const int i = 64 * w + wb;
    pivm |= 1ull << wb;
    // pivot K's record (compact row << 6 | column bit) goes to lane K of a
    // VGPR (no exec-masked LDS store per pivot); the block's pk / Jl / inJ
    // entries are written once after the engine loop
    pkv = lane == K ? ((f << 6) | wb) : pkv;
    if (i != 0) ++nJ;
    ++K;
    ++rank;
    if (rank >= rankH || rank >= m) done = true;
    if (i == 0 && done) rank = -1;                  // column 0 alone reaches rank(H): the
                                                    // greedy loop never breaks (:333-342)
  }
  return K;
}

// block_half on the smallest power-of-two slot count >= SF (code per count)
template <int SL, int SFMAX, bool HI>
__device__ __forceinline__ int block_half_n(int SF, uint32_t (&lo)[SL], uint32_t (&hi)[SL], uint32_t (&cl)[SL],
                                            uint32_t (&ch)[SL], uint64_t (&fm)[SL], uint32_t cols, int K,
                                            int w, int lane, int& rank, int& nJ, bool& done, uint64_t& pivm,
                                            int rankH, int m, int& pkv) {
  if constexpr (SFMAX > 1) {
    if (SF <= SFMAX / 2)
      return block_half_n<SL, SFMAX / 2, HI>(SF, lo, hi, cl, ch, fm, cols, K, w, lane, rank, nJ, done, pivm,
                                             rankH, m, pkv);
  }
  return block_half<SL, SFMAX, HI>(lo, hi, cl, ch, fm, cols, K, w, lane, rank, nJ, done, pivm, rankH, m, pkv);
}

// XOR of the 64-bit table entries tab[k] over the set bits k of v, four
// gathers in flight per trip
__device__ __forceinline__ uint64_t osd_gather_xor4(const uint64_t* tab, uint64_t v) {
  uint64_t acc = 0;
  while (v) {
    int k[4];
    uint64_t mk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mk[j] = v ? ~0ull : 0ull;
      k[j] = v ? (int)__builtin_ctzll(v) : 0;
      v &= v - 1;
    }
    uint64_t c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = tab[k[j]];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= c[j] & mk[j];
  }
  return acc;
}

template <int NW, int W0>
__device__ __forceinline__ void osd_apply_from(uint64_t (&R)[NW], uint64_t cm, const uint64_t* PW, const uint64_t* PX) {
  // a pivot row's words W0.. in one read batch, or in two when more than
  // QLDPC_OSD_DSPLIT words remain: the peak register need of phase D is the
  // rows' state plus one batch. QLDPC_OSD_PAIRS: pivots taken two at a time
  // (k = 2j, 2j + 1), PX[j] = PW[2j] ^ PW[2j + 1]: one row read per nonzero
  // pair of cm's bits instead of one per bit
  constexpr int NB = NW - W0, B1 = (QLDPC_OSD_DSPLIT > 0 && NB > QLDPC_OSD_DSPLIT) ? (NB + 1) / 2 : NB;
  uint64_t it = QLDPC_OSD_PAIRS ? (cm | (cm >> 1)) & 0x5555555555555555ull : cm;
  while (it) {
    const int k = (int)__builtin_ctzll(it);
    it &= it - 1;
    const uint64_t* src;
    if constexpr (QLDPC_OSD_PAIRS != 0) {
      const int b = (int)(cm >> k) & 3;
      src = b == 3 ? PX + (k >> 1) * NW : PW + (k + (b >> 1)) * NW;
    } else {
      src = PW + k * NW;
    }
    uint64_t v[B1];
#pragma unroll
    for (int x = 0; x < B1; ++x) v[x] = src[W0 + x];
#pragma unroll
    for (int x = 0; x < B1; ++x) R[W0 + x] ^= v[x];
    if constexpr (B1 < NB) {
      uint64_t u[NB - B1];
#pragma unroll
      for (int x = 0; x < NB - B1; ++x) u[x] = src[W0 + B1 + x];
#pragma unroll
      for (int x = 0; x < NB - B1; ++x) R[W0 + B1 + x] ^= u[x];
    }
  }
}

// R[x] ^= PW[k][x] for x >= w and every set bit k of cm (w wave-uniform)
template <int NW, int W0 = 0>
__device__ __forceinline__ void osd_apply_rows(uint64_t (&R)[NW], uint64_t cm, const uint64_t* PW, const uint64_t* PX,
                                               int w) {
  if constexpr (W0 < NW) {
    if (w == W0) osd_apply_from<NW, W0>(R, cm, PW, PX);
    else osd_apply_rows<NW, W0 + 1>(R, cm, PW, PX, w);
  }
}

// SL = rows per wave-0 lane (m <= 64 SL), sized to the code so the state stays
// in VGPRs; RT = rows per thread (thread t holds rows t, t + blockDim, ..):
// with 2, a 450-row shot takes 4 waves and a CU holds 4 shots (4 engines, one
// per SIMD) instead of 2
template <int NW, int SL, int RT>
__global__ void __launch_bounds__(64 * SL / RT) __attribute__((amdgpu_waves_per_eu(RT == 2 ? QLDPC_OSD_WPE : 1))) osd_block_kernel(OsdArgs a) {
  // LDS: inv_perm[n] | J list [m+2] | inJ bytes [n] | emask [NW] | Wd [MR] | Cm [MR] |
  //      PW [64][NW] | PX [32][NW] (QLDPC_OSD_PAIRS) | CT [64] | pkof [MR] | pidx [MR] | crow [MR] | pk [64] | misc [16] | set table
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int m = a.m, n = a.n;
  const int B = blockDim.x, MR = RT * B;
  int* inv = (int*)lds;
  int* Jl = inv + n;
  unsigned char* inJ = (unsigned char*)(Jl + m + 2);
  uint64_t* emask = (uint64_t*)(lds + ((4 * (n + m + 2) + n + 15) & ~15));
  uint64_t* Wd = emask + NW;
  uint64_t* Cm = Wd + MR;
  uint64_t* PW = Cm + MR;                            // [64][NW]
  uint64_t* PX = PW + 64 * NW;                       // [32][NW] pivot pairs (QLDPC_OSD_PAIRS)
  uint64_t* CT = PX + (QLDPC_OSD_PAIRS ? 32 * NW : 0);   // C of this block's pivot by its column bit
  int* pkof = (int*)(CT + 64);                       // pivot tag per row: 64 w + k, -1 none
  int* pidx = pkof + MR;                             // pivot index of each row (m: none)
  int* crow = pidx + MR;                             // compact position -> row (free rows)
  int* pk = crow + MR;                               // pivot k: compact position << 6 | column bit
  int* misc = pk + 64;                               // [0] nJ [1] rank [2] i0 [3] flag [4] done [5] K
                                                     // [6..7] this block's pivot-column mask
                                                     // [8..11] SIMD of each wave [12] engine SIMD
  int* table = misc + 16;

  const int t = threadIdx.x;
  // readfirstlane: `wave` is then known to be wave-uniform, so the engine's
  // branch is scalar and the counters it updates stay in SGPRs
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const long long shot = blockIdx.x;
  if (osd_host_shot(a, shot, n, misc + 7)) return;
  const int32_t* perm = a.perm + shot * (long long)n;
  const uint8_t* syn = a.syn + shot * (long long)m;
  uint8_t* ehat = a.ehat + shot * (long long)n;

  for (int i = t; i < n; i += blockDim.x) {
    inv[perm[i]] = i;
    inJ[i] = 0;
  }
#pragma unroll
  for (int h = 0; h < RT; ++h) {
    pkof[t + h * B] = -1;
    pidx[t + h * B] = m;
  }
  // Phase B runs on one "engine" wave while the workgroup's other waves wait
  // at the barrier, and a CU runs 4 shots (workgroups) whose 4 waves sit on
  // its 4 SIMDs, wave 0 on a SIMD that rotates between workgroups: engines of
  // co-resident shots often shared a SIMD. Each workgroup takes a per-CU
  // ticket and runs its engine on the wave placed on SIMD (ticket mod 4), so
  // the engines of 4 consecutive workgroups of a CU use 4 SIMDs.
  if (lane == 0 && wave < 4) misc[8 + wave] = (int)((__builtin_amdgcn_s_getreg(kHwRegHwId) >> 4) & 3u);
  if (t == 0) {
    misc[3] = 0;
    uint32_t tk = 0;
    if (a.cu_tickets) {
      const uint32_t hw = __builtin_amdgcn_s_getreg(kHwRegHwId), xcc = __builtin_amdgcn_s_getreg(kHwRegXccId);
      tk = atomicAdd(a.cu_tickets + (((xcc & 15u) << 8) | ((hw >> 8) & 0xffu)), 1u);
    }
    misc[12] = (int)(tk & 3u);
  }
  __syncthreads();
  int engine = 0;
  {
    const int target = misc[12], nwv = (int)(blockDim.x >> 6);
    for (int w = 0; w < 4 && w < nwv; ++w)
      if (misc[8 + w] == target) engine = w;
    engine = __builtin_amdgcn_readfirstlane(engine);
  }

  // my rows of Hp (+ syndrome bit at column n)
  uint64_t R[RT][NW];
  bool own[RT];
#pragma unroll
  for (int h = 0; h < RT; ++h) {
    const int r = t + h * B;
    own[h] = r < m;
#pragma unroll
    for (int w = 0; w < NW; ++w) R[h][w] = 0;
    if (own[h]) {
      for (int e = a.row_ptr[r]; e < a.row_ptr[r + 1]; ++e) {
        const int i = inv[a.col_idx[e]];
#pragma unroll
        for (int w = 0; w < NW; ++w)
          if ((i >> 6) == w) R[h][w] |= 1ull << (i & 63);
      }
      if (syn[r] & 1) {
#pragma unroll
        for (int w = 0; w < NW; ++w)
          if ((n >> 6) == w) R[h][w] |= 1ull << (n & 63);
      }
    }
  }

  int rank = 0, nJ = 1;
  bool done = a.rank == 0;                            // rank(H) = 0: IndexError below
  if (t == 0) {
    Jl[0] = 0;                                        // column 0 always (decoders.py:329)
    inJ[0] = 1;
  }

  // runtime block loop (one copy of phase B); R is only ever indexed by the
  // compile-time x of the unrolled word loops, so it stays in VGPRs
  unsigned long long tp[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long tc = QLDPC_OSD_TIMING ? clock64() : 0;
#define QLDPC_TICK(k)                            \
  if constexpr (QLDPC_OSD_TIMING != 0) {         \
    const unsigned long long now = clock64();    \
    tp[k] += now - tc;                           \
    tc = now;                                    \
  }
  QLDPC_TICK(0);                                      // setup
  for (int w = 0; w < NW && 64 * w < n && !done; ++w) {   // done: uniform, re-read per block
#pragma unroll
    for (int h = 0; h < RT; ++h)                      // A
      if (own[h]) {
        uint64_t v = 0;
#pragma unroll
        for (int x = 0; x < NW; ++x)
          if (x == w) v = R[h][x];
        Wd[t + h * B] = v;
      }
    __syncthreads();
    QLDPC_TICK(1);
    if (wave == engine) {                             // B
      // The engine is its shot's critical path while the SIMD also runs
      // other shots' phase-D waves: raised priority lets it issue first.
      if constexpr (QLDPC_OSD_PRIO != 0) __builtin_amdgcn_s_setprio(QLDPC_OSD_PRIO);
      // the engine works on the rows still free (no pivot yet), compacted:
      // crow[c] = the c-th free row; earlier pivots are reduced in phase D
      const int rank0 = rank;
      int F = 0;
      // every read of a slot loop issued before the first use (left alone,
      // each slot's read sat in its own exec-masked block with its own wait:
      // 8 dependent LDS round trips on the engine's chain, twice per block)
      int pv[SL];
#pragma unroll
      for (int s = 0; s < SL; ++s) pv[s] = pidx[64 * s + lane];     // (64 SL = MR row slots)
#pragma unroll
      for (int s = 0; s < SL; ++s) asm volatile("" : "+v"(pv[s]));
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const int row = 64 * s + lane;
        const bool fr = row < m && pv[s] == m;
        const uint64_t bf = __ballot(fr);
        if (fr) crow[F + __builtin_amdgcn_mbcnt_hi((uint32_t)(bf >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bf, 0))] = row;
        F += __builtin_popcountll(bf);
      }
      uint32_t lo[SL], hi[SL], cl[SL], ch[SL];
      uint64_t fm[SL];                                // slot s: lanes whose compact row is not yet a pivot
      uint32_t alo = 0, ahi = 0;                      // columns some free row holds
      int cr[SL];
#pragma unroll
      for (int s = 0; s < SL; ++s) cr[s] = crow[64 * s + lane];     // (this wave's writes above: in order)
#pragma unroll
      for (int s = 0; s < SL; ++s) asm volatile("" : "+v"(cr[s]));
      uint64_t wv[SL];
#pragma unroll
      for (int s = 0; s < SL; ++s) wv[s] = Wd[64 * s + lane < F ? cr[s] : 0];
#pragma unroll
      for (int s = 0; s < SL; ++s) asm volatile("" : "+v"(wv[s]));
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const int cp = 64 * s + lane;
        const uint64_t v = cp < F ? wv[s] : 0ull;
        lo[s] = (uint32_t)v;
        hi[s] = (uint32_t)(v >> 32);
        cl[s] = ch[s] = 0;
        fm[s] = __ballot(cp < F);
        alo |= lo[s];
        ahi |= hi[s];
      }
      uint64_t cols = ((uint64_t)wave_or32(ahi) << 32) | wave_or32(alo);
      if (n - 64 * w < 64) cols &= (1ull << (n - 64 * w)) - 1;
      if constexpr ((QLDPC_ABLATE_OSD & 2) != 0) cols = 0;
      const int SF = (F + 63) >> 6;
      uint64_t pivm = 0;
      // low half-word columns, then high (each loop's column order ascends)
      const int nJ0 = nJ;
      int pkv = 0;
      int K = block_half_n<SL, SL, false>(SF, lo, hi, cl, ch, fm, (uint32_t)cols, 0, w, lane, rank, nJ, done,
                                          pivm, a.rank, m, pkv);
      K = block_half_n<SL, SL, true>(SF, lo, hi, cl, ch, fm, (uint32_t)(cols >> 32), K, w, lane, rank, nJ, done,
                                     pivm, a.rank, m, pkv);
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const int cp = 64 * s + lane;
        if (cp < F) Cm[crow[cp]] = ((uint64_t)ch[s] << 32) | cl[s];
      }
      // (one wave: its LDS accesses complete in order, so the reads below see
      // the writes above)
      {
        // the block's J entries (column 0 is J's first entry from the start)
        const int ivv = 64 * w + (pkv & 63);
        const int z = (K > 0 && __builtin_amdgcn_readlane(ivv, 0) == 0) ? 1 : 0;
        if (lane < K) {
          pk[lane] = pkv;
          if (ivv != 0) {
            Jl[nJ0 + lane - z] = ivv;
            inJ[ivv] = 1;
          }
          const int e = pkv;
          const int row = crow[e >> 6];
          CT[e & 63] = Cm[row] ^ (1ull << lane);      // reduced pivot k = its own row + C
          pkof[row] = 64 * w + lane;
          pidx[row] = rank0 + lane;                   // REF moves the k-th pivot row to row k
        }
        if (lane == 0) {
          misc[0] = nJ;
          misc[1] = rank;
          misc[4] = done;
          misc[5] = K;
          misc[6] = (int)(uint32_t)pivm;
          misc[7] = (int)(uint32_t)(pivm >> 32);
        }
      }
      if constexpr (QLDPC_OSD_PRIO != 0) __builtin_amdgcn_s_setprio(0);
    }
    QLDPC_TICK(2);
    __syncthreads();
    QLDPC_TICK(3);
    nJ = __builtin_amdgcn_readfirstlane(misc[0]);    // (LDS loads count as per-lane values)
    rank = __builtin_amdgcn_readfirstlane(misc[1]);
    done = __builtin_amdgcn_readfirstlane(misc[4]) != 0;
    const int K = __builtin_amdgcn_readfirstlane(misc[5]);
    const uint64_t pivm = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(misc[7]) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane(misc[6]);
    // C: pivot rows publish their words w.. as they were at the block start
    int tag[RT];
#pragma unroll
    for (int h = 0; h < RT; ++h) {
      tag[h] = own[h] ? pkof[t + h * B] : -1;
      if (tag[h] >= 0 && (tag[h] >> 6) == w) {
        uint64_t* dst = PW + (tag[h] & 63) * NW;
#pragma unroll
        for (int x = 0; x < NW; ++x)
          if (x >= w) dst[x] = R[h][x];
      }
    }
    __syncthreads();
    if constexpr (QLDPC_OSD_PAIRS != 0) {
      // pair rows PX[j] = PW[2j] ^ PW[2j + 1], words w.. (pairs of this block's pivots)
      if (K > 1) {                                    // (uniform)
        const int np = K >> 1, nx = NW - w;
        for (int i = t; i < np * nx; i += B) {
          const int j = i / nx, x = w + i - j * nx;
          PX[j * NW + x] = PW[2 * j * NW + x] ^ PW[(2 * j + 1) * NW + x];
        }
        __syncthreads();
      }
    }
    QLDPC_TICK(4);
    // D: every row applies its combination of this block's pivot rows
#pragma unroll
    for (int h = 0; h < RT; ++h)
    if (own[h] && K > 0 && (QLDPC_ABLATE_OSD & 1) == 0) {
      uint64_t cm;
      if (tag[h] >= 0 && (tag[h] >> 6) < w) {
        // a pivot row of an earlier block: clear this block's pivot columns
        // from it. Its result is unique (word w + the reduced block pivots it
        // holds a 1 for), so C = XOR of those pivots' C (no engine pass).
        uint64_t v = 0;
#pragma unroll
        for (int x = 0; x < NW; ++x)
          if (x == w) v = R[h][x];
        cm = osd_gather_xor4(CT, v & pivm);
      } else {
        cm = Cm[t + h * B];
      }
      // (per-lane gathers of the pivot rows: a uniform loop over all K with
      // broadcast reads measured 2x slower, VALU-bound). The word range is a
      // compile-time one per block (switch on w), so a pivot row's words are
      // all read before any XOR — one LDS round trip per pivot row instead
      // of one per word behind a uniform branch.
      osd_apply_rows<NW>(R[h], cm, PW, PX, w);
    }
    QLDPC_TICK(5);
  }
  if constexpr (QLDPC_OSD_TIMING != 0) {
    if (lane == 0 && (wave == engine || wave == (engine ^ 1)))   // [0]: the engine wave, [1]: another
      for (int k = 0; k < 6; ++k) atomicAdd(a.prof + 8 * (wave == engine ? 0 : 1) + k, tp[k]);
  }
#undef QLDPC_TICK
  if (rank < a.rank) {                              // greedy loop runs past column n-1
    if (t == 0) a.status[shot] = 1;                 // (the reference raises IndexError)
    return;
  }
  // a row left without pivot is zero on every column of H; a 1 in its
  // syndrome column means s is outside H's column space (status 3)
  int mypos[RT];
#pragma unroll
  for (int h = 0; h < RT; ++h) {
    mypos[h] = own[h] ? pidx[t + h * B] : m;
    uint64_t sbit = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w)
      if (w == (n >> 6)) sbit = (R[h][w] >> (n & 63)) & 1ull;   // (compile-time R index)
    if (own[h] && mypos[h] >= nJ && sbit) misc[3] = 1;
  }
  if (t == 0) {
    int i0 = -1;
    if (a.order == 1 && nJ < n) i0 = first_setdiff(n, inJ, nJ, table);   // (decoders.py:344)
    misc[2] = i0;
  }
  __syncthreads();
  const int i0 = misc[2];
  if (misc[3]) {
    if (t == 0) a.status[shot] = 3;
    return;
  }
  // information-set values e_I (e_perm = e_hat[perm], decoders.py:345)
  for (int i0w = 64 * wave; i0w < 64 * NW; i0w += blockDim.x) {
    const int i = i0w + lane;
    const bool bit = i < n && !inJ[i] && (ehat[perm[i]] & 1);
    const uint64_t bits = __ballot(bit);
    if (lane == 0) emask[i0w >> 6] = bits;
  }
  __syncthreads();
  if (t == 0 && i0 >= 0) emask[i0 >> 6] ^= 1ull << (i0 & 63);   // order-1 flip (:349-350)
  __syncthreads();
  // e_J = (T sJ)[:|J|]: the k-th pivot row gives entry k   (decoders.py:352-358)
#pragma unroll
  for (int h = 0; h < RT; ++h)
    if (own[h] && mypos[h] < nJ) {
      uint64_t acc = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        if (w == (n >> 6)) acc ^= (R[h][w] >> (n & 63)) & 1ull;   // T s (augmented column)
        acc ^= (uint64_t)(__builtin_popcountll(R[h][w] & emask[w]) & 1);
      }
      ehat[perm[Jl[mypos[h]]]] = (uint8_t)(acc & 1ull);         // e_hat[perm] = ... (:368)
    }
  if (t == 0 && i0 >= 0) ehat[perm[i0]] ^= 1;
  if (t == 0) a.status[shot] = 0;
}

// ---------------------------------------------------------------------------
// Reliability order of one shot per wavefront: NumPy's own (decoders.py:
// 320-325), bit for bit and tie for tie. Keys by qldpc_osd_key_t (SVML exp8_ha
// restated, include/qldpc_libm.h); the order by x86-simd-sort's argsort as
// NumPy 2.2.6 dispatches it on AVX512_SKX (np_order.cpp states the algorithm
// and is its host twin). LDS holds the keys and indices in their current
// arrangement (both move together); segments come off a small stack:
//   * > 256 keys (argpartition_unrolled<4>): the pivot (5th smallest of 8
//     samples, every lane sorts the same 8); the (size % 32) scalar steps as a
//     walk over two 32-lane streams (left end, right end) whose comparisons
//     are one ballot — a scalar loop assigns each touched key its slot; the
//     32-aligned middle as ballots per 64-key row (8 vectors); x86-simd-sort's
//     block schedule (left or right end, by the store counts so far) as a
//     scalar loop over the blocks' counts held in lanes (readlane), giving each
//     8-key vector its store offsets; every key to its slot;
//   * <= 256 keys (argsort_n): the bitonic network in registers, 4 keys per
//     lane, flip + half-cleaner stages over max(8, 2^ceil) slots with +inf
//     pads; comparators swap only when the upper key is strictly smaller.
// tiepos = n for an exact order, -1 where NumPy's order is left to the host:
// a NaN key, or x86-simd-sort's std::sort fallback after 2 floor(log2 n)
// levels (not restated).
// ---------------------------------------------------------------------------
__constant__ double kExpHL[32] = QLDPC_EXP_HL_INIT;

// A key and its index travel as one 64-bit word: w = u << 11 | i, u =
// bits(key) - bits(0.5) (key in [0.5, 1]: u <= 2^52, order-preserving), i < 2048.
// Comparisons look at the key part only — equal keys compare equal whatever
// their indices, exactly as x86-simd-sort compares the float64 keys:
//   key(b) < key(a)  <=>  (b | 0x7ff) < (a & ~0x7ff)
constexpr uint64_t kOrdIdx = 0x7ffull;
__device__ __forceinline__ bool ord_less(uint64_t b, uint64_t a) { return (b | kOrdIdx) < (a & ~kOrdIdx); }

// compare-exchange of two registers of one lane (positions lo < hi)
__device__ __forceinline__ void ord_cx(uint64_t& lo, uint64_t& hi) {
  const bool sw = ord_less(hi, lo);
  const uint64_t t = lo;
  lo = sw ? hi : lo;
  hi = sw ? t : hi;
}

// within-lane stage: partner position x ^ M, M in {1, 2, 3}. Every stage is
// a compile-time instance: with the partner pattern a run-time value, the
// compiler kept the four words in scratch memory and addressed them by it.
template <int M>
__device__ __forceinline__ void ord_within(uint64_t (&w)[4]) {
  if constexpr (M == 1) {
    ord_cx(w[0], w[1]);
    ord_cx(w[2], w[3]);
  } else if constexpr (M == 2) {
    ord_cx(w[0], w[2]);
    ord_cx(w[1], w[3]);
  } else {
    ord_cx(w[0], w[3]);
    ord_cx(w[1], w[2]);
  }
}

// cross-lane stage: partner position x ^ m, m >= 4: lane ^ LM (LM = m >> 2),
// register r ^ M3 (M3 = m & 3); HB = the highest bit of LM decides which side
// is the lower position
template <int LM, int HB, int M3>
__device__ __forceinline__ void ord_cross(uint64_t (&w)[4], int lane) {
  const bool lo = (lane & HB) == 0;
  uint64_t nw[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint64_t pw = __shfl_xor(w[r ^ M3], LM, 64);
    const bool take = lo ? ord_less(pw, w[r]) : ord_less(w[r], pw);
    nw[r] = take ? pw : w[r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) w[r] = nw[r];
}

// half-cleaners J, J/2 .. 1
template <int J>
__device__ __forceinline__ void ord_half(uint64_t (&w)[4], int lane) {
  if constexpr (J >= 4) ord_cross<J / 4, J / 4, 0>(w, lane);
  else if constexpr (J >= 1) ord_within<J>(w);
  if constexpr (J > 1) ord_half<J / 2>(w, lane);
}

// bitonic merge of blocks of KK: flip(KK), then half-cleaners KK/4 .. 1
template <int KK>
__device__ __forceinline__ void ord_merge(uint64_t (&w)[4], int lane) {
  if constexpr (KK <= 4) ord_within<KK - 1>(w);              // flip(2) = x ^ 1, flip(4) = x ^ 3
  else ord_cross<(KK - 1) / 4, KK / 8, 3>(w, lane);          // flip(KK) = x ^ (KK - 1)
  if constexpr (KK >= 4) ord_half<KK / 4>(w, lane);
}

// argsort_n on positions [L, L + N), N <= 256, in registers
__device__ __forceinline__ void ord_small(uint64_t* W, int L, int N, int lane) {
  uint64_t w[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int x = 4 * lane + r;
    const uint64_t v = W[L + (x < N ? x : 0)];
    w[r] = x < N ? v : ~0ull;                               // +inf pads
  }
  // stages up to P = max(8, 2^ceil(log2 N)) (uniform branches)
  ord_merge<2>(w, lane);
  ord_merge<4>(w, lane);
  ord_merge<8>(w, lane);
  if (N > 8) ord_merge<16>(w, lane);
  if (N > 16) ord_merge<32>(w, lane);
  if (N > 32) ord_merge<64>(w, lane);
  if (N > 64) ord_merge<128>(w, lane);
  if (N > 128) ord_merge<256>(w, lane);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int x = 4 * lane + r;
    if (x < N) W[L + x] = w[r];
  }
}

__device__ __forceinline__ void ord_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

template <int EPL>                                          // keys per lane capacity: n <= 64 EPL
__global__ void __launch_bounds__(64) osd_order_kernel(OrderArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int n = a.n;
  uint64_t* W = (uint64_t*)lds;                              // [n] (key, index) words, current arrangement
  int* stk = (int*)(W + n);                                  // [32][3] (L, R, iters)
  uint16_t* VL = (uint16_t*)(stk + 96);                      // [256] per vector: lt store base
  uint16_t* VR = VL + 256;                                   // [256] per vector: ge store end
  const int lane = threadIdx.x;
  const long long shot = blockIdx.x;
  const double* post = a.post + shot * (long long)n;
  int32_t* perm = a.perm + shot * (long long)n;

  bool nan = false;
  for (int i = lane; i < n; i += 64) {
    const double k = qldpc_osd_key_t(post[i], kExpHL);
    nan |= k != k;
    W[i] = ((__builtin_bit_cast(uint64_t, k) - 0x3FE0000000000000ull) << 11) | (uint64_t)i;
  }
  bool fallback = __ballot(nan) != 0;                        // std_argsort_withnan: the host's
  int lg = 0;
  while ((2 << lg) <= n) ++lg;                               // floor(log2 n)
  int sp = 0;
  if (n > 1 && !fallback) {
    if (lane == 0) {
      stk[0] = 0;
      stk[1] = n - 1;
      stk[2] = 2 * lg;
    }
    sp = 1;
  }
  ord_fence();
  while (sp > 0 && !fallback) {
    --sp;
    const int L = __builtin_amdgcn_readfirstlane(stk[3 * sp]);
    const int R = __builtin_amdgcn_readfirstlane(stk[3 * sp + 1]);
    const int it = __builtin_amdgcn_readfirstlane(stk[3 * sp + 2]);
    if (it <= 0) {                                           // argsort_64bit_: std_argsort
      fallback = true;
      break;
    }
    if (R + 1 - L <= 256) {
      if constexpr ((QLDPC_ABLATE_ORD & 1) == 0) ord_small(W, L, R + 1 - L, lane);
      ord_fence();
      continue;
    }
    if constexpr ((QLDPC_ABLATE_ORD & 2) != 0) continue;
    // ---- argpartition_unrolled<4> ----
    // pivot: the 5th smallest key of the 8 samples (every lane sorts the same
    // words; equal keys in any order give the same key)
    const int q = (R - L) >> 3;
    uint64_t sm[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sm[i] = W[L + q * (i + 1)];
#pragma unroll
    for (int i = 1; i < 8; ++i)
#pragma unroll
      for (int j = i; j > 0; --j) {
        const uint64_t lo = sm[j - 1], hi = sm[j];
        sm[j - 1] = lo < hi ? lo : hi;
        sm[j] = lo < hi ? hi : lo;
      }
    const uint64_t pf = sm[4] & ~kOrdIdx;                    // key < pivot <=> w < pf
    const uint64_t pc = pf | kOrdIdx;                        // key > pivot <=> w > pc
    bool lt = false, gt = false;
    int left = L, right = R + 1;
    const int rem = (R + 1 - L) & 31;
    if (rem) {
      // the scalar steps: examine the key at `left`; < pivot: it stays, left
      // advances (the next key is the next of the left stream); >= pivot: it
      // swaps with the key at --right (the right stream's next), which is
      // examined next. Lane i < 32 holds left-stream key i (position L + i),
      // lane 32 + i right-stream key i (position R - i).
      const int pos = lane < 32 ? L + lane : R - (lane - 32);
      const uint64_t wv = W[pos];
      const uint64_t ltm = __ballot(wv < pf);
      int cur = 0, dest = -1;
      bool ex = false;
      for (int s = 0; s < rem; ++s) {
        if (lane == cur) ex = true;
        if ((ltm >> cur) & 1ull) {
          if (lane == cur) dest = left;
          ++left;
          cur = left - L;
        } else {
          --right;
          if (lane == cur) dest = right;
          cur = 32 + (R - right);
        }
      }
      if (lane == cur) dest = left;                          // moved to `left`, not examined
      lt |= ex && wv < pf;
      gt |= ex && wv > pc;
      if (dest >= 0) W[dest] = wv;
      ord_fence();
    }
    // the 32-aligned middle [left, right): rows of 64 keys (8 vectors)
    const int M = right - left, nb = M >> 5;
    uint64_t ev[EPL];
    uint32_t byt[(EPL + 3) / 4];                             // row r's vector byte at bits 8 (r % 4)
    uint32_t mym = 0;
#pragma unroll
    for (int r = 0; r < EPL; ++r) {
      if (64 * r >= M) break;
      const int o = 64 * r + lane;
      ev[r] = W[left + (o < M ? o : 0)];
    }
#pragma unroll
    for (int r = 0; r < EPL; ++r) {
      if (64 * r >= M) break;
      const bool valid = 64 * r + lane < M;
      lt |= valid && ev[r] < pf;
      gt |= valid && ev[r] > pc;
      const uint64_t bm = __ballot(valid && ev[r] >= pf);
      if ((lane >> 1) == r) mym = (lane & 1) ? (uint32_t)(bm >> 32) : (uint32_t)bm;
      const uint32_t by = (uint32_t)(bm >> (lane & 56)) & 0xffu;
      byt[r / 4] = (r % 4 ? byt[r / 4] : 0u) | (by << (8 * (r % 4)));
    }
    // x86-simd-sort's block schedule: blocks 1 .. nb-2 from the left or the
    // right end, then the held-back first and last blocks
    const int g = __builtin_popcount(mym);                   // lane b: >= pivot keys of block b
    int lsto = left, rend = right, lp = left + 32, rp = right - 32;
    int myl = 0, myr = 0;
    for (int step = 0; step < nb; ++step) {
      int b;
      if (step < nb - 2) {
        if (rend - rp < lp - lsto) {
          rp -= 32;
          b = (rp - left) >> 5;
        } else {
          b = (lp - left) >> 5;
          lp += 32;
        }
      } else {
        b = step == nb - 2 ? 0 : nb - 1;
      }
      if (lane == b) {
        myl = lsto;
        myr = rend;
      }
      const int gb = __builtin_amdgcn_readlane(g, b);
      lsto += 32 - gb;
      rend -= gb;
    }
    const int pidx = lsto;
    if (lane < nb) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int c = __builtin_popcount((mym >> (8 * ii)) & 0xffu);
        VL[4 * lane + ii] = (uint16_t)myl;
        VR[4 * lane + ii] = (uint16_t)myr;
        myl += 8 - c;
        myr -= c;
      }
    }
    ord_fence();
#pragma unroll
    for (int r = 0; r < EPL; ++r) {
      if (64 * r >= M) break;
      const int o = 64 * r + lane;
      const int v = o < M ? o >> 3 : 0;
      const int vl = VL[v], vr = VR[v];
      if (o < M) {
        const int kk = o & 7;
        const uint32_t byte = (byt[r / 4] >> (8 * (r % 4))) & 0xffu;
        const uint32_t below = byte & ((1u << kk) - 1u);
        const int dst = (byte >> kk) & 1u ? vr - __builtin_popcount(byte) + __builtin_popcount(below)
                                          : vl + kk - __builtin_popcount(below);
        W[dst] = ev[r];
      }
    }
    ord_fence();
    // children: pivot != smallest -> the left part, pivot != biggest -> the right part
    const bool lany = __ballot(lt) != 0, gany = __ballot(gt) != 0;
    if (lane == 0) {
      if (lany) {
        stk[3 * sp] = L;
        stk[3 * sp + 1] = pidx - 1;
        stk[3 * sp + 2] = it - 1;
      }
      if (gany) {
        const int s2 = sp + (lany ? 1 : 0);
        stk[3 * s2] = pidx;
        stk[3 * s2 + 1] = R;
        stk[3 * s2 + 2] = it - 1;
      }
    }
    sp += (lany ? 1 : 0) + (gany ? 1 : 0);
    ord_fence();
  }
  for (int i = lane; i < n; i += 64) perm[i] = (int32_t)(W[i] & kOrdIdx);
  if (lane == 0) a.tiepos[shot] = fallback ? -1 : n;
}

size_t osd_order_lds(int n) { return (size_t)8 * n + 96 * 4 + 512 * 2 + 16; }

hipError_t launch_osd_order(const OrderArgs& a, long long count, hipStream_t stream) {
  const void* k = a.n <= 256 ? (const void*)&osd_order_kernel<4>
                : a.n <= 512 ? (const void*)&osd_order_kernel<8>
                : a.n <= 1024 ? (const void*)&osd_order_kernel<16>
                : (const void*)&osd_order_kernel<32>;
  long long done = 0;
  while (done < count) {
    const long long g = count - done < (1ll << 30) ? count - done : (1ll << 30);
    OrderArgs ai = a;
    ai.post = a.post + done * a.n;
    ai.perm = a.perm + done * a.n;
    ai.tiepos = a.tiepos + done;
    void* params[] = {(void*)&ai};
    hipError_t e = hipLaunchKernel(k, dim3((unsigned)g), dim3(64), params, osd_order_lds(a.n), stream);
    if (e != hipSuccess) return e;
    done += g;
  }
  return hipSuccess;
}

// CPython setobject.c emulation (set_difference -> set_add_entry with
// resize; LINEAR_PROBES 9, PERTURB_SHIFT 5) for small-int keys, one thread.
__device__ int first_setdiff(int n, const unsigned char* inJ, int nJ, int* table) {
  if ((n >> 2) > nJ) {
    for (int i = 0; i < n; ++i)
      if (!inJ[i]) return i;
    return -1;
  }
  unsigned mask = 7, fill = 0, used = 0;
  for (unsigned s = 0; s <= mask; ++s) table[s] = -1;
  for (int key = 0; key < n; ++key) {
    if (inJ[key]) continue;
    unsigned perturb = (unsigned)key, i = (unsigned)key & mask;
    while (true) {
      unsigned probes = (i + 9 <= mask) ? 9 : 0, k = i;
      bool placed = false;
      while (true) {
        if (table[k] < 0) { table[k] = key; placed = true; break; }
        if (probes-- == 0) break;
        ++k;
      }
      if (placed) break;
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & mask;
    }
    ++fill;
    ++used;
    if (fill * 5 >= mask * 3) {
      const unsigned minused = used > 50000 ? used * 2 : used * 4;
      unsigned newsize = 8;
      while (newsize <= minused) newsize <<= 1;
      // re-insert (old table order) into the new one: copy old entries to the
      // upper half of the scratch first (newsize > 2*(mask+1) always here)
      int* old = table + newsize;
      for (unsigned s = 0; s <= mask; ++s) old[s] = table[s];
      for (unsigned s = 0; s < newsize; ++s) table[s] = -1;
      const unsigned nmask = newsize - 1;
      for (unsigned s = 0; s <= mask; ++s) {
        const int kk = old[s];
        if (kk < 0) continue;
        unsigned pt = (unsigned)kk, j = (unsigned)kk & nmask;
        while (true) {
          if (table[j] < 0) { table[j] = kk; break; }
          bool ok = false;
          if (j + 9 <= nmask) {
            for (int q = 0; q < 9; ++q) {
              ++j;
              if (table[j] < 0) { table[j] = kk; ok = true; break; }
            }
          }
          if (ok) break;
          pt >>= 5;
          j = (j * 5 + 1 + pt) & nmask;
        }
      }
      mask = nmask;
    }
  }
  for (unsigned s = 0; s <= mask; ++s)
    if (table[s] >= 0) return table[s];
  return -1;
}

const void* select_osd_kernel(int nw) {
  if (nw <= 0) return nullptr;                      // (osd_nw_of: more than 33 words)
  if (nw <= 4) return (const void*)&osd_kernel<4>;
  if (nw <= 9) return (const void*)&osd_kernel<9>;
  if (nw <= 17) return (const void*)&osd_kernel<17>;
  if (nw <= 33) return (const void*)&osd_kernel<33>;
  return nullptr;
}

// ---------------------------------------------------------------------------
// OSD for codes past the register / LDS kernels (m > 1024 rows, or more than
// 33 row words: n > 2111): osd_kernel's exact-REF column protocol with the
// working matrix in a per-shot global scratch slice (OsdHbmArgs). Thread t
// owns the REF row positions t, t + B, ...; the current word of every row is
// cached in LDS (cw), so the pivot search and the "holds a 1" tests never
// touch global memory; a pivot's words w.. are staged in LDS (prow, and the
// row it displaces in xr), and every row holding a 1 in the column XORs them
// into its words w.. in global memory (word-major, so a word of consecutive
// positions is contiguous). Per column: the pivot is the first position >=
// xrow holding a 1 (REF, gf2math.py:139-187), rows below and above are
// reduced, J and e_J as in osd_kernel (decoders.py:329-368). Two workgroup
// barriers per pivot column, one per dependent column.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) osd_hbm_kernel(OsdArgs a, OsdHbmArgs h) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int m = a.m, n = a.n, NWr = h.nwr, MP = h.mp;
  uint64_t* cw = (uint64_t*)lds;                       // [MP] word w of each row position
  uint64_t* prow = cw + MP;                            // [NWr] the pivot row
  uint64_t* xr = prow + NWr;                           // [NWr] the row the pivot displaces
  uint64_t* emask = xr + NWr;                          // [NWr] e_I bits (decoders.py:345)
  int* slots = (int*)(emask + NWr);                    // [2][16] per-wave candidates
  int* misc = slots + 32;
  const int t = threadIdx.x, B = blockDim.x, lane = t & 63, wave = t >> 6, nwaves = B >> 6;
  const long long shot = blockIdx.x;
  if (osd_host_shot(a, shot, n, slots)) return;
  unsigned char* base = h.scratch + (size_t)shot * (size_t)h.stride;
  uint64_t* R = (uint64_t*)base;
  int* inv = (int*)(base + h.off_inv);
  int* Jl = (int*)(base + h.off_jl);
  unsigned char* inJ = base + h.off_inj;
  int* table = (int*)(base + h.off_table);
  const int32_t* perm = a.perm + shot * (long long)n;
  const uint8_t* syn = a.syn + shot * (long long)m;
  uint8_t* ehat = a.ehat + shot * (long long)n;
  auto word = [&](int q, int p) -> uint64_t& { return R[(size_t)q * MP + p]; };

  for (int i = t; i < n; i += B) {
    inv[perm[i]] = i;
    inJ[i] = 0;
  }
  for (size_t x = t; x < (size_t)NWr * MP; x += B) R[x] = 0;
  __syncthreads();
  // Hp's rows (+ the syndrome bit at column n); row r starts at position r
  for (int r = t; r < m; r += B) {
    for (int e = a.row_ptr[r]; e < a.row_ptr[r + 1]; ++e) {
      const int i = inv[a.col_idx[e]];
      word(i >> 6, r) |= 1ull << (i & 63);
    }
    if (syn[r] & 1) word(n >> 6, r) |= 1ull << (n & 63);
  }
  int xrow = 0, rank = 0, nJ = 1, step = 0;
  bool done = a.rank == 0;                              // rank(H) = 0: IndexError below
  if (t == 0) {
    Jl[0] = 0;                                          // column 0 always (decoders.py:329)
    inJ[0] = 1;
  }
  const int K = (m + B - 1) / B;
  for (int w = 0; w < NWr && 64 * w < n && !done; ++w) {
    __syncthreads();                                    // (the previous word's last pivot applied)
    for (int p = t; p < m; p += B) cw[p] = word(w, p);
    for (int b = 0; b < 64; ++b) {
      const int i = 64 * w + b;
      if (i >= n || done) break;
      // the first position >= xrow holding a 1 in column i: per wave, the
      // lowest hit of the lowest position round that has one
      int cand = 0x7fffffff;
      for (int k = 0; k < K; ++k) {
        const int p = t + k * B;
        const uint64_t bal = __ballot(p < m && p >= xrow && ((cw[p] >> b) & 1ull));
        if (bal) {
          cand = k * B + 64 * wave + __builtin_ctzll(bal);
          break;
        }
      }
      // two slot sets alternate (a wave writing set s at column k + 2 has
      // passed column k + 1's barrier, after every read of column k's set s)
      const int set = step & 1;
      if (lane == 0) slots[16 * set + wave] = cand;
      __syncthreads();
      int piv = 0x7fffffff;
      for (int q = 0; q < nwaves; ++q) piv = min(piv, slots[16 * set + q]);
      ++step;
      if (piv == 0x7fffffff) continue;                // dependent column: not in J
      for (int q = w + t; q < NWr; q += B) {
        prow[q] = word(q, piv);
        xr[q] = word(q, xrow);
      }
      __syncthreads();
      // the pivot row moves to position xrow (REF's swap; the row it
      // displaces has a 0 in column i), every other row holding a 1 in
      // column i takes it, below and above (rows at positions >= xrow are 0
      // left of column i, and so is the pivot row: words < w never change)
      for (int p = t; p < m; p += B) {
        const uint64_t c = cw[p];
        if (p == piv && piv != xrow) {
          for (int q = w; q < NWr; ++q) word(q, p) = xr[q];
          cw[p] = xr[w];
        } else if (p == xrow) {
          for (int q = w; q < NWr; ++q) word(q, p) = prow[q];
          cw[p] = prow[w];
        } else if ((c >> b) & 1ull) {
          for (int q = w; q < NWr; ++q) word(q, p) ^= prow[q];
          cw[p] = c ^ prow[w];
        }
      }
      if (i != 0) {
        if (t == 0) {
          Jl[nJ] = i;
          inJ[i] = 1;
        }
        ++nJ;
      }
      ++xrow;
      ++rank;
      if (rank >= a.rank || xrow >= m) done = true;
      if (i == 0 && done) rank = -1;                  // column 0 alone reaches rank(H): the
    }                                                 // greedy loop never breaks (:333-342)
  }
  if (rank < a.rank) {                                // greedy loop runs past column n-1
    if (t == 0) a.status[shot] = 1;                   // (the reference raises IndexError)
    return;
  }
  __syncthreads();
  // information-set values e_I (e_perm = e_hat[perm], decoders.py:345)
  for (int i0w = 64 * wave; i0w < 64 * NWr; i0w += B) {
    const int i = i0w + lane;
    const bool bit = i < n && !inJ[i] && (ehat[perm[i]] & 1);
    const uint64_t bits = __ballot(bit);
    if (lane == 0) emask[i0w >> 6] = bits;
  }
  if (t == 0) {
    int i0 = -1;
    if (a.order == 1 && nJ < n) i0 = first_setdiff(n, inJ, nJ, table);   // (decoders.py:344)
    misc[2] = i0;
  }
  __syncthreads();
  const int i0 = misc[2];
  if (t == 0 && i0 >= 0) emask[i0 >> 6] ^= 1ull << (i0 & 63);  // order-1 flip (:349-350)
  __syncthreads();
  // e_J = (T sJ)[:|J|], T sJ = T s + R[:, I] e_I (mod 2)   (decoders.py:352-358)
  for (int p = t; p < nJ && p < m; p += B) {
    uint64_t acc = (word(n >> 6, p) >> (n & 63)) & 1ull;   // T s (augmented column)
    for (int q = 0; q < NWr; ++q) acc ^= (uint64_t)(__builtin_popcountll(word(q, p) & emask[q]) & 1);
    ehat[perm[Jl[p]]] = (uint8_t)(acc & 1ull);            // e_hat[perm] = ... (:368)
  }
  // an all-zero column 0 with rank(H) = m: J holds m + 1 entries, one more
  // than T sJ has rows (the reference's assignment fails to broadcast); the
  // host OSD writes 0 there, and so does this kernel
  if (t == 0)
    for (int p = m; p < nJ; ++p) ehat[perm[Jl[p]]] = 0;
  if (t == 0 && i0 >= 0) ehat[perm[i0]] ^= 1;
  if (t == 0) a.status[shot] = 0;
}

const void* osd_hbm_kernel_ptr() { return (const void*)&osd_hbm_kernel; }

template <int NW>
static const void* osd_block_by_rows(int m, int* rt) {
  *rt = m <= 256 ? 1 : 2;
  if (m <= 256) return (const void*)&osd_block_kernel<NW, 4, 1>;
  if (m <= 512) return (const void*)&osd_block_kernel<NW, 8, 2>;
  return nullptr;                                   // (the engine state would spill: column kernel)
}

// block kernel configurations whose state fits the VGPR budget without
// spills (m <= 512 rows, n <= 1087 columns); null -> osd_kernel
const void* select_osd_block_kernel(int nw, int m, int* rows_per_thread) {
  if (nw <= 0) return nullptr;
  if (nw <= 4) return osd_block_by_rows<4>(m, rows_per_thread);
  if (nw <= 9) return osd_block_by_rows<9>(m, rows_per_thread);
  if (nw <= 17) return osd_block_by_rows<17>(m, rows_per_thread);
  return nullptr;
}

int osd_nw_of(int nw) { return nw <= 4 ? 4 : nw <= 9 ? 9 : nw <= 17 ? 17 : nw <= 33 ? 33 : 0; }

}  // namespace qldpc
