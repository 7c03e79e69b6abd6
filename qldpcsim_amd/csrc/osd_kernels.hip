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

namespace qldpc {

__device__ int first_setdiff(int n, const unsigned char* inJ, int nJ, int* table);

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
  if (a.tiepos) {
    // device-computed order: the result depends only on perm[0 .. need]
    // (the columns the elimination visited and, for order 1, the flipped
    // position); it equals NumPy's order there unless a key gap inside that
    // prefix is within the certification margin -> leave it to the host
    if (t == 0) {
      int need = Jl[nJ - 1];
      if (a.order == 1 && nJ < n) need = max(need, first_setdiff(n, inJ, nJ, table));
      misc[3] = a.tiepos[shot] <= need;
    }
    __syncthreads();
    if (misc[3]) {
      if (t == 0) a.status[shot] = 2;
      return;
    }
  }
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
  if (t == 0 && i0 >= 0) ehat[perm[i0]] ^= 1;
  if (t == 0) a.status[shot] = 0;
}

// ---------------------------------------------------------------------------
// Reliability order of one shot per workgroup (np2 / 2 threads): keys as
// NumPy forms them in decoders.py:320-325 (clip, exp, 1 / (1 + e),
// max(prob, 1 - prob)), with the device exp; a key lies in [0.5, 1], so
// (bits - bits(0.5)) fits 53 bits and (that << 11 | index) sorts by key, then
// index, as one 64-bit integer (bitonic network in LDS). NumPy's argsort
// breaks ties its own way and its exp may differ from the device's in the
// last bits, so the caller trusts this order only up to tiepos (the first
// adjacent pair closer than kOrderMarginUlp units in the last place).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) osd_order_kernel(OrderArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  uint64_t* key = (uint64_t*)lds;                   // [np2]
  int* tmin = (int*)(lds + 8 * a.np2);               // [1]
  const int t = threadIdx.x, nt = blockDim.x;
  const long long shot = blockIdx.x;
  const double* post = a.post + shot * (long long)a.n;
  const int n = a.n, np2 = a.np2;
  constexpr uint64_t kHalf = 0x3FE0000000000000ull;  // bits of 0.5
  bool bad = false;
  for (int i = t; i < np2; i += nt) {
    uint64_t c = ~0ull;                               // padding sorts last
    if (i < n) {
      double x = post[i];
      x = x < -100.0 ? -100.0 : (x > 100.0 ? 100.0 : x);   // np.clip(P, -100, 100)
      const double e = exp(x);
      const double prob = 1.0 / (1.0 + e);
      const double q = 1.0 - prob;
      const double rel = prob > q ? prob : q;         // np.maximum(prob, 1 - prob)
      if (!(rel >= 0.5 && rel <= 1.0)) bad = true;    // NaN posterior: host decides
      const uint64_t u = (__builtin_bit_cast(uint64_t, rel) - kHalf) & ((1ull << 53) - 1);
      c = (u << 11) | (uint64_t)i;
    }
    key[i] = c;
  }
  if (t == 0) *tmin = n;
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < np2 / 2; i += nt) {
        const int lo = 2 * i - (i & (j - 1)), hi = lo + j;
        const bool up = (lo & k) == 0;
        const uint64_t x = key[lo], y = key[hi];
        if ((x > y) == up) {
          key[lo] = y;
          key[hi] = x;
        }
      }
      __syncthreads();
    }
  }
  int first = bad ? 0 : n;
  for (int i = t; i + 1 < n; i += nt)
    if ((key[i + 1] >> 11) - (key[i] >> 11) <= (uint64_t)kOrderMarginUlp) first = min(first, i);
  for (int off = 32; off > 0; off >>= 1) first = min(first, __shfl_xor(first, off, 64));
  if ((t & 63) == 0) atomicMin(tmin, first);
  int32_t* perm = a.perm + shot * (long long)n;
  for (int i = t; i < n; i += nt) perm[i] = (int32_t)(key[i] & 2047u);
  __syncthreads();
  if (t == 0) a.tiepos[shot] = *tmin;
}

hipError_t launch_osd_order(const OrderArgs& a, long long count, hipStream_t stream) {
  long long done = 0;
  while (done < count) {
    const long long g = count - done < (1ll << 30) ? count - done : (1ll << 30);
    OrderArgs ai = a;
    ai.post = a.post + done * a.n;
    ai.perm = a.perm + done * a.n;
    ai.tiepos = a.tiepos + done;
    void* params[] = {(void*)&ai};
    const size_t lds = (size_t)8 * a.np2 + 16;
    hipError_t e = hipLaunchKernel((const void*)&osd_order_kernel, dim3((unsigned)g), dim3(a.np2 / 2), params,
                                   lds, stream);
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
  if (nw <= 4) return (const void*)&osd_kernel<4>;
  if (nw <= 9) return (const void*)&osd_kernel<9>;
  if (nw <= 17) return (const void*)&osd_kernel<17>;
  if (nw <= 33) return (const void*)&osd_kernel<33>;
  return nullptr;
}

int osd_nw_of(int nw) { return nw <= 4 ? 4 : nw <= 9 ? 9 : nw <= 17 ? 17 : nw <= 33 ? 33 : 0; }

}  // namespace qldpc
