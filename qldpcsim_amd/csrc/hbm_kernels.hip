// hbm_kernels.hip — min-sum / BP decoding with the message state in HBM, for
// codes the LDS-resident kernels cannot hold (per-half-shot state beyond a
// CU's LDS, or tables past the 16-bit formats). Same arithmetic as the
// LDS kernels and the oracle, bit for bit (decoders.py:110-182, :189-290).
//
// Layout and execution:
//  * one workgroup = one TILE of 64 half-shot slots: lane l of every wave
//    works on slot l, and the workgroup's W waves split each layer's rows
//    (check nodes) and adjacent variables (variable nodes) between them, with
//    a workgroup barrier between the two phases. A tile's state is contiguous
//    in HBM, element-major inside the tile: c2v[g][p][64] (CSC position p),
//    posterior[g][v][64], syndrome[g][c][64] — every message access is one
//    coalesced 256 / 512-byte row, and all the waves of a CU touch the same
//    ~20 MB (a handful of 2 MB pages: the CU's address-translation working set
//    stays small; one thread per half-shot with slot-major rows over the whole
//    grid made every access a translation miss);
//  * graph tables are read wave-uniformly (scalar loads);
//  * min-sum keeps the float32 column sum S per variable (posterior = L +
//    (f64)S, decoders.py:172-173, rebuilt on read): 4-byte rows, SURVEY.md
//    §8(d)'s w = 4; BP keeps the float64 posterior;
//  * slots recycle: a slot whose decode stops (or reaches max_iter) writes its
//    outputs and takes the next half-shot from a global ticket counter at the
//    next iteration boundary, so early-stopping decodes keep the tile busy;
//  * no state initialisation pass when the layers partition the rows (always
//    for the reference's schedules): in a slot's first iteration, a message
//    of a check its layer has not reached yet reads as 0 and a posterior no
//    variable node has written yet as L (per-edge / per-variable "first layer"
//    tables) — the same values the reference's freshly zeroed arrays hold;
//  * stop test after every layer (decoders.py:175-176, :283-285): 32 parity
//    filters (F == B, kept current from the hard-decision flips the variable
//    nodes see, combined over the waves through LDS) gate the exact check over
//    all rows, as in ms_layered_kernel.
// HBM traffic per executed half-shot iteration is SURVEY.md §8(d)'s model
// (flooding MS: 4(3E + 2n) bytes + the old-posterior read for the flip test).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "decoder_kernels.h"
#include "hbm_kernels.h"
#include "../../include/qldpc_libm.h"

namespace qldpc {

__constant__ qldpc_libm_tab qldpc_libm_hbm_dev = QLDPC_LIBM_TAB_INIT;

// NumPy's DOUBLE_pairwise_sum (np.sum of a 1-D float64 array) over a strided
// column of the c2v rows: 0.0 + pairwise(all), 8 accumulators for d >= 8
// (decoders.py:269, :276); entries with zero[t] read as +0.0.
template <typename Get>
__device__ __forceinline__ double np_pairwise_strided(int d, Get get) {
  if (d < 8) {
    double res = -0.0;
    for (int i = 0; i < d; ++i) res += get(i);
    return 0.0 + res;
  }
  double r0 = get(0), r1 = get(1), r2 = get(2), r3 = get(3), r4 = get(4), r5 = get(5), r6 = get(6), r7 = get(7);
  int i = 8;
  const int nb = d - (d % 8);
  for (; i < nb; i += 8) {
    r0 += get(i + 0); r1 += get(i + 1); r2 += get(i + 2); r3 += get(i + 3);
    r4 += get(i + 4); r5 += get(i + 5); r6 += get(i + 6); r7 += get(i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < d; ++i) res += get(i);
  return 0.0 + res;
}

// Graph tables are read-only for the whole launch: reading them through the
// constant address space lets the compiler use scalar loads (wave-uniform
// indices) — through a generic pointer it must assume the kernel's own stores
// may alias them and issues a vector load + readfirstlane per table word.
template <typename T>
__device__ __forceinline__ T tb(const T* p, int i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// combine one word per wave and lane through LDS: every wave writes its
// partial, a barrier, every wave reads all W partials. `buf` [W][64] may be
// rewritten only after the next workgroup barrier (all readers passed it).
template <int W, typename Op>
__device__ __forceinline__ uint32_t wg_combine(uint32_t* buf, uint32_t x, int wave, int lane, Op op) {
  buf[wave * 64 + lane] = x;
  __syncthreads();
  uint32_t r = buf[lane];
#pragma unroll
  for (int w = 1; w < W; ++w) r = op(r, buf[w * 64 + lane]);
  return r;
}

template <int ALGO, int DCMAX, int W>
__global__ void __launch_bounds__(64 * W) hbm_tile_kernel(HbmArgs a, const int32_t* __restrict__ fl_var,
                                                        const int32_t* __restrict__ fl_pos, int lazy) {
  using Msg = typename std::conditional<ALGO == ALGO_MS, float, double>::type;
  using Post = Msg;                                 // MS: float32 column sum S; BP: float64 posterior
  constexpr int UC = QLDPC_HBM_UC;                   // checks per load step (1: 16 waves per CU; 2: 12, 4: 8 — slower, r03o)
  constexpr int UV = 4, KV = 8;                   // variables per load batch, messages loaded up front
  __shared__ uint32_t xb[3][W * 64];              // per-wave partials: [0] filters / flags, [1] stop test, [2] B
  __shared__ long long shot_s[64];
  const qldpc_libm_tab* lt = nullptr;
  if constexpr (ALGO == ALGO_BP) {
    __shared__ qldpc_libm_tab lt_s;
    const uint4* src = (const uint4*)&qldpc_libm_hbm_dev;
    uint4* dst = (uint4*)&lt_s;
    for (int i = threadIdx.x; i < (int)(sizeof(qldpc_libm_tab) / 16); i += blockDim.x) dst[i] = src[i];
    lt = &lt_s;
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = a.m, n = a.n, E = a.E;
  const double L = a.L;
  // this tile's rows: element i of slot `lane` at base[i * 64 + lane] (uniform
  // 64-bit base, 32-bit per-lane offset: one saddr load / store per access)
  const long long g = blockIdx.x;
  Msg* const c2v_t = (Msg*)a.c2v + g * (long long)E * 64;
  Post* const post_t = (Post*)a.post + g * (long long)n * 64;
  uint8_t* const syn_t = a.synT + g * (long long)m * 64;
  auto C2V = [&](int p) -> Msg& { return c2v_t[(uint32_t)p * 64u + (uint32_t)lane]; };
  auto POST = [&](int v) -> Post& { return post_t[(uint32_t)v * 64u + (uint32_t)lane]; };
  auto SYN = [&](int c) -> uint8_t& { return syn_t[(uint32_t)c * 64u + (uint32_t)lane]; };
  auto rd_post = [&](int v) -> double {
    if constexpr (ALGO == ALGO_MS) return L + (double)POST(v);
    else return POST(v);
  };

  // Check node of a row of more than DCMAX edges (rows of any degree decode,
  // as the reference's load_matrix takes any H): the same arithmetic in two
  // passes over the edges in CSR (ascending variable) order — pass 1 forms
  // min1 / min2 and the sign parity (MS) or np.prod's sequential fold (BP),
  // pass 2 re-forms each edge's v2c (its own c2v is still the old one: each
  // edge is read before it is written) and writes the new message.
  int fl = 0;
  auto cn_wide = [&](int e0, int d, uint32_t sbit, bool first, int l, bool lzf) {
    auto v2c = [&](int k) -> double {                 // post - c2v of edge k (:155-156, :247-248)
      const int e = e0 + k, var = tb(a.row_var, e), pos = tb(a.row_pos, e);
      if (ALGO == ALGO_MS && first && l == 0) return (double)a.L32;   // msg_v2c = float32(L) (:148-149)
      const bool okv = !lzf || !first || tb(fl_var, var) < l;
      const bool okc = !lzf || !first || tb(fl_pos, pos) < l;
      return (okv ? rd_post(var) : L) - (double)(okc ? C2V(pos) : (Msg)0);
    };
    if constexpr (ALGO == ALGO_MS) {
      uint32_t par = sbit;
      double min1 = __builtin_inf(), min2 = __builtin_inf();
      for (int k = 0; k < d; ++k) {
        const double v = v2c(k);
        par ^= (uint32_t)(v < 0.0);                   // np.sign, 0 -> +1 (:157-158)
        const double x = __builtin_fabs(v);
        min2 = __builtin_fmin(min2, __builtin_fmax(min1, x));   // min of the rest (:162-164)
        min1 = __builtin_fmin(min1, x);
      }
      const double m1 = __builtin_isinf(min1) ? 0.0 : min1, m2 = __builtin_isinf(min2) ? 0.0 : min2;
      if (m1 == 0.0) fl |= FLAG_MIN_ZERO;
      const float c1 = (float)(a.beta * m1), c2 = (float)(a.beta * m2);   // (:167-168)
      for (int k = 0; k < d; ++k) {
        const double v = v2c(k);
        const float mag = (__builtin_fabs(v) == min1) ? c2 : c1;
        C2V(tb(a.row_pos, e0 + k)) = ((uint32_t)(v < 0.0) ^ par) ? -mag : mag;
      }
    } else {
      double prod = 1.0;
      for (int k = 0; k < d; ++k) prod *= qldpc_tanh_t(v2c(k) / 2.0, lt->tanh_c);   // np.prod (:254)
      for (int k = 0; k < d; ++k) {
        const double th = qldpc_tanh_t(v2c(k) / 2.0, lt->tanh_c);
        if (th == 0.0) fl |= FLAG_NONFINITE;
        double th2 = prod / th;                                        // (:256)
        th2 = (__builtin_fabs(th2) >= 1.0 - a.eps) ? th2 - __builtin_copysign(a.eps, th2) : th2;
        double val = 2.0 * qldpc_atanh_t(th2, lt->atanh_hl, lt->atanh_rcp);   // (:259)
        if (sbit) val = -val;                                          // (:260-261)
        if (!__builtin_isfinite(val)) fl |= FLAG_NONFINITE;
        C2V(tb(a.row_pos, e0 + k)) = val;
      }
    }
  };

  long long shot = -1;
  bool need = true;          // take a half-shot at the next iteration boundary (same on every wave)
  int it = 0, lstop = 0;
  uint32_t F = 0, B = 0;

  for (;;) {
    // --- slots without work take half-shots (one ticket per tile, wave 0) ---
    const uint64_t nm = __ballot(need);
    if (nm) {
      if (wave == 0) {
        const int leader = __builtin_ctzll(nm);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(a.queue, (uint32_t)__builtin_popcountll(nm));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
        if (need) {
          const long long t = (long long)base +
                              __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0));
          shot_s[lane] = t < a.batch ? t : -1;
        }
      }
      __syncthreads();
      const bool init = need;
      if (need) {
        shot = shot_s[lane];
        need = false;
        it = 0;
        fl = 0;
        F = (L < 0.0) ? a.filt_all : 0u;            // every posterior starts at L
      }
      // stage the new half-shots' syndromes (rows split over the waves) and
      // form their filter word B
      uint32_t bp = 0;
      const bool st = init && shot >= 0;
      if (__ballot(st)) {
        for (int c = wave; c < m; c += W) {
          if (st) {
            uint32_t b;
            if (a.syn_bits) b = (uint32_t)(((const uint64_t*)a.syn)[shot * a.wm + (c >> 6)] >> (c & 63)) & 1u;
            else b = a.syn[shot * (long long)m + c] & 1u;
            SYN(c) = (uint8_t)b;
            bp ^= b ? tb(a.wc, c) : 0u;
          }
        }
        if (!lazy) {                                // rows not a partition: zero the state
          for (int v = wave; v < n; v += W)
            if (st) POST(v) = ALGO == ALGO_MS ? (Post)0 : (Post)L;
          for (int p = wave; p < E; p += W)
            if (st) C2V(p) = (Msg)0;
        }
      }
      const uint32_t bt = wg_combine<W>(xb[2], bp, wave, lane, [](uint32_t x, uint32_t y) { return x ^ y; });
      if (init) B = bt;
      __syncthreads();                              // staged rows visible to every wave
    }
    if (__ballot(shot >= 0) == 0) break;             // queue drained, every slot idle (uniform)

    // --- one iteration over the layers ---
    bool stop = false;                               // this slot's decode ended inside the iteration
    for (int l = 0; l < a.n_layers; ++l) {
      const bool act = shot >= 0 && !stop;
      const bool first = it == 0;
      const bool it0 = __ballot(!first) == 0;        // uniform: no slot past its first iteration
      // check nodes of the layer (Jacobi: all read the same posteriors), UC
      // checks per step with every message load issued before any arithmetic
      const int q0 = tb(a.lay_ptr, l), q1 = tb(a.lay_ptr, l + 1);
      const bool lzf = lazy && __ballot(first && shot >= 0) != 0;   // (uniform) lazy init, a slot in its first iteration
      if (__ballot(act)) {
        for (int qb = q0 + wave * UC; qb < q1; qb += W * UC) {
          int e0[UC], dg[UC];
          uint32_t sb[UC];
          double pj[UC][DCMAX];
          Msg cj[UC][DCMAX];
          const bool l0 = ALGO == ALGO_MS && it0 && l == 0;   // every slot at v2c = float32(L): nothing to read
          // every load of the step is issued before the first wait: indices
          // past the row's degree read edge 0 (discarded), and the per-slot
          // choices (inactive slot, first-iteration "not reached yet") are
          // selects after the loads, not branches around them
          Post rp[UC][DCMAX];
          Msg rc[UC][DCMAX];
#pragma unroll
          for (int u = 0; u < UC; ++u) {
            const int c = qb + u < q1 ? tb(a.lay_rows, qb + u) : 0;
            e0[u] = tb(a.row_ptr, c);
            dg[u] = qb + u < q1 ? tb(a.row_ptr, c + 1) - e0[u] : 0;
            sb[u] = SYN(c);
#pragma unroll
            for (int k0 = 0; k0 < DCMAX; k0 += 8) {
              if (!l0 && (k0 == 0 || k0 < dg[u])) {    // (uniform)
#pragma unroll
                for (int k = k0; k < k0 + 8 && k < DCMAX; ++k) {
                  const int e = k < dg[u] ? e0[u] + k : 0;
                  rp[u][k] = POST(tb(a.row_var, e));
                  rc[u][k] = C2V(tb(a.row_pos, e));
                }
              }
            }
          }
#pragma unroll
          for (int u = 0; u < UC; ++u) {
            sb[u] = dg[u] ? sb[u] : 0u;
#pragma unroll
            for (int k = 0; k < DCMAX; ++k) {
              pj[u][k] = L;
              cj[u][k] = (Msg)0;
              if (k < dg[u] && !l0) {
                bool okv = true, okc = true;
                if (lzf) {                               // (uniform) first-layer tables
                  okv = !first || tb(fl_var, tb(a.row_var, e0[u] + k)) < l;
                  okc = !first || tb(fl_pos, tb(a.row_pos, e0[u] + k)) < l;
                }
                const double pv = ALGO == ALGO_MS ? L + (double)rp[u][k] : (double)rp[u][k];
                pj[u][k] = okv ? pv : L;
                cj[u][k] = okc ? rc[u][k] : (Msg)0;
              }
            }
          }
#pragma unroll
          for (int u = 0; u < UC; ++u) {
            const int d = dg[u];
            if (!act || d == 0) continue;
            if (d > DCMAX) {                            // (uniform) a row wider than the kernel's
              cn_wide(e0[u], d, sb[u], first, l, lzf);  // registers: two passes over its edges
              continue;
            }
            if constexpr (ALGO == ALGO_MS) {
              double av[DCMAX];
              uint64_t negm = 0;
              double min1 = __builtin_inf(), min2 = __builtin_inf();
#pragma unroll
              for (int k = 0; k < DCMAX; ++k) {
                if (k < d) {
                  // v2c = post - c2v (:177); the first layer of the first
                  // iteration reads msg_v2c[H == 1] = L_ch as float32 (:148-149)
                  const double v = (first && l == 0) ? (double)a.L32 : pj[u][k] - (double)cj[u][k];
                  negm |= (uint64_t)(v < 0.0) << k;      // np.sign, 0 -> +1 (:157-158)
                  const double x = __builtin_fabs(v);
                  av[k] = x;
                  min2 = __builtin_fmin(min2, __builtin_fmax(min1, x));   // min of the rest (:162-164)
                  min1 = __builtin_fmin(min1, x);
                }
              }
              const double m1 = __builtin_isinf(min1) ? 0.0 : min1;        // (:165)
              const double m2 = __builtin_isinf(min2) ? 0.0 : min2;        // (:166)
              if (m1 == 0.0) fl |= FLAG_MIN_ZERO;                          // App. A.1.6 (flagged, not emulated)
              const uint32_t negprod = (uint32_t)(__builtin_popcountll(negm) & 1) ^ sb[u];
              const float c1 = (float)(a.beta * m1), c2 = (float)(a.beta * m2);   // fl32(beta * min) (:167-168)
#pragma unroll
              for (int k = 0; k < DCMAX; ++k) {
                if (k < d) {
                  const float mag = (av[k] == min1) ? c2 : c1;
                  C2V(tb(a.row_pos, e0[u] + k)) = (((negm >> k) & 1u) ^ negprod) ? -mag : mag;
                }
              }
            } else {
              double th[DCMAX];
              double prod = 1.0;
#pragma unroll
              for (int k = 0; k < DCMAX; ++k) {
                if (k < d) {
                  th[k] = qldpc_tanh_t((pj[u][k] - cj[u][k]) / 2.0, lt->tanh_c);   // v2c (:269), np.tanh (:254)
                  prod *= th[k];                                                  // np.prod: sequential fold
                }
              }
#pragma unroll
              for (int k = 0; k < DCMAX; ++k) {
                if (k < d) {
                  if (th[k] == 0.0) fl |= FLAG_NONFINITE;
                  double th2 = prod / th[k];                            // (:256)
                  th2 = (__builtin_fabs(th2) >= 1.0 - a.eps) ? th2 - __builtin_copysign(a.eps, th2) : th2;  // (:257-258)
                  double val = 2.0 * qldpc_atanh_t(th2, lt->atanh_hl, lt->atanh_rcp);   // (:259)
                  if (sb[u]) val = -val;                                // (:260-261)
                  if (!__builtin_isfinite(val)) fl |= FLAG_NONFINITE;
                  C2V(tb(a.row_pos, e0[u] + k)) = val;
                }
              }
            }
          }
        }
      }
      __syncthreads();                               // every c2v row of the layer written
      // variable nodes adjacent to the layer (others are unchanged, :172-177 /
      // :265-278), UV variables per step, their first KV messages loaded up front
      uint32_t Fp = 0;                               // this wave's flips
      const int v0 = tb(a.adj_ptr, l), v1 = tb(a.adj_ptr, l + 1);
      if (__ballot(act)) {
        for (int qb = v0 + wave * UV; qb < v1; qb += W * UV) {
          int vv[UV], p0[UV], dg[UV];
          double old[UV];
          Msg cv[UV][KV];
          Post ro[UV];
          Msg rv[UV][KV];
#pragma unroll
          for (int u = 0; u < UV; ++u) {                // loads (past the degree: edge 0, discarded)
            vv[u] = qb + u < v1 ? tb(a.adj_vars, qb + u) : 0;
            p0[u] = tb(a.col_ptr, vv[u]);
            dg[u] = qb + u < v1 ? tb(a.col_ptr, vv[u] + 1) - p0[u] : 0;
            ro[u] = POST(vv[u]);
#pragma unroll
            for (int t = 0; t < KV; ++t) rv[u][t] = C2V(t < dg[u] ? p0[u] + t : 0);
          }
#pragma unroll
          for (int u = 0; u < UV; ++u) {                // per-slot selects
            const bool okv = !lzf || !first || tb(fl_var, vv[u]) < l;
            old[u] = dg[u] && okv ? (ALGO == ALGO_MS ? L + (double)ro[u] : (double)ro[u]) : L;
#pragma unroll
            for (int t = 0; t < KV; ++t) {
              const bool ok = !lzf || !first || (t < dg[u] && tb(fl_pos, p0[u] + t) <= l);
              cv[u][t] = t < dg[u] && ok ? rv[u][t] : (Msg)0;
            }
          }
#pragma unroll
          for (int u = 0; u < UV; ++u) {
            const int d = dg[u];
            if (!act || qb + u >= v1) continue;
            auto get = [&](int t) -> Msg {              // message t of the column (zeros past the layer)
              if (t < KV) return cv[u][t];
              const bool ok = !lzf || !first || tb(fl_pos, p0[u] + t) <= l;
              return ok ? C2V(p0[u] + t) : (Msg)0;
            };
            double nw;
            if constexpr (ALGO == ALGO_MS) {
              float S = 0.0f;                              // float32, ascending check (:172)
#pragma unroll
              for (int t = 0; t < KV; ++t)
                if (t < d) S += cv[u][t];
              for (int t = KV; t < d; ++t) S += get(t);
              POST(vv[u]) = S;
              nw = L + (double)S;                          // (:173)
            } else {
              if (d <= KV) {
                double r = -0.0;                           // np.sum: sequential below 8 terms
                if (d < 8) {
#pragma unroll
                  for (int t = 0; t < KV; ++t)
                    if (t < d) r += cv[u][t];
                } else {                                   // exactly 8: one pairwise block
                  r = ((cv[u][0] + cv[u][1]) + (cv[u][2] + cv[u][3])) + ((cv[u][4] + cv[u][5]) + (cv[u][6] + cv[u][7]));
                }
                nw = d == 0 ? L : L + (0.0 + r);           // (:269, :276; no edges: L0, :277-278)
              } else {
                nw = L + np_pairwise_strided(d, get);
              }
              POST(vv[u]) = nw;
            }
            if ((old[u] < 0.0) != (nw < 0.0)) Fp ^= tb(a.avar, vv[u]);   // hard decision flipped
          }
        }
      }
      // filters of every wave's flips; the barrier inside also publishes the
      // layer's posteriors to the stop test / the next layer
      F ^= wg_combine<W>(xb[0], Fp, wave, lane, [](uint32_t x, uint32_t y) { return x ^ y; });
      // stop test after the layer: filters, then the exact check (:174-176)
      const bool cand = act && F == B;
      if (__ballot(cand)) {                          // same on every wave (F, B, act are)
        uint32_t un = 0;
        if (cand) {
          for (int c = wave; c < m && !un; c += W) {
            uint32_t par = SYN(c);
            for (int e = tb(a.row_ptr, c); e < tb(a.row_ptr, c + 1); ++e) {
              const int j = tb(a.row_var, e);
              const bool pv = !first || !lazy || tb(fl_var, j) <= l;
              par ^= (uint32_t)((pv ? rd_post(j) : L) < 0.0);
            }
            un |= par;
          }
        }
        un = wg_combine<W>(xb[1], un, wave, lane, [](uint32_t x, uint32_t y) { return x | y; });
        if (cand && !un) {
          stop = true;
          lstop = l;
        }
      }
    }
    // --- end of an iteration: finished decodes write their outputs ---
    bool fin = false;
    if (shot >= 0) {
      if (stop) {
        fin = true;
      } else if (it + 1 == a.max_iter) {
        fin = true;
        lstop = a.n_layers - 1;                      // every layer ran
      } else {
        ++it;
      }
    }
    if (__ballot(fin)) {
      __syncthreads();                               // xb[0] readers of the last layer are done
      const int fla = (int)wg_combine<W>(xb[0], (uint32_t)(fl & (FLAG_MIN_ZERO | FLAG_NONFINITE)), wave, lane,
                                         [](uint32_t x, uint32_t y) { return x | y; });
      if (fin && wave == 0) {
        if (stop) {
          if (a.flags) a.flags[shot] = FLAG_CONVERGED | fla;
          a.iters[shot] = it + 1;
        } else {
          if (a.flags) a.flags[shot] = fla;
          a.iters[shot] = a.max_iter;
        }
      }
      const bool lz = lazy != 0;
      for (int j0 = 64 * wave; j0 < n; j0 += 64 * W) {
        uint64_t w = 0;
        for (int jj = 0; jj < 64 && j0 + jj < n; ++jj) {
          if (fin) {
            const int j = j0 + jj, v = tb(a.vinv, j);
            // a variable no layer has reached yet keeps L (never written in
            // this decode: no layer adjacent to it, or a first-iteration stop)
            const bool unwritten = lz && (tb(fl_var, v) >= a.n_layers || (it == 0 && tb(fl_var, v) > lstop));
            const double pv = unwritten ? L : rd_post(v);
            const bool bit = pv < 0.0;                   // (:174 / :280)
            if (a.eh_bits) w |= (uint64_t)bit << jj;
            else a.ehat[shot * (long long)n + j] = (uint8_t)bit;
            if (a.out_post) a.out_post[shot * (long long)n + j] = pv;
          }
        }
        if (fin && a.eh_bits) ((uint64_t*)a.ehat)[shot * a.wn + (j0 >> 6)] = w;
      }
      if (fin) need = true;
      __syncthreads();                               // xb[0] free again; outputs read before slots are reused
    }
  }
}

// kernel names as rocprofv3 reports them (ALGO_MS = 0, ALGO_BP = 1)
#define QLDPC_HBM(ALG, A, D)                                                                   \
  if (algo == ALG && dcmax <= D) {                                                             \
    if (name) *name = "hbm_tile_kernel<" #A ", " #D ", 4>";                                    \
    return (const void*)&hbm_tile_kernel<ALG, D, kHbmWaves>;                                   \
  }
// (rows past 64 edges take the 64-wide instance's two-pass cn_wide)
const void* select_hbm_kernel(int algo, int dcmax, const char** name) {
  QLDPC_HBM(ALGO_MS, 0, 8) QLDPC_HBM(ALGO_MS, 0, 16) QLDPC_HBM(ALGO_MS, 0, 32)
  QLDPC_HBM(ALGO_BP, 1, 8) QLDPC_HBM(ALGO_BP, 1, 16) QLDPC_HBM(ALGO_BP, 1, 32)
  if (name) *name = algo == ALGO_MS ? "hbm_tile_kernel<0, 64, 4>" : "hbm_tile_kernel<1, 64, 4>";
  return algo == ALGO_MS ? (const void*)&hbm_tile_kernel<ALGO_MS, 64, kHbmWaves>
                         : (const void*)&hbm_tile_kernel<ALGO_BP, 64, kHbmWaves>;
}
#undef QLDPC_HBM

hipError_t launch_hbm(const void* kernel, const HbmArgs& a, int tiles, const int32_t* fl_var, const int32_t* fl_pos,
                      int lazy, hipStream_t stream) {
  void* params[] = {(void*)&a, (void*)&fl_var, (void*)&fl_pos, (void*)&lazy};
  return hipLaunchKernel(kernel, dim3(tiles), dim3(64 * kHbmWaves), params, 0, stream);
}

}  // namespace qldpc
