// hbm_kernels.hip — min-sum / BP decoding with the message state in HBM, for
// codes the LDS-resident kernels cannot hold (per-half-shot state beyond a
// CU's LDS, or tables past the 16-bit formats). Same arithmetic as the
// LDS kernels and the oracle, bit for bit (decoders.py:110-182, :189-290).
//
// Layout and execution:
//  * one thread = one half-shot slot; the T slots of the grid hold their
//    state slot-major in HBM: c2v[p * T + s] (CSC position p), post[v * T + s],
//    synT[c * T + s]. A wave's 64 lanes walk the same check / variable at the
//    same time, so the graph tables are read wave-uniformly (scalar loads) and
//    every message access is a coalesced 256/512-byte row;
//  * lanes recycle: a lane whose decode stops (or reaches max_iter) writes its
//    outputs and takes the next half-shot from a global ticket counter at the
//    next iteration boundary, so early-stopping decodes keep the wave busy;
//  * no state initialisation pass when the layers partition the rows (always
//    for the reference's schedules): in a lane's first iteration, a message
//    of a check its layer has not reached yet reads as 0 and a posterior no
//    variable node has written yet as L (per-edge / per-variable "first layer"
//    tables) — the same values the reference's freshly zeroed arrays hold;
//  * stop test after every layer (decoders.py:175-176, :283-285): 32 parity
//    filters (F == B, kept current from the hard-decision flips the variable
//    node sees) gate the exact check over all rows, as in ms_layered_kernel.
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
// column of the slot-major c2v: 0.0 + pairwise(all), 8 accumulators for d >= 8
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

template <int ALGO, int DCMAX>
__global__ void __launch_bounds__(256) hbm_decode_kernel(HbmArgs a, const int32_t* __restrict__ fl_var,
                                                       const int32_t* __restrict__ fl_pos, int lazy) {
  using Msg = typename std::conditional<ALGO == ALGO_MS, float, double>::type;
  constexpr int UC = DCMAX <= 8 ? (ALGO == ALGO_MS ? 4 : 2) : (DCMAX <= 16 ? 2 : 1);   // checks per load batch
  constexpr int UV = 4, KV = 8;                   // variables per load batch, messages loaded up front
  const qldpc_libm_tab* lt = nullptr;
  if constexpr (ALGO == ALGO_BP) {
    __shared__ qldpc_libm_tab lt_s;
    const uint4* src = (const uint4*)&qldpc_libm_hbm_dev;
    uint4* dst = (uint4*)&lt_s;
    for (int i = threadIdx.x; i < (int)(sizeof(qldpc_libm_tab) / 16); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    lt = &lt_s;
  }
  const long long T = a.T;
  const long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // this lane's slot
  const int lane = threadIdx.x & 63;
  Msg* c2v = (Msg*)a.c2v;
  double* post = a.post;
  const int m = a.m, n = a.n;
  const double L = a.L;

  long long shot = -1;
  bool need = true;          // take a half-shot at the next iteration boundary
  int it = 0, fl = 0, lstop = 0;
  uint32_t F = 0, B = 0;

  for (;;) {
    // --- lanes without work take half-shots (wave-aggregated tickets) ---
    const uint64_t nm = __ballot(need);
    if (nm) {
      const int leader = __builtin_ctzll(nm);
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(a.queue, (uint32_t)__builtin_popcountll(nm));
      base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
      if (need) {
        const long long t = (long long)base +
                            __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0));
        shot = t < a.batch ? t : -1;
        need = false;
        it = 0;
        fl = 0;
        F = (L < 0.0) ? a.filt_all : 0u;             // every posterior starts at L
        B = 0;
      }
      // stage the new half-shots' syndromes slot-major (+ their filter word)
      const bool init = shot >= 0 && it == 0 && ((nm >> lane) & 1);
      if (__ballot(init)) {
        for (int c = 0; c < m; ++c) {
          if (init) {
            uint32_t b;
            if (a.syn_bits) b = (uint32_t)(((const uint64_t*)a.syn)[shot * a.wm + (c >> 6)] >> (c & 63)) & 1u;
            else b = a.syn[shot * (long long)m + c] & 1u;
            a.synT[(long long)c * T + s] = (uint8_t)b;
            B ^= b ? a.wc[c] : 0u;
          }
        }
        if (!lazy) {                                 // rows not a partition: zero the state
          for (int v = 0; v < n; ++v)
            if (init) post[(long long)v * T + s] = L;
          for (int p = 0; p < a.E; ++p)
            if (init) c2v[(long long)p * T + s] = (Msg)0;
        }
      }
    }
    if (__ballot(shot >= 0) == 0) break;             // queue drained, every lane idle

    // --- one iteration over the layers ---
    bool stop = false;                               // this lane's decode ended inside the iteration
    for (int l = 0; l < a.n_layers; ++l) {
      const bool act = shot >= 0 && !stop;
      const bool first = it == 0;
      // check nodes of the layer (Jacobi: all read the same posteriors), UC
      // checks per step with every message load issued before any arithmetic
      // (a lane walks its half-shot alone: memory-level parallelism comes
      // from the loads in flight per step)
      const int q1 = a.lay_ptr[l + 1];
      for (int qb = a.lay_ptr[l]; qb < q1; qb += UC) {
        int e0[UC], dg[UC];
        uint32_t sb[UC];
        double pj[UC][DCMAX];
        Msg cj[UC][DCMAX];
#pragma unroll
        for (int u = 0; u < UC; ++u) {
          const int c = qb + u < q1 ? a.lay_rows[qb + u] : 0;
          e0[u] = a.row_ptr[c];
          dg[u] = qb + u < q1 ? a.row_ptr[c + 1] - e0[u] : 0;
          sb[u] = act && dg[u] ? a.synT[(long long)c * T + s] : 0u;
          const bool l0 = ALGO == ALGO_MS && first && l == 0;   // v2c = float32(L): nothing to read
#pragma unroll
          for (int k = 0; k < DCMAX; ++k) {
            pj[u][k] = L;
            cj[u][k] = (Msg)0;
            if (k < dg[u] && act && !l0) {
              const int jv = a.row_var[e0[u] + k], p = a.row_pos[e0[u] + k];
              if (!first || !lazy || fl_var[jv] < l) pj[u][k] = post[(long long)jv * T + s];
              if (!first || !lazy || fl_pos[p] < l) cj[u][k] = c2v[(long long)p * T + s];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < UC; ++u) {
          const int d = dg[u];
          if (!act || d == 0) continue;
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
                c2v[(long long)a.row_pos[e0[u] + k] * T + s] = (((negm >> k) & 1u) ^ negprod) ? -mag : mag;
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
                c2v[(long long)a.row_pos[e0[u] + k] * T + s] = val;
              }
            }
          }
        }
      }
      // variable nodes adjacent to the layer (others are unchanged, :172-177 /
      // :265-278), UV variables per step, their first KV messages loaded up front
      const int v1 = a.adj_ptr[l + 1];
      for (int qb = a.adj_ptr[l]; qb < v1; qb += UV) {
        int vv[UV], p0[UV], dg[UV];
        double old[UV];
        Msg cv[UV][KV];
#pragma unroll
        for (int u = 0; u < UV; ++u) {
          vv[u] = qb + u < v1 ? a.adj_vars[qb + u] : 0;
          p0[u] = a.col_ptr[vv[u]];
          dg[u] = qb + u < v1 ? a.col_ptr[vv[u] + 1] - p0[u] : 0;
          old[u] = L;
          if (act && dg[u] && (!first || !lazy || fl_var[vv[u]] < l)) old[u] = post[(long long)vv[u] * T + s];
#pragma unroll
          for (int t = 0; t < KV; ++t) {
            cv[u][t] = (Msg)0;
            if (t < dg[u] && act && (!first || !lazy || fl_pos[p0[u] + t] <= l))
              cv[u][t] = c2v[(long long)(p0[u] + t) * T + s];
          }
        }
#pragma unroll
        for (int u = 0; u < UV; ++u) {
          const int d = dg[u];
          if (!act || qb + u >= v1) continue;
          auto get = [&](int t) -> Msg {              // message t of the column (zeros past the layer)
            if (t < KV) return cv[u][t];
            const bool ok = !first || !lazy || fl_pos[p0[u] + t] <= l;
            return ok ? c2v[(long long)(p0[u] + t) * T + s] : (Msg)0;
          };
          double nw;
          if constexpr (ALGO == ALGO_MS) {
            float S = 0.0f;                              // float32, ascending check (:172)
#pragma unroll
            for (int t = 0; t < KV; ++t)
              if (t < d) S += cv[u][t];
            for (int t = KV; t < d; ++t) S += get(t);
            nw = L + (double)S;                          // (:173)
          } else if (d <= KV) {
            double r = -0.0;                             // np.sum: sequential below 8 terms
            if (d < 8) {
#pragma unroll
              for (int t = 0; t < KV; ++t)
                if (t < d) r += cv[u][t];
            } else {                                     // exactly 8: one pairwise block
              r = ((cv[u][0] + cv[u][1]) + (cv[u][2] + cv[u][3])) + ((cv[u][4] + cv[u][5]) + (cv[u][6] + cv[u][7]));
            }
            nw = d == 0 ? L : L + (0.0 + r);             // (:269, :276; no edges: L0, :277-278)
          } else {
            nw = L + np_pairwise_strided(d, get);
          }
          post[(long long)vv[u] * T + s] = nw;
          if ((old[u] < 0.0) != (nw < 0.0)) F ^= a.avar[vv[u]];   // hard decision flipped
        }
      }
      // stop test after the layer: filters, then the exact check (:174-176)
      if (act && F == B) {
        uint32_t un = 0;
        for (int c = 0; c < m && !un; ++c) {
          uint32_t par = a.synT[(long long)c * T + s];
          for (int e = a.row_ptr[c]; e < a.row_ptr[c + 1]; ++e) {
            const int j = a.row_var[e];
            const bool pv = !first || !lazy || fl_var[j] <= l;
            par ^= (uint32_t)((pv ? post[(long long)j * T + s] : L) < 0.0);
          }
          un |= par;
        }
        if (!un) {
          stop = true;
          lstop = l;
          if (a.flags) a.flags[shot] = FLAG_CONVERGED | (fl & (FLAG_MIN_ZERO | FLAG_NONFINITE));
          a.iters[shot] = it + 1;
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
        if (a.flags) a.flags[shot] = fl & (FLAG_MIN_ZERO | FLAG_NONFINITE);
        a.iters[shot] = a.max_iter;
      } else {
        ++it;
      }
    }
    if (__ballot(fin)) {
      const bool lz = lazy != 0;
      for (int j0 = 0; j0 < n; j0 += 64) {
        uint64_t w = 0;
        for (int jj = 0; jj < 64 && j0 + jj < n; ++jj) {
          if (fin) {
            const int j = j0 + jj, v = a.vinv[j];
            // a variable no layer has reached yet keeps L (never written in
            // this decode: no layer adjacent to it, or a first-iteration stop)
            const bool unwritten = lz && (fl_var[v] >= a.n_layers || (it == 0 && fl_var[v] > lstop));
            const double pv = unwritten ? L : post[(long long)v * T + s];
            const bool bit = pv < 0.0;                   // (:174 / :280)
            if (a.eh_bits) w |= (uint64_t)bit << jj;
            else a.ehat[shot * (long long)n + j] = (uint8_t)bit;
            if (a.out_post) a.out_post[shot * (long long)n + j] = pv;
          }
        }
        if (fin && a.eh_bits) ((uint64_t*)a.ehat)[shot * a.wn + (j0 >> 6)] = w;
      }
      if (fin) need = true;
    }
  }
}

// kernel names as rocprofv3 reports them (ALGO_MS = 0, ALGO_BP = 1)
#define QLDPC_HBM(ALG, A, D)                                                                   \
  if (algo == ALG && dcmax <= D) {                                                             \
    if (name) *name = "hbm_decode_kernel<" #A ", " #D ">";                                     \
    return (const void*)&hbm_decode_kernel<ALG, D>;                                            \
  }
const void* select_hbm_kernel(int algo, int dcmax, const char** name) {
  QLDPC_HBM(ALGO_MS, 0, 8) QLDPC_HBM(ALGO_MS, 0, 16) QLDPC_HBM(ALGO_MS, 0, 32) QLDPC_HBM(ALGO_MS, 0, 64)
  QLDPC_HBM(ALGO_BP, 1, 8) QLDPC_HBM(ALGO_BP, 1, 16) QLDPC_HBM(ALGO_BP, 1, 32) QLDPC_HBM(ALGO_BP, 1, 64)
  return nullptr;
}
#undef QLDPC_HBM

hipError_t launch_hbm(const void* kernel, const HbmArgs& a, int grid, int block, const int32_t* fl_var,
                      const int32_t* fl_pos, int lazy, hipStream_t stream) {
  void* params[] = {(void*)&a, (void*)&fl_var, (void*)&fl_pos, (void*)&lazy};
  return hipLaunchKernel(kernel, dim3(grid), dim3(block), params, 0, stream);
}

}  // namespace qldpc
