/*
 * qldpc_oracle.c — CPU restatement of the reference decoders, TEST
 * INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle for the MI355X decoder. It is never linked
 * into, loaded by, or called from the product (qldpcsim_amd/); only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / CPU baseline. Parity pinned: tests/test_oracle_golden.py checks
 * it against golden vectors captured from the unmodified reference decoders
 * (tests/golden/gen_golden.py).
 *
 * Reference: albertogp71/qLDPCsim @ 2025-12-26, qLDPCsim/decoders.py.
 *   MS_decoder  decoders.py:110-182   (normalized min-sum, dense m x n NumPy)
 *   BP_decoder  decoders.py:189-290   (sum-product on an edge list)
 * The restatement is sparse (CSR/CSC) but reproduces the reference's exact
 * floating-point contract:
 *   MS: c2v stored float32, rounded once from a float64 product
 *       (decoders.py:167-168); VN sum = float32 sequential sum over rows in
 *       ascending check order (np.sum axis=0, :172); posterior and v2c float64
 *       (:173, :177); the first layer of the first iteration sees float32(L)
 *       (:148-149).
 *   BP: float64; product of tanh = sequential fold (np.prod, :254); division
 *       extrinsic (:256); eps clip (:257-258); column sums follow NumPy's
 *       pairwise_sum (0.0 + pairwise(all), 8-accumulator blocks for n >= 8,
 *       :269/:276). tanh/atanh (and, for both decoders, the log of the prior)
 *       come from include/qldpc_libm.h: NumPy's own float64 tanh and SVML's
 *       atanh / log as NumPy runs them on the reference's host, restated bit
 *       for bit — the same code the GPU kernels run, so GPU, oracle and
 *       reference agree bit for bit, 100-iteration chaotic decodes included.
 * Build: oracle/Makefile  ->  oracle/_build/libqldpc_oracle.so
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/qldpc_libm.h" /* NumPy-exact tanh/atanh/log, shared with the GPU kernels */

#define ORACLE_FLAG_MIN_ZERO 1  /* MS: a check saw min|v| == 0 (App. A.1.6 leak case, not emulated) */
#define ORACLE_FLAG_NONFINITE 2 /* BP: tanh(v/2)==0 or a non-finite message */

typedef struct {
    int m, n, E;
    const int32_t *row_ptr, *col_idx; /* CSR, ascending column per row (np.where(H) order) */
    int32_t *col_ptr, *col_edge;      /* CSC: per column, CSR edge ids in ascending row order */
} graph_t;

static int graph_init(graph_t *g, int m, int n, const int32_t *row_ptr, const int32_t *col_idx) {
    g->m = m; g->n = n; g->E = row_ptr[m];
    g->row_ptr = row_ptr; g->col_idx = col_idx;
    g->col_ptr = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
    g->col_edge = (int32_t *)malloc(sizeof(int32_t) * (size_t)(g->E > 0 ? g->E : 1));
    if (!g->col_ptr || !g->col_edge) return -1;
    for (int e = 0; e < g->E; ++e) g->col_ptr[col_idx[e] + 1]++;
    for (int j = 0; j < n; ++j) g->col_ptr[j + 1] += g->col_ptr[j];
    int32_t *fill = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    memcpy(fill, g->col_ptr, sizeof(int32_t) * (size_t)n);
    for (int r = 0; r < m; ++r)               /* rows ascending => CSC lists ascending */
        for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) g->col_edge[fill[col_idx[e]]++] = e;
    free(fill);
    return 0;
}

static void graph_free(graph_t *g) { free(g->col_ptr); free(g->col_edge); }

/* H.dot(e_hat) % 2 == syndrome  (decoders.py:175, :283-284) */
static int syndrome_ok(const graph_t *g, const uint8_t *ehat, const uint8_t *syn) {
    for (int r = 0; r < g->m; ++r) {
        int par = 0;
        for (int e = g->row_ptr[r]; e < g->row_ptr[r + 1]; ++e) par ^= ehat[g->col_idx[e]];
        if (par != (syn[r] & 1)) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------- */
/* Min-Sum (decoders.py:110-182)                                             */
/* ------------------------------------------------------------------------- */
static int ms_decode_one(const graph_t *g, const uint8_t *syn, double p, int max_iter,
                         int n_layers, const int32_t *layer_ptr, const int32_t *layer_rows,
                         double beta, double eps, uint8_t *ehat, double *post_out,
                         int *flags, float *c2v, float *c2v_new, float *S, double *post) {
    const int n = g->n;
    const double L = qldpc_prior_llr(p, eps);               /* :147 np.log (np.float64) */
    const float L32 = (float)L;                              /* :148-149 float32 store */
    for (int e = 0; e < g->E; ++e) c2v[e] = 0.0f;           /* :150 */
    for (int j = 0; j < n; ++j) { S[j] = 0.0f; post[j] = L + (double)0.0f; }
    int first = 1;
    *flags = 0;
    for (int it = 0; it < max_iter; ++it) {
        for (int l = 0; l < n_layers; ++l) {
            const int r0 = layer_ptr[l], r1 = layer_ptr[l + 1];
            /* Check-node update (:155-169), Jacobi over the layer: new values are
               staged and committed after the whole layer has been computed. */
            for (int q = r0; q < r1; ++q) {
                const int r = layer_rows[q];
                const int e0 = g->row_ptr[r], e1 = g->row_ptr[r + 1];
                if (e1 == e0) continue;
                double min1 = INFINITY, min2 = INFINITY;
                int argk = -1, negprod = syn[r] & 1;  /* syn_sign (:151) folded into the sign product */
                for (int e = e0; e < e1; ++e) {
                    const double v = first ? (double)L32 : post[g->col_idx[e]] - (double)c2v[e];
                    const double a = fabs(v);
                    negprod ^= (v < 0.0);              /* np.sign, 0 -> +1 (:157-158) */
                    if (a < min1) { min2 = min1; min1 = a; argk = e; }  /* first argmin (:161) */
                    else if (a < min2) { min2 = a; }                  /* min over the rest (:162-164) */
                }
                if (isinf(min1)) min1 = 0.0;          /* :165 */
                if (isinf(min2)) min2 = 0.0;          /* :166 */
                if (min1 == 0.0) *flags |= ORACLE_FLAG_MIN_ZERO;
                for (int e = e0; e < e1; ++e) {
                    const double v = first ? (double)L32 : post[g->col_idx[e]] - (double)c2v[e];
                    const int neg = (v < 0.0) ^ negprod;     /* syn * prod * sign / sign_e */
                    /* |v_e| == min1 gets min2 (:167-168); with ties min2 == min1. */
                    const double mag = (e == argk) ? min2 : min1;
                    const double val = beta * mag;           /* exact product order: beta*syn*prod*min/sign */
                    c2v_new[e] = (float)(neg ? -val : val);
                }
            }
            for (int q = r0; q < r1; ++q) {
                const int r = layer_rows[q];
                for (int e = g->row_ptr[r]; e < g->row_ptr[r + 1]; ++e) c2v[e] = c2v_new[e];
            }
            first = 0;
            /* Variable-node update (:172-174): float32 sequential column sums. */
            for (int j = 0; j < n; ++j) {
                float acc = 0.0f;
                for (int k = g->col_ptr[j]; k < g->col_ptr[j + 1]; ++k) acc += c2v[g->col_edge[k]];
                S[j] = acc;
                post[j] = L + (double)S[j];
                ehat[j] = post[j] < 0.0;
            }
            if (syndrome_ok(g, ehat, syn)) {          /* :175-176 */
                if (post_out) memcpy(post_out, post, sizeof(double) * (size_t)n);
                return it + 1;
            }
        }
    }
    if (post_out) memcpy(post_out, post, sizeof(double) * (size_t)n);
    return max_iter;                                   /* :182 (OSD applied by the caller) */
}

/* ------------------------------------------------------------------------- */
/* BP (decoders.py:189-290)                                                  */
/* ------------------------------------------------------------------------- */

/* NumPy DOUBLE_pairwise_sum (used by np.sum for a contiguous 1-D float64). */
static double np_pairwise(const double *a, long n) {
    if (n < 8) {
        double res = -0.0;
        for (long i = 0; i < n; ++i) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        long i;
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
    }
}

static double np_sum(const double *a, long n) { return 0.0 + np_pairwise(a, n); }

static int bp_decode_one(const graph_t *g, const uint8_t *syn, double p, int max_iter,
                         int n_layers, const int32_t *layer_ptr, const int32_t *layer_rows,
                         double eps, uint8_t *ehat, double *post_out, int *flags,
                         double *v2c, double *c2v, double *tmp, double *post) {
    const int n = g->n;
    const double L0 = qldpc_prior_llr(p, eps);              /* :232 np.log */
    for (int e = 0; e < g->E; ++e) { v2c[e] = L0; c2v[e] = 0.0; }  /* :235-236 */
    *flags = 0;
    for (int it = 0; it < max_iter; ++it) {
        for (int l = 0; l < n_layers; ++l) {
            for (int q = layer_ptr[l]; q < layer_ptr[l + 1]; ++q) {  /* :249-262 */
                const int i = layer_rows[q];
                const int e0 = g->row_ptr[i], e1 = g->row_ptr[i + 1];
                if (e1 == e0) continue;
                double prod = 1.0;
                for (int e = e0; e < e1; ++e) prod *= qldpc_tanh(v2c[e] / 2.0);
                for (int e = e0; e < e1; ++e) {
                    const double t = qldpc_tanh(v2c[e] / 2.0);
                    double th2 = prod / t;
                    if (t == 0.0) *flags |= ORACLE_FLAG_NONFINITE;
                    if (fabs(th2) >= 1.0 - eps) th2 = th2 - eps * (th2 > 0 ? 1.0 : (th2 < 0 ? -1.0 : 0.0));
                    double val = 2.0 * qldpc_atanh(th2);
                    if (syn[i] & 1) val = -val;
                    c2v[e] = val;
                }
            }
            for (int j = 0; j < n; ++j) {                /* :265-278 */
                const int k0 = g->col_ptr[j], k1 = g->col_ptr[j + 1];
                if (k1 == k0) { post[j] = L0; ehat[j] = post[j] < 0.0; continue; }
                for (int k = k0; k < k1; ++k) tmp[k - k0] = c2v[g->col_edge[k]];
                const double tot = L0 + np_sum(tmp, k1 - k0);
                for (int k = k0; k < k1; ++k) v2c[g->col_edge[k]] = tot - c2v[g->col_edge[k]];
                post[j] = tot;
                ehat[j] = post[j] < 0.0;                  /* :280 */
            }
            if (syndrome_ok(g, ehat, syn)) {              /* :283-285 */
                if (post_out) memcpy(post_out, post, sizeof(double) * (size_t)n);
                return it + 1;
            }
        }
    }
    if (post_out) memcpy(post_out, post, sizeof(double) * (size_t)n);
    return max_iter;                                       /* :290 */
}

/* ------------------------------------------------------------------------- */
/* Batched entry points (OpenMP over shots).                                  */
/* algo: 0 = MS, 1 = BP.  syn u8[B*m], ehat u8[B*n], iters i32[B],           */
/* post f64[B*n] (nullable), flags i32[B] (nullable).  Returns 0 on success. */
/* ------------------------------------------------------------------------- */
int oracle_decode_batch(int algo, int m, int n, const int32_t *row_ptr, const int32_t *col_idx,
                        int n_layers, const int32_t *layer_ptr, const int32_t *layer_rows,
                        const uint8_t *syn, long B, double p, int max_iter, double beta,
                        double eps, uint8_t *ehat, int32_t *iters, double *post, int32_t *flags,
                        int nthreads) {
    graph_t g;
    if (graph_init(&g, m, n, row_ptr, col_idx)) return -1;
    int rc = 0;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
    {
        const size_t E = (size_t)(g.E > 0 ? g.E : 1), N = (size_t)(n > 0 ? n : 1);
        double *d0 = (double *)malloc(sizeof(double) * (2 * E + E + 2 * N));
        float *f0 = (float *)malloc(sizeof(float) * (2 * E + N));
        if (!d0 || !f0) {
#pragma omp atomic write
            rc = -1;
        } else {
#pragma omp for schedule(dynamic, 16)
            for (long b = 0; b < B; ++b) {
                int fl = 0;
                int it;
                if (algo == 0)
                    it = ms_decode_one(&g, syn + b * m, p, max_iter, n_layers, layer_ptr, layer_rows,
                                       beta, eps, ehat + b * n, post ? post + b * n : NULL, &fl,
                                       f0, f0 + E, f0 + 2 * E, d0);
                else
                    it = bp_decode_one(&g, syn + b * m, p, max_iter, n_layers, layer_ptr, layer_rows,
                                       eps, ehat + b * n, post ? post + b * n : NULL, &fl,
                                       d0, d0 + E, d0 + 2 * E, d0 + 3 * E);
                iters[b] = it;
                if (flags) flags[b] = fl;
            }
        }
        free(d0);
        free(f0);
    }
    graph_free(&g);
    return rc;
}

/* ------------------------------------------------------------------------
 * Channel sampler restatement (checker for qldpc_channel_sample,
 * channel_kernels.hip). The shot source it replaces is the reference's Stim
 * circuit sample (simulator.py:107 PAULI_CHANNEL_1(p/3,p/3,p/3) on every data
 * qubit, :196-197 sampling, :249-252 row slicing); this stream is its
 * statistical equivalent, so parity is defined on the
 * stream itself: Philox4x32-10 as published by Salmon, Moraes, Dror and
 * Shaw, "Parallel random numbers: as easy as 1, 2, 3" (SC'11), round
 * multipliers 0xD2511F53 / 0xCD9E8D57, Weyl key increments 0x9E3779B9 /
 * 0xBB67AE85. Outputs are unpacked bytes (errX, errZ uint8 [B][n]). */
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

int oracle_channel_sample(int n, int mx, const int32_t *rpx, const int32_t *cix, int mz,
                          const int32_t *rpz, const int32_t *ciz, uint64_t t1, uint64_t t2,
                          uint64_t t3, uint64_t seed, uint64_t shot0, long batch, uint8_t *errx,
                          uint8_t *errz, uint8_t *syz, uint8_t *syx) {
  for (long b = 0; b < batch; ++b) {
    const uint64_t s = shot0 + (uint64_t)b;
    uint8_t *ex = errx + b * (long)n, *ez = errz + b * (long)n;
    for (int j = 0; j < n; ++j) {
      const int w = j / 64;
      uint32_t c[4] = {(uint32_t)(j % 64), (uint32_t)(w / 4), (uint32_t)s, (uint32_t)(s >> 32)};
      philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
      const uint64_t u = c[w % 4];
      ex[j] = u < t2;                 /* X or Y */
      ez[j] = u >= t1 && u < t3;      /* Y or Z */
    }
    for (int r = 0; r < mz; ++r) {
      int par = 0;
      for (int e = rpz[r]; e < rpz[r + 1]; ++e) par ^= ex[ciz[e]];
      syz[b * (long)mz + r] = (uint8_t)par;
    }
    for (int r = 0; r < mx; ++r) {
      int par = 0;
      for (int e = rpx[r]; e < rpx[r + 1]; ++e) par ^= ez[cix[e]];
      syx[b * (long)mx + r] = (uint8_t)par;
    }
  }
  return 0;
}

/* raw block function, for the published known-answer vectors (tests) */
void oracle_philox4x32_10(uint32_t *ctr, uint32_t k0, uint32_t k1) { philox4x32_10(ctr, k0, k1); }
