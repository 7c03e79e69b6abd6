/*
 * qldpc_libm.h — NumPy's own float64 tanh / arctanh / log, restated bit for bit.
 *
 * BP_decoder (qLDPCsim/decoders.py:254-259) computes
 *     prod = np.prod(np.tanh(msgs / 2.0));  th2 = prod / np.tanh(v / 2.0)
 *     val  = 2 * np.arctanh(th2)
 * and both decoders start from L = np.log((1 - p) / max(p, eps)) (:147, :232).
 * BP run for 100 iterations is chaotic: a last-bit difference in tanh or
 * atanh grows into different hard decisions. So the GPU kernels and the CPU
 * oracle evaluate exactly the functions NumPy evaluates on the reference's
 * host (NumPy 2.2.6, x86-64 AVX512_SKX dispatch):
 *   np.tanh    -> NumPy simd_tanh_f64 (loops_hyperbolic.dispatch.c.src):
 *                 tanh(|x|) = Horner(c16 .. c0 of interval i)(|x| - b_i), the
 *                 interval from the exponent and top 3 mantissa bits of x;
 *   np.arctanh -> Intel SVML __svml_atanh8_ha (vendored by NumPy, BSD-3):
 *                 0.5 (log(1+|x|) - log(1-|x|)) with each log reduced by a
 *                 4-bit rounded reciprocal R (log(Y) = -log(R) + log1p(R Y - 1),
 *                 R Y - 1 exact by FMA, two-term table of log(1 + i/16)) and
 *                 one shared degree-9 series, summed with error terms;
 *   np.log     -> Intel SVML __svml_log8_ha (host only: the prior L).
 * The tables are NumPy's / SVML's own constants (include/qldpc_numpy_tables.h,
 * generated from the installed NumPy by tools/gen_numpy_libm_tables.py). The
 * SVML reciprocal is vrcp14pd rounded to a 4-bit mantissa; that rounded value
 * is a step function of the top 18 mantissa bits, restated as 16 probed
 * thresholds. Every other step is an IEEE-754 +, -, * or fused multiply-add
 * in round-to-nearest, as in SVML's {rn-sae} code; callers compile with
 * -ffp-contract=off (no other contraction) and the host build with -mfma.
 * tests/test_libm.py checks the three functions against NumPy itself.
 *
 * Table image: host code reads qldpc_libm_host; device kernels stage the same
 * image (qldpc_libm_tab) into LDS and pass pointers into it.
 */
#ifndef QLDPC_LIBM_H
#define QLDPC_LIBM_H

#include <stdint.h>

#include "qldpc_numpy_tables.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define QLDPC_HD __host__ __device__ __forceinline__
#else
#define QLDPC_HD static inline
#endif

QLDPC_HD double qldpc_bits2d(uint64_t u) {
  double d;
  __builtin_memcpy(&d, &u, sizeof d);
  return d;
}

QLDPC_HD uint64_t qldpc_d2bits(double d) {
  uint64_t u;
  __builtin_memcpy(&u, &d, sizeof u);
  return u;
}

#if defined(__HIP_DEVICE_COMPILE__)
/* v_fma_f64 with every operand in a register. Written as __builtin_fma, a
   Horner step q = fma(q, r, c) became v_mov (copy the coefficient c into the
   destination) + v_fmac_f64 (accumulate form, c tied to the destination):
   two VALU ops per step in a VALU-bound kernel. Same operation, same
   rounding. */
__device__ __forceinline__ double qldpc_fma_dev(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
#define QLDPC_FMA(a, b, c) qldpc_fma_dev((a), (b), (c))
/* a / b correctly rounded, for finite b != 0 and NONZERO a, both well inside
   the normal range (2^-500 < |a|, |b| < 2^500). It is the compiler's IEEE
   division sequence (v_rcp_f64, two Newton steps, q = a r, one FMA
   correction) without v_div_scale / v_div_fixup, which are the identity in
   that range: the same result, bit for bit, in 8 instead of 11 VALU ops.
   (a = -0 would come out +0: v_div_fixup is what sets that sign.) Callers
   guarantee the range. */
__device__ __forceinline__ double qldpc_div_dev(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = qldpc_fma_dev(-b, r, 1.0);
  r = qldpc_fma_dev(r, e, r);
  e = qldpc_fma_dev(-b, r, 1.0);
  r = qldpc_fma_dev(r, e, r);
  const double q = a * r;
  const double rem = qldpc_fma_dev(-b, q, a);
  return qldpc_fma_dev(rem, r, q);
}
#define QLDPC_DIV(a, b) qldpc_div_dev((a), (b))
/* the same v_fma_f64 with a wave-uniform addend taken from an SGPR pair (a
   library constant): a "v" operand made the compiler copy every constant
   into VGPRs with a v_mov_b64 per use */
__device__ __forceinline__ double qldpc_fma_dev_s(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}
#define QLDPC_FMA_K(a, b, c) qldpc_fma_dev_s((a), (b), (c))
/* ... and with a wave-uniform multiplier b */
__device__ __forceinline__ double qldpc_fma_dev_sb(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
  return r;
}
#define QLDPC_FMA_KB(a, b, c) qldpc_fma_dev_sb((a), (b), (c))
#else
#define QLDPC_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define QLDPC_FMA_K(a, b, c) __builtin_fma((a), (b), (c))
#define QLDPC_FMA_KB(a, b, c) __builtin_fma((a), (b), (c))
#define QLDPC_DIV(a, b) ((a) / (b))
#endif

/* the table image: NumPy's tanh intervals (rows b, c0 .. c16 as [9][16][2]
   row pairs), SVML atanh's log(1 + i/16) [16][2] (hi, lo) and its
   reciprocal step buckets */
typedef struct __attribute__((aligned(16))) {   /* 16-byte pair reads on the device */
  double tanh_c[16 * 18];
  double atanh_hl[16 * 2];
  uint32_t atanh_rcp[64];
} qldpc_libm_tab;

#define QLDPC_LIBM_TAB_INIT { QLDPC_TANH_LUT_INIT, QLDPC_ATANH_HL_INIT, QLDPC_ATANH_RCP_INIT }

/* np.tanh (NumPy simd_tanh_f64). tc = qldpc_libm_tab.tanh_c. fin != 0 (a
   constant): the caller guarantees |x| < 2^1023 (no NaN, no infinity), where
   the two range selects at the end are the identity, so they are left out. */
QLDPC_HD double qldpc_tanh_x(double x, const double* tc, int fin) {
  const uint64_t u = qldpc_d2bits(x);
  const uint64_t nd = u & 0x7ff8000000000000ull;      /* exponent + top 3 mantissa bits */
  int32_t h = (int32_t)(uint32_t)(nd >> 32) - 0x3fc00000;
  h = h < 0 ? 0 : h;
  h = h > 0x780000 ? 0x780000 : h;
  const double* c = tc + 2 * (h >> 19);               /* interval 0 .. 15; row k at c[32 (k/2) + k%2] */
#if defined(__HIP_DEVICE_COMPILE__)
  /* the nine coefficient pairs as 16-byte LDS reads (ds_read_b128: 4 LDS
     cycles, conflict-free across intervals), all issued before the Horner
     chain; as double loads the compiler emitted ds_read2_b64 (8 cycles,
     2-way conflicts between intervals i and i + 8) with a wait before each
     step. Same coefficients, same operations. */
  typedef double qldpc_d2 __attribute__((ext_vector_type(2)));
  const qldpc_d2* c2 = (const qldpc_d2*)c;            /* pair j (rows 2j, 2j+1) at c2[16 j] */
  qldpc_d2 q[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) q[j] = c2[16 * j];
#define QLDPC_TC(k) q[(k) / 2][(k) & 1]
#else
#define QLDPC_TC(k) c[32 * ((k) / 2) + ((k) & 1)]
#endif
  const double y = qldpc_bits2d(u & 0x7fffffffffffffffull) - QLDPC_TC(0);
  double r = QLDPC_TC(17);
  r = QLDPC_FMA(r, y, QLDPC_TC(16));
  r = QLDPC_FMA(r, y, QLDPC_TC(15));
  r = QLDPC_FMA(r, y, QLDPC_TC(14));
  r = QLDPC_FMA(r, y, QLDPC_TC(13));
  r = QLDPC_FMA(r, y, QLDPC_TC(12));
  r = QLDPC_FMA(r, y, QLDPC_TC(11));
  r = QLDPC_FMA(r, y, QLDPC_TC(10));
  r = QLDPC_FMA(r, y, QLDPC_TC(9));
  r = QLDPC_FMA(r, y, QLDPC_TC(8));
  r = QLDPC_FMA(r, y, QLDPC_TC(7));
  r = QLDPC_FMA(r, y, QLDPC_TC(6));
  r = QLDPC_FMA(r, y, QLDPC_TC(5));
  r = QLDPC_FMA(r, y, QLDPC_TC(4));
  r = QLDPC_FMA(r, y, QLDPC_TC(3));
  r = QLDPC_FMA(r, y, QLDPC_TC(2));
  r = QLDPC_FMA(r, y, QLDPC_TC(1));
#undef QLDPC_TC
  if (!fin) r = nd <= 0x7fe0000000000000ull ? r : 1.0;   /* |x| >= 2^1023, inf */
  r = qldpc_bits2d(qldpc_d2bits(r) | (u & 0x8000000000000000ull));
  return (fin || x == x) ? r : qldpc_bits2d(0x7ff8000000000000ull);
}

QLDPC_HD double qldpc_tanh_t(double x, const double* tc) { return qldpc_tanh_x(x, tc, 0); }

/* vrcp14pd(Y) rounded half-up to a 4-bit mantissa (SVML atanh), for a
   positive normal Y: R = 2^-e (1 - c/32) with c = the number of probed steps
   at or below Y's mantissa (bucketed by its top 6 bits); *ge = getexp(R). */
QLDPC_HD double qldpc_svml_rrcp(double Y, const uint32_t* rb, double* ge, int* ti) {
  const uint64_t u = qldpc_d2bits(Y);
  const int e = (int)((u >> 52) & 0x7ff) - 1023;
  const uint32_t p = (uint32_t)(u >> 34) & 0x3ffffu;
  const uint32_t ent = rb[p >> 12];
  const int c = (int)(ent & 0xffu) + (p >= (ent >> 8) ? 1 : 0);
  *ge = (double)((c == 0 ? 0 : -1) - e);
  *ti = (16 - c) & 15;                                 /* table index = R's top mantissa bits */
  return qldpc_bits2d(((uint64_t)(0x3ff0 - c) << 48) + ((uint64_t)(int64_t)(-e) << 52));
}

/* np.arctanh (SVML __svml_atanh8_ha). hl = qldpc_libm_tab.atanh_hl, rb =
   .atanh_rcp. |x| >= 1 and NaN take SVML's rare path: +-inf at |x| == 1,
   NaN otherwise (signs / payloads as below; BP flags them non-finite).
   fin != 0 (a constant): the caller guarantees |x| < 1, so the rare-path
   tests are left out. */
QLDPC_HD double qldpc_atanh_x(double x, const double* hl, const uint32_t* rb, int fin) {
  const uint64_t u = qldpc_d2bits(x);
  const uint64_t sgn = u & 0x8000000000000000ull;
  const double ax = qldpc_bits2d(u & 0x7fffffffffffffffull);
  if (!fin && !(ax == ax)) return x;
  if (!fin && ax >= 1.0) return qldpc_bits2d(((ax == 1.0) ? 0x7ff0000000000000ull : 0x7ff8000000000000ull) | sgn);
  const double Yp = ax + 1.0, Ym = 1.0 - ax;
  const double Yp_lo = ax - (Yp - 1.0);                /* 1 + ax = Yp + Yp_lo */
  const double Ym_nlo = ax + (Ym - 1.0);               /* 1 - ax = Ym - Ym_nlo */
  double gp, gm;
  int ip, im;
  const double Rp = qldpc_svml_rrcp(Yp, rb, &gp, &ip);
  const double Rm = qldpc_svml_rrcp(Ym, rb, &gm, &im);
  const double dp = QLDPC_FMA(Yp_lo, Rp, QLDPC_FMA(Rp, Yp, -1.0));   /* Rp (1 + ax) - 1 */
  const double dm = QLDPC_FMA(-Ym_nlo, Rm, QLDPC_FMA(Ym, Rm, -1.0)); /* Rm (1 - ax) - 1 */
  const double ediff = gm - gp;
#if defined(__HIP_DEVICE_COMPILE__)
  /* (hi, lo) of log(1 + i/16) as one 16-byte LDS read per index */
  typedef double qldpc_d2 __attribute__((ext_vector_type(2)));
  const qldpc_d2 hm = ((const qldpc_d2*)hl)[im], hp = ((const qldpc_d2*)hl)[ip];
  const double hdiff = hm[0] - hp[0], ldiff = hm[1] - hp[1];
#else
  const double hdiff = hl[2 * im] - hl[2 * ip], ldiff = hl[2 * im + 1] - hl[2 * ip + 1];
#endif
  double Pp = QLDPC_FMA_K(dp, QLDPC_ATANH_C0, QLDPC_ATANH_C1);   /* C0 dp + C1 (fma commutes a, b) */
  double Pm = QLDPC_FMA_K(dm, QLDPC_ATANH_C0, QLDPC_ATANH_C1);
  const double K = QLDPC_FMA_KB(ediff, QLDPC_ATANH_LN2HI, hdiff);
  Pp = QLDPC_FMA_K(dp, Pp, QLDPC_ATANH_C2);
  Pm = QLDPC_FMA_K(dm, Pm, QLDPC_ATANH_C2);
  Pp = QLDPC_FMA_K(dp, Pp, QLDPC_ATANH_C3);
  Pm = QLDPC_FMA_K(dm, Pm, QLDPC_ATANH_C3);
  const double Klo = QLDPC_FMA_KB(ediff, QLDPC_ATANH_LN2LO, ldiff);
  const double dp2 = dp * dp;
  Pp = QLDPC_FMA_K(dp, Pp, QLDPC_ATANH_C4);
  Pm = QLDPC_FMA_K(dm, Pm, QLDPC_ATANH_C4);
  const double S1 = dp + K;
  Pp = QLDPC_FMA_K(dp, Pp, QLDPC_ATANH_C5);
  Pm = QLDPC_FMA_K(dm, Pm, QLDPC_ATANH_C5);
  const double dm2 = dm * dm;
  Pp = QLDPC_FMA_K(dp, Pp, QLDPC_ATANH_C6);
  Pm = QLDPC_FMA_K(dm, Pm, QLDPC_ATANH_C6);
  const double t4 = K - S1;
  const double S2 = S1 - dm;
  Pp = QLDPC_FMA_K(dp, Pp, QLDPC_ATANH_C7);
  Pm = QLDPC_FMA_K(dm, Pm, QLDPC_ATANH_C7);
  Pp = QLDPC_FMA_K(dp, Pp, QLDPC_ATANH_C8);
  Pm = QLDPC_FMA_K(dm, Pm, QLDPC_ATANH_C8);
  const double e1 = dp + t4;                           /* rounding error of S1 */
  const double t5 = S2 - S1;
  const double A = QLDPC_FMA(dp2, Pp, Klo);
  const double B = QLDPC_FMA(-dm2, Pm, e1);
  const double e2 = dm + t5;                           /* (minus) rounding error of S2 */
  const double r = S2 + ((A + B) - e2);
  return r * qldpc_bits2d(0x3fe0000000000000ull | sgn);   /* +-0.5 */
}

QLDPC_HD double qldpc_atanh_t(double x, const double* hl, const uint32_t* rb) {
  return qldpc_atanh_x(x, hl, rb, 0);
}

/* np.exp (SVML __svml_exp8_ha, DOUBLE_exp_AVX512_SKX's loop for operands
   that do not overlap) for |x| < QLDPC_EXP_RARE, NaN included (propagated);
   hl = QLDPC_EXP_HL_INIT (2^(j/16) hi, lo pairs). SVML:
     z = fma_rz(x, log2e, S)       S = 1.5 * 2^48 (+ 0x3ff0 ulps): z - S = k/16,
                                   k = floor(16 x log2e) (rounding toward zero,
                                   the sum being positive), j = k mod 16 = the
                                   low 4 bits of z
     r = (x - N ln2hi) - N ln2lo   N = z - S, two FMAs; bit 62 of r cleared
     p = r (c0 + c1 r + ... + c5 r^5) + lo_j   (Estrin, as the SVML code)
     exp(x) = scalef(hi_j p + hi_j, N) = (hi_j p + hi_j) * 2^floor(N)
   The FMA in round-toward-zero is restated in round-to-nearest: z_rn, then
   the sign of the exact x log2e + S - z_rn (one FMA: S - z_rn is exact, and
   a round-to-nearest result keeps the sign of a nonzero exact value) says
   whether z_rn lies above the exact sum, where z_rz is the next value down
   (same binade: |x log2e| <= 1022 << 2^48). Used by the OSD reliability key
   (decoders.py:323) only, whose clipped arguments lie in [-100, 100]. */
QLDPC_HD double qldpc_np_exp_t(double x, const double* hl) {
  const double S = qldpc_bits2d(QLDPC_EXP_SHIFTER_BITS);
  if (x != x) return x;                          /* scalef(., NaN) = NaN */
  const double zr = QLDPC_FMA(x, QLDPC_EXP_LOG2E, S);
  const double below = QLDPC_FMA(x, QLDPC_EXP_LOG2E, S - zr);
  const uint64_t zb = qldpc_d2bits(zr) - (below < 0.0 ? 1u : 0u);
  const double N = qldpc_bits2d(zb) - S;                       /* k / 16, exact */
  const int64_t k = (int64_t)(zb - QLDPC_EXP_SHIFTER_BITS);     /* (same binade) */
  const int j = (int)(k & 15);
  double r = QLDPC_FMA(-N, QLDPC_EXP_LN2HI, x);
  r = QLDPC_FMA(-QLDPC_EXP_LN2LO, N, r);
  r = qldpc_bits2d(qldpc_d2bits(r) & QLDPC_EXP_RMASK_BITS);
  const double r2 = r * r;
  double a = QLDPC_FMA(QLDPC_EXP_C5, r, QLDPC_EXP_C4);
  const double b = QLDPC_FMA(QLDPC_EXP_C3, r, QLDPC_EXP_C2);
  const double c = QLDPC_FMA(QLDPC_EXP_C1, r, QLDPC_EXP_C0);
  a = QLDPC_FMA(a, r2, b);
  a = QLDPC_FMA(a, r2, c);
  const double hi = hl[2 * j], lo = hl[2 * j + 1];
  const double p = QLDPC_FMA(r, a, lo);
  const double res = QLDPC_FMA(hi, p, hi);
  /* scalef by floor(N) = k >> 4: an exact power-of-two scaling (the result
     is normal for |x| <= 700) */
  int64_t e = k >> 4;
  e = e < -1022 ? -1022 : (e > 1023 ? 1023 : e);
  return res * qldpc_bits2d((uint64_t)(1023 + e) << 52);
}

/* The OSD reliability key of one posterior, NumPy's element for element
   (decoders.py:320-324): sat = P if |P| < 100 else 100 sign(P) (NaN stays
   NaN), prob = 1 / (1 + np.exp(sat)), key = prob if prob > 0.5 else 1 - prob.
   Each step an IEEE-754 double operation in round-to-nearest (the divide and
   add are NumPy's AVX-512 loops: correctly rounded). The key lies in
   [0.5, 1] or is NaN. */
QLDPC_HD double qldpc_osd_key_t(double P, const double* hl) {
  const double aP = P < 0.0 ? -P : P;
  const double sat = aP < 100.0 ? P : (P > 0.0 ? 100.0 : (P < 0.0 ? -100.0 : P));
  const double t = 1.0 + qldpc_np_exp_t(sat, hl);
  const double prob = 1.0 / t;
  return prob > 0.5 ? prob : 1.0 - prob;
}

/* host image of the tables (the oracle, the library's host code; in HIP
   sources these are host functions, never emitted for the device) */
static const qldpc_libm_tab qldpc_libm_host = QLDPC_LIBM_TAB_INIT;
static const uint64_t qldpc_log_rcp_t[16] = QLDPC_LOG_RCP_T_INIT;
static const double qldpc_log_ab[32] = QLDPC_LOG_AB_INIT;
static const double qldpc_exp_hl[32] = QLDPC_EXP_HL_INIT;

static inline double qldpc_np_exp(double x) { return qldpc_np_exp_t(x, qldpc_exp_hl); }
static inline double qldpc_osd_key(double P) { return qldpc_osd_key_t(P, qldpc_exp_hl); }

static inline double qldpc_tanh(double x) { return qldpc_tanh_t(x, qldpc_libm_host.tanh_c); }
static inline double qldpc_atanh(double x) {
  return qldpc_atanh_t(x, qldpc_libm_host.atanh_hl, qldpc_libm_host.atanh_rcp);
}

/* np.log (SVML __svml_log8_ha) for positive normal finite x; other inputs
   (0, negative, subnormal, inf, NaN — SVML's rare path) return NaN, -inf or
   the input as IEEE log does. The prior L = log((1-p)/max(p, eps)) only
   ever sees finite positive normal arguments. */
static inline double qldpc_np_log(double x) {
  const uint64_t u = qldpc_d2bits(x);
  const int ex = (int)((u >> 52) & 0x7ff);
  if (x != x || x < 0.0) return qldpc_bits2d(0x7ff8000000000000ull);
  if (x == 0.0) return -qldpc_bits2d(0x7ff0000000000000ull);
  if (ex == 0x7ff) return x;
  if (ex == 0) return qldpc_bits2d(0x7ff8000000000000ull);   /* subnormal: not restated */
  double e = (double)(ex - 1023);
  const uint64_t mb = u & 0x000fffffffffffffull;
  const double m = qldpc_bits2d(mb | 0x3ff0000000000000ull);            /* getmant [1, 2) */
  int c = 0;
  for (int k = 0; k < 16; ++k) c += mb >= qldpc_log_rcp_t[k];
  const double R = qldpc_bits2d((uint64_t)(0x3ff0 - c) << 48);          /* vrndscale(vrcp14(m), 2^-5) */
  const int idx = (16 - c) & 15;
  const double r = __builtin_fma(R, m, -QLDPC_LOG_C100);
  const double A1 = __builtin_fma(QLDPC_LOG_C200, r, QLDPC_LOG_C240);
  const double A0 = __builtin_fma(QLDPC_LOG_C180, r, QLDPC_LOG_C1c0);
  const double r2 = r * r;
  const double A2 = __builtin_fma(QLDPC_LOG_C280, r, QLDPC_LOG_C2c0);
  const double B0 = __builtin_fma(r2, A0, A1);
  const double r4 = r2 * r2;
  const double A3 = __builtin_fma(QLDPC_LOG_C300, r, QLDPC_LOG_C340);
  if (R < QLDPC_LOG_C140) e = e + QLDPC_LOG_C100;
  const double B1 = __builtin_fma(r2, A2, A3);
  const double H = __builtin_fma(QLDPC_LOG_C380, e, qldpc_log_ab[2 * idx]);
  const double P = __builtin_fma(r4, B0, B1);
  const double S = H + r;
  const double err = r - (S - H);
  const double Q = __builtin_fma(r2, P, err);
  const double E2 = __builtin_fma(QLDPC_LOG_C3c0, e, qldpc_log_ab[2 * idx + 1]);
  return S + (Q + E2);
}

/* L_ch = np.log((1 - p) / max(p, eps))   (decoders.py:147, :232) */
static inline double qldpc_prior_llr(double p, double eps) {
  return qldpc_np_log((1.0 - p) / (p > eps ? p : eps));
}

#endif /* QLDPC_LIBM_H */
