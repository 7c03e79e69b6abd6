/*
 * qldpc_libm.h — reproducible double-precision tanh / atanh for BP.
 *
 * BP_decoder (qLDPCsim/decoders.py:254-259) computes 2*atanh(prod/tanh(v/2)),
 * with atanh evaluated next to +-1 where it is ill-conditioned (|th2| up to
 * 1 - 1e-9): a one-ULP difference between two libms' tanh grows into ~1e-4
 * relative differences in converged posteriors. To make the GPU kernel and the
 * CPU oracle agree bit for bit, both evaluate these two functions with this
 * header: only IEEE-754 +, -, *, / and explicit fused multiply-add (each
 * correctly rounded on gfx950 — v_fma_f64 — and on x86-64 with FMA3; callers
 * compile with -ffp-contract=off so no other contraction happens, and the
 * host build needs -mfma so fma is the instruction, not glibc's emulation),
 * integer bit operations and comparisons. Accuracy against NumPy's
 * tanh/arctanh: <= 3 ULP over the BP domain (tests/test_libm.py).
 *
 * Method: tanh = e/(e+2), e = expm1(2|x|) (Cody–Waite reduction y = k ln2 + r,
 * |r| <= ln2/2, degree-14 Taylor polynomial, 2^k (1 + expm1 r) - 1
 * reassembled exactly); atanh(a) = k ln2/2 + atanh(s), s = (N - D 2^k) /
 * (N + D 2^k) with N = 1 + a and D = 1 - a held as exact two-term sums and
 * 2^k the power of two nearest N / D (|s| <= 3 - 2 sqrt2; odd series in s).
 * One division each and no data-dependent branches below the special values,
 * because GPU lanes diverge (atanh: 133 -> ~60 gfx950 instructions; fewer
 * 2-3 ULP cases than the fdlibm log1p form it replaced).
 */
#ifndef QLDPC_LIBM_H
#define QLDPC_LIBM_H

#include <stdint.h>

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
/* a / b correctly rounded, for finite b != 0 and operands whose exponents lie
   well inside the normal range (here: 2^-500 < |a|, |b| < 2^500, or a == 0).
   It is the compiler's IEEE division sequence (v_rcp_f64, two Newton steps,
   q = a r, one FMA correction) without v_div_scale / v_div_fixup, which are the
   identity in that range: the same result, bit for bit, in 8 instead of 11
   VALU ops. Callers guarantee the range. */
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
#else
#define QLDPC_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define QLDPC_DIV(a, b) ((a) / (b))
#endif

#define QLDPC_LN2_HI 6.93147180369123816490e-01 /* 0x3fe62e42fee00000: k*LN2_HI exact for |k| < 2^11 */
#define QLDPC_LN2_LO 1.90821492927058770002e-10 /* 0x3dea39ef35793c76 */
#define QLDPC_INV_LN2 1.44269504088896338700e+00

/* e^r - 1 for |r| <= ln2/2 (+ a little): r + r^2 * sum_{k>=2} r^(k-2)/k!
   (Horner with fused multiply-adds) */
QLDPC_HD double qldpc_expm1_small(double r) {
  double q = 1.0 / 87178291200.0;                 /* 1/14! */
  q = QLDPC_FMA(q, r, 1.0 / 6227020800.0);        /* 1/13! */
  q = QLDPC_FMA(q, r, 1.0 / 479001600.0);         /* 1/12! */
  q = QLDPC_FMA(q, r, 1.0 / 39916800.0);          /* 1/11! */
  q = QLDPC_FMA(q, r, 1.0 / 3628800.0);           /* 1/10! */
  q = QLDPC_FMA(q, r, 1.0 / 362880.0);            /* 1/9!  */
  q = QLDPC_FMA(q, r, 1.0 / 40320.0);             /* 1/8!  */
  q = QLDPC_FMA(q, r, 1.0 / 5040.0);              /* 1/7!  */
  q = QLDPC_FMA(q, r, 1.0 / 720.0);               /* 1/6!  */
  q = QLDPC_FMA(q, r, 1.0 / 120.0);               /* 1/5!  */
  q = QLDPC_FMA(q, r, 1.0 / 24.0);                /* 1/4!  */
  q = QLDPC_FMA(q, r, 1.0 / 6.0);                 /* 1/3!  */
  q = QLDPC_FMA(q, r, 0.5);                       /* 1/2!  */
  return QLDPC_FMA(r * r, q, r);
}

/* e^y - 1 for 0 <= y <= 64 */
QLDPC_HD double qldpc_expm1_pos(double y) {
  const int k = (int)(y * QLDPC_INV_LN2 + 0.5);
  const double fk = (double)k;
  const double r = QLDPC_FMA(-fk, QLDPC_LN2_LO, y - fk * QLDPC_LN2_HI);  /* fk*LN2_HI exact */
  const double em = qldpc_expm1_small(r);
  const double two_k = qldpc_bits2d((uint64_t)(k + 1023) << 52);
  return QLDPC_FMA(two_k, em, two_k - 1.0);      /* two_k - 1 exact for k <= 53; k = 0: em */
}

QLDPC_HD double qldpc_tanh(double x) {
  const uint64_t sgn = qldpc_d2bits(x) & 0x8000000000000000ull;
  const double a = qldpc_bits2d(qldpc_d2bits(x) & 0x7fffffffffffffffull);
  if (!(a == a)) return x;                        /* NaN */
  /* branch-free (lanes diverge): the range cases are selects */
  const double ac = a < 22.0 ? a : 22.0;
  const double em = qldpc_expm1_pos(ac + ac);
  double t = QLDPC_DIV(em, em + 2.0);             /* one division (<= 3 ULP); em + 2 in [2, 2^64],
                                                     em = 0 or > 2^-500 where t is kept */
  t = a >= 22.0 ? 1.0 : t;                        /* 1 - tanh(22) < 2^-62 */
  t = a < 3.7252902984e-09 ? a : t;               /* 2^-28: tanh(x) = x in double */
  return qldpc_bits2d(qldpc_d2bits(t) | sgn);
}

/* log(1 + f) for f > -1 */
QLDPC_HD double qldpc_log1p(double f) {
  if (!(f == f)) return f;
  if (f <= -1.0) return (f == -1.0) ? -qldpc_bits2d(0x7ff0000000000000ull) : qldpc_bits2d(0x7ff8000000000000ull);
  const double af = f < 0 ? -f : f;
  if (af < 5.551115123125783e-17) return f;        /* 2^-54 */
  if (f == qldpc_bits2d(0x7ff0000000000000ull)) return f;
  int k = 0;
  double fm = f, c = 0.0;
  if (!(f > -0.2928932188134524 && f < 0.41421356237309503)) {
    /* u = 1 + f = 2^k m, m in [sqrt2/2, sqrt2); c = rounding error of u,
       relative to u (fdlibm's c). Inside (1/sqrt2 - 1, sqrt2 - 1), k = 0 and
       f itself is the reduced argument (no rounding, no correction). */
    const double u = 1.0 + f;
    const uint64_t ub = qldpc_d2bits(u);
    k = (int)((ub >> 52) & 0x7ff) - 1023;
    uint64_t mb = (ub & 0x000fffffffffffffull) | 0x3ff0000000000000ull;   /* m in [1, 2) */
    if (mb > 0x3ff6a09e667f3bcdull) {                                     /* m > sqrt(2) */
      mb = (mb & 0x000fffffffffffffull) | 0x3fe0000000000000ull;          /* m / 2 */
      k += 1;
    }
    fm = qldpc_bits2d(mb) - 1.0;                   /* exact (Sterbenz) */
    if (k < 54) {
      /* c / u needs ~1e-6 relative accuracy only (|c/u| <= 2^-53 here and
         the result is >= 0.34): multiply by a three-step Newton reciprocal of
         the mantissa instead of dividing. */
      const double cc = (k > 0) ? 1.0 - (u - f) : f - (u - 1.0);
      const double mu = qldpc_bits2d((ub & 0x000fffffffffffffull) | 0x3ff0000000000000ull);  /* [1,2) */
      double r = 1.4571067811865475 - 0.5 * mu;     /* |r - 1/mu| < 0.09 */
      r = r * QLDPC_FMA(-mu, r, 2.0);
      r = r * QLDPC_FMA(-mu, r, 2.0);
      r = r * QLDPC_FMA(-mu, r, 2.0);
      const double two_mk = qldpc_bits2d((uint64_t)(1023 - ((int)((ub >> 52) & 0x7ff) - 1023)) << 52);
      c = cc * r * two_mk;
    }
  }
  const double s = fm / (2.0 + fm);
  const double z = s * s;
  double R = 2.0 / 25.0;
  R = QLDPC_FMA(R, z, 2.0 / 23.0);
  R = QLDPC_FMA(R, z, 2.0 / 21.0);
  R = QLDPC_FMA(R, z, 2.0 / 19.0);
  R = QLDPC_FMA(R, z, 2.0 / 17.0);
  R = QLDPC_FMA(R, z, 2.0 / 15.0);
  R = QLDPC_FMA(R, z, 2.0 / 13.0);
  R = QLDPC_FMA(R, z, 2.0 / 11.0);
  R = QLDPC_FMA(R, z, 2.0 / 9.0);
  R = QLDPC_FMA(R, z, 2.0 / 7.0);
  R = QLDPC_FMA(R, z, 2.0 / 5.0);
  R = QLDPC_FMA(R, z, 2.0 / 3.0);
  R = R * z;
  const double hfsq = 0.5 * fm * fm;
  const double fk = (double)k;
  return QLDPC_FMA(fk, QLDPC_LN2_HI, (fm - QLDPC_FMA(-s, hfsq + R, hfsq)) + QLDPC_FMA(fk, QLDPC_LN2_LO, c));
}

/* atanh(s) for |s| <= 0.1716: s + s^3 (1/3 + s^2/5 + ... + s^20/21)
   (first omitted term < 2^-60 |s|) */
QLDPC_HD double qldpc_atanh_small(double s) {
  const double z = s * s;
  double q = 1.0 / 21.0;
  q = QLDPC_FMA(q, z, 1.0 / 19.0);
  q = QLDPC_FMA(q, z, 1.0 / 17.0);
  q = QLDPC_FMA(q, z, 1.0 / 15.0);
  q = QLDPC_FMA(q, z, 1.0 / 13.0);
  q = QLDPC_FMA(q, z, 1.0 / 11.0);
  q = QLDPC_FMA(q, z, 1.0 / 9.0);
  q = QLDPC_FMA(q, z, 1.0 / 7.0);
  q = QLDPC_FMA(q, z, 1.0 / 5.0);
  q = QLDPC_FMA(q, z, 1.0 / 3.0);
  return QLDPC_FMA(s * z, q, s);
}

/* atanh(a) = atanh(s) + k ln2 / 2 with s = (N - D 2^k) / (N + D 2^k),
   N = 1 + a, D = 1 - a (ratio of the two = 2^k m, m in [sqrt2/2, sqrt2],
   so |s| <= 3 - 2 sqrt2). N and D are carried as exact two-term sums (their
   rounding errors by Fast2Sum), N - D 2^k is exact (Sterbenz) and the
   corrections enter once: one division in all, no logarithm. Below
   3 - 2 sqrt2, k = 0 and s = a exactly. */
QLDPC_HD double qldpc_atanh(double x) {
  const uint64_t sgn = qldpc_d2bits(x) & 0x8000000000000000ull;
  const double a = qldpc_bits2d(qldpc_d2bits(x) & 0x7fffffffffffffffull);
  if (!(a == a)) return x;
  if (a >= 1.0)
    return qldpc_bits2d(((a == 1.0) ? 0x7ff0000000000000ull : 0x7ff8000000000000ull) | sgn);
  /* branch-free below 1 (lanes diverge): both ranges share one series */
  const double N = 1.0 + a, eN = (1.0 - N) + a;    /* N + eN = 1 + a exactly */
  const double D = 1.0 - a, eD = (1.0 - D) - a;    /* D + eD = 1 - a exactly */
  /* k = round(log2(N / D)): N in [1, 2); D = 2^-e mD, mD in [1, 2) */
  const uint64_t db = qldpc_d2bits(D);
  int k = 1023 - (int)((db >> 52) & 0x7ff);         /* e */
  const double mD = qldpc_bits2d((db & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  if (N > 1.4142135623730951 * mD) k += 1;          /* N / (D 2^k) into [sqrt2/2, sqrt2] */
  const double p2k = qldpc_bits2d((uint64_t)(1023 + k) << 52);
  const double Dk = D * p2k, eDk = eD * p2k;        /* exact */
  const double num = (N - Dk) + (eN - eDk);         /* N - Dk exact (Sterbenz) */
  const double den = (N + Dk) + (eN + eDk);
  const int big = a > 0.17157287525381;             /* 3 - 2 sqrt2 (rounded down) */
  const double sr = big ? QLDPC_DIV(num, den) : a; /* below: k = 0, s = a exactly; den in [1, 4],
                                                     num = 0 or |num| > 2^-110 where big */
  const double fk = big ? (double)k : 0.0;
  const double t = QLDPC_FMA(fk, 0.5 * QLDPC_LN2_HI, qldpc_atanh_small(sr) + fk * (0.5 * QLDPC_LN2_LO));
  return qldpc_bits2d(qldpc_d2bits(t) | sgn);
}

#endif /* QLDPC_LIBM_H */
