"""Generate include/qldpc_numpy_tables.h: the constant tables of the float64
tanh / arctanh / log that NumPy evaluates on the reference's host, so that
include/qldpc_libm.h reproduces them bit for bit (GPU and oracle alike).

Which code NumPy runs (NumPy 2.2.6, x86-64 with AVX512_SKX — the host the
golden vectors were captured on; `numpy._core._multiarray_umath.__cpu_dispatch__`):
  * np.tanh (float64)    DOUBLE_tanh_AVX512_SKX: NumPy's own simd_tanh_f64
    (numpy/_core/src/umath/loops_hyperbolic.dispatch.c.src), a 16-interval
    lookup of degree-16 polynomials, table `lut16x18` (18 rows x 16: the
    interval origin b, then c0..c16).
  * np.arctanh (float64) DOUBLE_arctanh_AVX512_SKX -> __svml_atanh8_ha
    (Intel SVML as vendored by NumPy, numpy/SVML, BSD-3), data block
    __svml_datanh_ha_data_internal_avx512.
  * np.log (float64)     DOUBLE_log_AVX512_SKX -> __svml_log8_ha, data block
    __svml_dlog_ha_data_internal_avx512 (the prior L = np.log((1-p)/p),
    decoders.py:147 / :232).
  * np.exp (float64)     DOUBLE_exp_AVX512_SKX -> __svml_exp8_ha for
    non-overlapping operands (the OSD reliability key, decoders.py:323), data
    block __svml_dexp_ha_data_internal_avx512: 2^(j/16) as hi (+0x00) and lo
    (+0x80) tables, log2(e), the round-toward-zero shifter, ln2 hi / lo, a
    degree-6 series and the rare-path threshold.
The SVML kernels start from vrcp14pd rounded to a 4-bit mantissa (atanh:
add-half-and-truncate; log: vrndscalepd, round-half-even). vrcp14pd depends
on the top 18 mantissa bits of its input only; the rounded value is a
monotone step function of the mantissa whose 16 step positions are found
here by bisection on this host's vrcp14pd and written as thresholds.

Build container only (reads the installed NumPy's shared object and runs an
AVX-512 probe); the generated header is committed.

Usage:  python tools/gen_numpy_libm_tables.py
"""
import os
import struct
import subprocess
import sys
import tempfile

import numpy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "include", "qldpc_numpy_tables.h")
LLVM = "/opt/rocm/lib/llvm/bin"

PROBE = r"""
#include <immintrin.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t b(double d){uint64_t u; memcpy(&u,&d,8); return u;}
static double d(uint64_t u){double x; memcpy(&x,&u,8); return x;}
static uint64_t R(uint64_t m, int mode){
  __m512d r=_mm512_rcp14_pd(_mm512_set1_pd(d(m))); double o[8];
  if (mode) r=_mm512_roundscale_pd(r,0x58);          /* svml log: vrndscalepd $0x58 */
  _mm512_storeu_pd(o,r);
  return mode ? b(o[0]) : ((b(o[0])+0x0000800000000000ull)&0xffff000000000000ull);  /* svml atanh */
}
int main(int argc, char** argv){
  int mode = argv[1][0]=='1';
  uint64_t lo=0x3ff0000000000000ull, hi=0x3fffffffffffffffull, cur=lo, Rc=R(lo,mode);
  for(int t=0;t<16;t++){
    uint64_t a=cur, z=cur;
    while(R(z,mode)==Rc){ a=z; z+=(1ull<<34); if(z>hi){z=hi;break;} }
    while(z-a>1){ uint64_t mid=a+(z-a)/2; if(R(mid,mode)==Rc) a=mid; else z=mid; }
    uint64_t Rn=R(z,mode);
    if (Rn != Rc - 0x0001000000000000ull) { fprintf(stderr,"non-unit step\n"); return 1; }
    uint64_t s=99;                                   /* monotone step check around it */
    for(int k=0;k<400000;k++){ s^=s<<13; s^=s>>7; s^=s<<17;
      int64_t off=(int64_t)(s%(1ull<<36))-(1ll<<35); uint64_t x=z+off; if(x<lo||x>hi) continue;
      uint64_t r=R(x,mode); if((x<z && r!=Rc)||(x>=z && r!=Rn)){ fprintf(stderr,"not a step\n"); return 1; } }
    printf("%llu\n",(unsigned long long)(z&0xfffffffffffffull));
    cur=z; Rc=Rn;
  }
  return 0;
}
"""


def so_path():
    d = os.path.join(os.path.dirname(numpy.__file__), "_core")
    return [os.path.join(d, f) for f in os.listdir(d) if f.startswith("_multiarray_umath") and f.endswith(".so")][0]


def symbols(so):
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-t", so], capture_output=True, text=True, check=True).stdout
    syms = {}
    for line in out.splitlines():
        p = line.split()
        if len(p) >= 5:
            syms[p[-1]] = int(p[0], 16)
    return syms


def reader(so):
    out = subprocess.run([f"{LLVM}/llvm-readelf", "-lW", so], capture_output=True, text=True, check=True).stdout
    segs = []
    for line in out.splitlines():
        p = line.split()
        if p and p[0] == "LOAD":
            segs.append((int(p[2], 16), int(p[1], 16), int(p[4], 16)))
    data = open(so, "rb").read()

    def rd(va, n):
        for v, o, fs in segs:
            if v <= va < v + fs:
                return list(struct.unpack(f"<{n}d", data[o + va - v:o + va - v + 8 * n]))
        raise KeyError(hex(va))
    return rd


def tanh_table(syms, rd):
    # lut16x18 sits right after NumPy's float32 lut32x8 in .rodata; locate it by
    # its first rows (b_0 = 0, b_1 = 0.21875; c0_0 = 0; c1_0 = 1) instead of
    # trusting a fixed offset
    base = syms["lut32x8.1"]
    for off in range(0, 0x8000, 0x40):
        row = rd(base + off, 16)
        if row[0] == 0.0 and row[1] == 0.21875 and row[2] == 0.3125:
            t = rd(base + off, 18 * 16)
            if t[16] == 0.0 and t[32] == 1.0:
                return [t[r * 16:(r + 1) * 16] for r in range(18)]
    raise RuntimeError("tanh table not found")


def probe_thresholds(mode):
    with tempfile.TemporaryDirectory() as td:
        src, exe = os.path.join(td, "p.c"), os.path.join(td, "p")
        open(src, "w").write(PROBE)
        subprocess.run(["gcc", "-O2", "-mavx512f", src, "-o", exe], check=True)
        out = subprocess.run([exe, str(mode)], capture_output=True, text=True, check=True).stdout
    t = [int(x) for x in out.split()]
    assert len(t) == 16 and all((x & ((1 << 34) - 1)) == 0 for x in t), t
    return t


def hexd(x):
    return float(x).hex()


def main():
    so = so_path()
    syms = symbols(so)
    rd = reader(so)
    tanh = tanh_table(syms, rd)
    at = rd(syms["__svml_datanh_ha_data_internal_avx512"], 0x500 // 8)
    lg = rd(syms["__svml_dlog_ha_data_internal_avx512"], 0x400 // 8)
    ex = rd(syms["__svml_dexp_ha_data_internal_avx512"], 0x500 // 8)
    c = lambda blk, off: blk[off // 8]  # noqa: E731  (broadcast constants: lane 0)
    t_at = probe_thresholds(0)
    t_lg = probe_thresholds(1)
    # atanh reciprocal: per 6-bit bucket of the 18-bit mantissa prefix p, the
    # count of thresholds below the bucket and the one inside it (spacing of
    # the thresholds > the bucket width, checked)
    pre = [t >> 34 for t in t_at]
    assert all(b - a > (1 << 12) for a, b in zip(pre, pre[1:]))
    buckets = []
    for bkt in range(64):
        lo, hi = bkt << 12, (bkt + 1) << 12
        below = sum(1 for x in pre if x < lo)
        inside = [x for x in pre if lo <= x < hi]
        thr = inside[0] if inside else (1 << 18)
        buckets.append(below | (thr << 8))
    L = []
    L.append("/* Generated by tools/gen_numpy_libm_tables.py from NumPy %s (%s): DO NOT EDIT." % (numpy.__version__, os.path.basename(so)))
    L.append(" * tanh:   NumPy simd_tanh_f64 lut16x18 (loops_hyperbolic.dispatch.c.src), stored as [9][16][2] row pairs.")
    L.append(" * atanh:  __svml_atanh8_ha data (__svml_datanh_ha_data_internal_avx512).")
    L.append(" * log:    __svml_log8_ha data (__svml_dlog_ha_data_internal_avx512).")
    L.append(" * exp:    __svml_exp8_ha data (__svml_dexp_ha_data_internal_avx512).")
    L.append(" * rcp:    mantissa thresholds of the rounded vrcp14pd step functions (probed on the capture host). */")
    L.append("#ifndef QLDPC_NUMPY_TABLES_H\n#define QLDPC_NUMPY_TABLES_H\n")
    L.append("/* [9][16][2]: row pair (2q, 2q+1) of interval i, rows = b, c0 .. c16 of")
    L.append("   tanh(|x|) = sum c_k (|x| - b)^k. Pair-major: one 16-byte read fetches two")
    L.append("   rows of a lane's interval, and 16 lanes' reads of a pair fall in one 256-byte")
    L.append("   block (distinct LDS banks whatever the intervals). */")
    L.append("#define QLDPC_TANH_LUT_INIT { \\")
    for q in range(9):
        L.append("  " + ", ".join(f"{hexd(tanh[2 * q][i])}, {hexd(tanh[2 * q + 1][i])}" for i in range(16)) + ", \\")
    L.append("}")
    L.append("/* [16][2]: log(1 + i/16) as hi + lo (atanh) */")
    L.append("#define QLDPC_ATANH_HL_INIT { \\")
    for i in range(16):
        L.append("  %s, %s, \\" % (hexd(at[i]), hexd(at[16 + i])))
    L.append("}")
    for k, off in enumerate(range(0x200, 0x440, 0x40)):
        L.append("#define QLDPC_ATANH_C%d %s" % (k, hexd(c(at, off))))
    L.append("#define QLDPC_ATANH_LN2HI %s" % hexd(c(at, 0x440)))
    L.append("#define QLDPC_ATANH_LN2LO %s" % hexd(c(at, 0x480)))
    L.append("/* [64]: (#thresholds below bucket) | (threshold inside bucket, 18-bit prefix, or 2^18) << 8 */")
    L.append("#define QLDPC_ATANH_RCP_INIT { \\")
    for i in range(0, 64, 8):
        L.append("  " + ", ".join("0x%08xu" % x for x in buckets[i:i + 8]) + ", \\")
    L.append("}")
    L.append("#define QLDPC_LOG_RCP_T_INIT { " + ", ".join("0x%013xull" % x for x in t_lg) + " }")
    L.append("/* [16][2]: table A (hi, with the -ln2 fold for R < 3/4), table B (lo) */")
    L.append("#define QLDPC_LOG_AB_INIT { \\")
    for i in range(16):
        L.append("  %s, %s, \\" % (hexd(lg[i]), hexd(lg[16 + i])))
    L.append("}")
    for off in range(0x100, 0x400, 0x40):
        L.append("#define QLDPC_LOG_C%03x %s" % (off, hexd(c(lg, off))))
    L.append("/* [16][2]: 2^(j/16) as hi, lo (exp) */")
    L.append("#define QLDPC_EXP_HL_INIT { \\")
    for i in range(16):
        L.append("  %s, %s, \\" % (hexd(ex[i]), hexd(ex[16 + i])))
    L.append("}")
    bits = lambda off: struct.unpack("<Q", struct.pack("<d", c(ex, off)))[0]  # noqa: E731
    L.append("#define QLDPC_EXP_LOG2E %s" % hexd(c(ex, 0x100)))
    L.append("#define QLDPC_EXP_SHIFTER_BITS 0x%016xull" % bits(0x140))
    L.append("#define QLDPC_EXP_LN2HI %s" % hexd(c(ex, 0x180)))
    L.append("#define QLDPC_EXP_LN2LO %s" % hexd(c(ex, 0x1c0)))
    L.append("#define QLDPC_EXP_RMASK_BITS 0x%016xull" % bits(0x200))
    for k, off in enumerate(range(0x240, 0x3c0, 0x40)):
        L.append("#define QLDPC_EXP_C%d %s" % (5 - k, hexd(c(ex, off))))
    L.append("#define QLDPC_EXP_RARE %s" % hexd(c(ex, 0x400)))
    L.append("\n#endif")
    open(OUT, "w").write("\n".join(L) + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
