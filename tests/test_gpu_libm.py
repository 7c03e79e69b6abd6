"""include/qldpc_libm.h evaluates bit-identically on gfx950 and on the host
(the property that makes BP GPU == oracle == reference exact): NumPy's tanh
and SVML's atanh with their tables read from device memory, and the device
division."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

HIP_SRC = r'''
#include <hip/hip_runtime.h>
#include "qldpc_libm.h"
__constant__ qldpc_libm_tab tab = QLDPC_LIBM_TAB_INIT;
__global__ void k(const double* x, double* t, double* a, double* l, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) {
    t[i] = qldpc_tanh_t(x[i], tab.tanh_c);
    a[i] = qldpc_atanh_t(x[i], tab.atanh_hl, tab.atanh_rcp);
    l[i] = qldpc_tanh_t(2.0 * x[i], tab.tanh_c);
  }
}
__global__ void kd(const double* x, const double* y, double* q, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) q[i] = QLDPC_DIV(x[i], y[i]);
}
extern "C" int run_div(const double* hx, const double* hy, double* hq, long n) {
  double *x, *y, *q;
  if (hipMalloc(&x, n * 8) || hipMalloc(&y, n * 8) || hipMalloc(&q, n * 8)) return 1;
  hipMemcpy(x, hx, n * 8, hipMemcpyHostToDevice);
  hipMemcpy(y, hy, n * 8, hipMemcpyHostToDevice);
  kd<<<(n + 255) / 256, 256>>>(x, y, q, n);
  hipMemcpy(hq, q, n * 8, hipMemcpyDeviceToHost);
  hipFree(x); hipFree(y); hipFree(q);
  return 0;
}
extern "C" int run(const double* hx, double* ht, double* ha, double* hl, long n) {
  double *x, *t, *a, *l;
  if (hipMalloc(&x, n * 8) || hipMalloc(&t, n * 8) || hipMalloc(&a, n * 8) || hipMalloc(&l, n * 8)) return 1;
  hipMemcpy(x, hx, n * 8, hipMemcpyHostToDevice);
  k<<<(n + 255) / 256, 256>>>(x, t, a, l, n);
  hipMemcpy(ht, t, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(ha, a, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(hl, l, n * 8, hipMemcpyDeviceToHost);
  hipFree(x); hipFree(t); hipFree(a); hipFree(l);
  return 0;
}
'''
C_SRC = r'''
#include "qldpc_libm.h"
int run(const double* x, double* t, double* a, double* l, long n) {
  for (long i = 0; i < n; ++i) { t[i] = qldpc_tanh(x[i]); a[i] = qldpc_atanh(x[i]); l[i] = qldpc_tanh(2.0 * x[i]); }
  return 0;
}
'''


def test_libm_bit_identical_gpu_vs_host(tmp_path):
    import qldpcsim_amd._lib  # noqa: F401  (one HIP runtime: torch's)
    inc = os.path.join(ROOT, "include")
    (tmp_path / "g.hip").write_text(HIP_SRC)
    (tmp_path / "c.c").write_text(C_SRC)
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fPIC", "-shared",
                    "-I", inc, "-o", str(tmp_path / "g.so"), str(tmp_path / "g.hip")], check=True)
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-fPIC", "-shared", "-I", inc, "-o",
                    str(tmp_path / "c.so"), str(tmp_path / "c.c")], check=True)
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-40, 40, 200000), rng.uniform(-1, 1, 200000),
                        1 - 10 ** rng.uniform(-16, 0, 100000), -(1 - 10 ** rng.uniform(-16, 0, 50000)),
                        10 ** rng.uniform(-14, 3, 100000), rng.uniform(-0.999, 5, 100000)])
    outs = {}
    for name in ("g", "c"):
        L = ctypes.CDLL(str(tmp_path / f"{name}.so"))
        t, a, l = (np.empty_like(x) for _ in range(3))
        P = lambda v: v.ctypes.data_as(ctypes.c_void_p)
        rc = L.run(P(x), P(t), P(a), P(l), ctypes.c_long(len(x)))
        assert not rc
        outs[name] = (t, a, l)
    for fn, g, c in zip(("tanh", "atanh", "tanh(2x)"), outs["g"], outs["c"]):
        bad = np.flatnonzero(g.view(np.uint64) != c.view(np.uint64))
        assert bad.size == 0, f"{fn}: {bad.size} differ, e.g. x={x[bad[:5]]} gpu={g[bad[:5]]} host={c[bad[:5]]}"


def test_device_division_is_ieee_in_range(tmp_path):
    """QLDPC_DIV on the device (the compiler's division sequence without the
    v_div_scale / v_div_fixup range steps) equals IEEE a / b bit for bit over
    the range its callers guarantee: 2^-500 < |a|, |b| < 2^500 (a != 0: a
    -0 numerator would lose its sign without v_div_fixup, so the BP kernels
    send zero products to the general division), including quotients next to
    1 (P / t_k), mantissas at the edges of [1, 2) and random exponent pairs."""
    import qldpcsim_amd._lib  # noqa: F401
    inc = os.path.join(ROOT, "include")
    (tmp_path / "g.hip").write_text(HIP_SRC)
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fPIC", "-shared",
                    "-I", inc, "-o", str(tmp_path / "g.so"), str(tmp_path / "g.hip")], check=True)
    rng = np.random.default_rng(7)
    N = 400000
    sgn = lambda k: np.where(rng.random(k) < 0.5, -1.0, 1.0)
    a = np.concatenate([sgn(N) * rng.uniform(1, 2, N) * 2.0 ** rng.integers(-499, 499, N),
                        sgn(N) * rng.uniform(0, 1, N),
                        np.nextafter(1.0, 0) ** rng.integers(0, 64, N),
                        1 + np.arange(1000) * 2.0 ** -52])
    b = np.concatenate([sgn(N) * rng.uniform(1, 2, N) * 2.0 ** rng.integers(-499, 499, N),
                        sgn(N) * (1 - rng.uniform(0, 1, N) * 0.999),
                        np.nextafter(1.0, 2) ** rng.integers(0, 64, N),
                        2 - np.arange(1000) * 2.0 ** -52])
    q = np.empty_like(a)
    L = ctypes.CDLL(str(tmp_path / "g.so"))
    P = lambda v: v.ctypes.data_as(ctypes.c_void_p)
    assert L.run_div(P(a), P(b), P(q), ctypes.c_long(len(a))) == 0
    ref = a / b
    bad = np.flatnonzero(q.view(np.uint64) != ref.view(np.uint64))
    assert bad.size == 0, f"{bad.size} differ, e.g. a={a[bad[:3]]} b={b[bad[:3]]} gpu={q[bad[:3]]} ieee={ref[bad[:3]]}"
