"""include/qldpc_libm.h evaluates bit-identically on gfx950 and on the host
(the property that makes BP GPU-vs-oracle parity exact)."""
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
__global__ void k(const double* x, double* t, double* a, double* l, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) { t[i] = qldpc_tanh(x[i]); a[i] = qldpc_atanh(x[i]); l[i] = qldpc_log1p(x[i]); }
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
  for (long i = 0; i < n; ++i) { t[i] = qldpc_tanh(x[i]); a[i] = qldpc_atanh(x[i]); l[i] = qldpc_log1p(x[i]); }
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
    for fn, g, c in zip(("tanh", "atanh", "log1p"), outs["g"], outs["c"]):
        bad = np.flatnonzero(g.view(np.uint64) != c.view(np.uint64))
        assert bad.size == 0, f"{fn}: {bad.size} differ, e.g. x={x[bad[:5]]} gpu={g[bad[:5]]} host={c[bad[:5]]}"
