"""Throughput of the device-memory OSD kernel (osd_hbm_kernel): a code past the
register / LDS kernels (random row-weight-8 H, m x n), and LP118_2 with the
kernel forced (option osd_hbm) beside the default block kernel. Prints one
JSON line per case: shots, ms per call (HIP events), shots/s."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from qldpcsim_amd import _lib, codes, decoders  # noqa: E402


def run(H, k, opt_hbm, label, reps=3):
    m, n = H.shape
    rng = np.random.default_rng(1)
    err = (rng.random((k, n)) < 0.03).astype(np.int64)
    syn = ((err @ H.T.astype(np.int64)) % 2).astype(np.uint8)
    post = rng.normal(0, 3, (k, n))
    code = _lib.code_for(H, 0)
    d = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dt), device="cuda")  # noqa: E731
    s_d, perm = d(syn, np.uint8), d(decoders.osd_perms(post), np.int32)
    st = torch.empty(k, dtype=torch.int32, device="cuda")
    best = None
    with _lib.options(osd_hbm=opt_hbm):
        for _ in range(reps + 1):
            e_d = d((post < 0).astype(np.uint8), np.uint8)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            _lib.check(_lib.lib.qldpc_osd_device(code.handle, k, s_d.data_ptr(), perm.data_ptr(), 0,
                                                 e_d.data_ptr(), st.data_ptr(), None))
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b)
            best = ms if best is None else min(best, ms)
    print(json.dumps({"case": label, "m": m, "n": n, "shots": k, "ms": round(best, 3),
                      "shots_per_s": round(k / best * 1e3, 1), "osd_hbm": opt_hbm,
                      "status0": int((st == 0).sum())}), flush=True)


if __name__ == "__main__":
    t0 = time.time()
    Hx, _ = codes.load_code("LP118_2")
    run(Hx, 8192, 0, "LP118_2 block kernel")
    run(Hx, 8192, 1, "LP118_2 osd_hbm_kernel (forced)")
    for m, n in ((1100, 2300), (3000, 6000)):
        rng = np.random.default_rng(m + n)
        H = np.zeros((m, n), np.uint8)
        for r in range(m):
            H[r, rng.choice(n, 8, replace=False)] = 1
        run(H, 2048 if m < 2000 else 256, 0, f"random {m} x {n} (osd_hbm_kernel)")
    print(f"# {time.time() - t0:.1f} s", file=sys.stderr)
