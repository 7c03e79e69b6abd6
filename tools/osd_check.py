"""GPU OSD (qldpc_osd_device, host orders) against the host C++ OSD on random
consistent / inconsistent syndromes with tie-heavy posteriors, over many seeds
(the shape of tests/test_gpu_osd.py::test_gpu_osd_matches_host_osd).
usage: python tools/osd_check.py CODE ORDER SEEDS [K]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import _lib, codes, decoders  # noqa: E402

code, order, seeds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
k = int(sys.argv[4]) if len(sys.argv) > 4 else 48
Hx, Hz = codes.load_code(code)
bad = []
for seed in range(seeds):
    rng = np.random.default_rng(seed)
    for hi, H in enumerate((Hx, Hz)):
        syn = rng.integers(0, 2, (k, H.shape[0])).astype(np.uint8)
        err = (rng.random((k // 2, H.shape[1])) < 0.05).astype(np.int64)
        syn[: k // 2] = (err @ H.T.astype(np.int64)) % 2
        post = rng.normal(0, 3, (k, H.shape[1]))
        post[:, ::5] = 1.75
        e0 = (post < 0).astype(np.uint8)
        hc = _lib.code_for(H, 0)
        perms = np.ascontiguousarray(decoders.osd_perms(post), np.int32)
        pd = torch.as_tensor(perms, device="cuda")
        s = torch.as_tensor(syn, device="cuda")
        ed = torch.as_tensor(e0, device="cuda")
        st = torch.empty(k, dtype=torch.int32, device="cuda")
        _lib.check(_lib.lib.qldpc_osd_device(hc.handle, k, s.data_ptr(), pd.data_ptr(), order, ed.data_ptr(),
                                             st.data_ptr(), None))
        got = ed.cpu().numpy()
        want = e0.copy()
        _lib.check(_lib.lib.qldpc_osd_decode_batch(hc.handle, k, _lib.ptr(syn), _lib.ptr(perms), order,
                                                   _lib.ptr(want), 1))
        rows = np.flatnonzero((got != want).any(axis=1))
        if rows.size:
            sat_g = ((got[rows].astype(np.int64) @ H.T) % 2 == syn[rows]).all(axis=1)
            sat_w = ((want[rows].astype(np.int64) @ H.T) % 2 == syn[rows]).all(axis=1)
            bad.append({"seed": seed, "half": hi, "rows": rows.tolist()[:6], "consistent": (rows < k // 2).tolist()[:6],
                        "status": st.cpu().numpy()[rows].tolist()[:6], "gpu_sat": sat_g.tolist()[:6],
                        "host_sat": sat_w.tolist()[:6]})
print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "options": os.environ.get("QLDPC_OPTIONS", ""), "code": code, "order": order, "seeds": seeds,
                  "bad": bad[:3], "n_bad": len(bad)}))
