"""Locate GPU-vs-oracle BP divergences: for mismatching shots, the first
iteration count at which posteriors differ, and the differing values."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from oracle import oracle  # noqa: E402
from qldpcsim_amd import codes, decoders, schedule  # noqa: E402
from test_gpu_parity import _channel  # noqa: E402

Hx, Hz = codes.load_code("LP118_0")
sz, sx = _channel(Hx, Hz, 0.05, 512, 7)
for H, syn, name in ((Hz, sz, "X"), (Hx, sx, "Z")):
    r = decoders.decode_batch(H, syn, 0.05 / 3, 100, algo="BP", want_post=True)
    e, it, post, fl = oracle.decode_batch("BP", H, syn, 0.05 / 3, 100)
    bad = np.flatnonzero((r.iters != it) | np.any(r.post.view(np.uint64) != post.view(np.uint64), axis=1))
    print(name, "mismatching shots", bad.tolist(), "gpu iters", r.iters[bad].tolist(), "oracle", it[bad].tolist(),
          "flags", r.flags[bad].tolist(), fl[bad].tolist())
    for b in bad[:2]:
        for mi in range(1, 101):
            rg = decoders.decode_batch(H, syn[b:b + 1], 0.05 / 3, mi, algo="BP", want_post=True)
            eo, io, po, fo = oracle.decode_batch("BP", H, syn[b:b + 1], 0.05 / 3, mi)
            d = np.flatnonzero(rg.post[0].view(np.uint64) != po[0].view(np.uint64))
            if d.size:
                print(f"  shot {b}: first differs at max_iter={mi}: {d.size} vars, e.g. var {d[:4].tolist()} "
                      f"gpu {rg.post[0][d[:4]].tolist()} oracle {po[0][d[:4]].tolist()}")
                break
