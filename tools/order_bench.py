"""The device reliability order alone (qldpc_osd_order_device) on realistic
inputs: the non-converged shots of one simulate_p-style batch (device
sampler, decode with posteriors), timed over repeats with HIP events; the
order's hash and the host restatement's agreement say whether a build
variant still computes NumPy's order.
usage: python tools/order_bench.py [CODE DEC SCHED ITERS P B REPS]"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import _lib, codes, decoders, schedule, simulator  # noqa: E402

a = sys.argv[1:] + [None] * 7
code, dec, sched = a[0] or "LP118_2", a[1] or "MS", a[2] or "L"
it, p, B, reps = int(a[3] or 50), float(a[4] or 0.1), int(a[5] or 131072), int(a[6] or 5)
Hx, Hz = codes.load_code(code)
lx, _ = schedule.select_layers(Hx, Hz, sched)
lp, lr = schedule.pack_layers(lx, Hz.shape[0])
dev = torch.device("cuda", 0)
ch = simulator.DeviceChannel(Hx, Hz, dev, 1)
sy_z = ch.sample(p, B)[0]
r = decoders.decode_batch(Hz, sy_z, p / 3, it, algo=dec, want_post=True, layer_ptr=lp, layer_rows=lr)
bad = ((r.flags & _lib.FLAG_CONVERGED) == 0).nonzero().flatten()
k, n = int(bad.numel()), Hz.shape[1]
post = r.post.index_select(0, bad).contiguous()
h = _lib.code_for(Hz, 0)
perm = torch.empty((k, n), dtype=torch.int32, device=dev)
tie = torch.empty(k, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream(dev)
ms = []
for rep in range(reps + 1):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    _lib.check(_lib.lib.qldpc_osd_order_device(h.handle, k, post.data_ptr(), perm.data_ptr(), tie.data_ptr(),
                                               st.cuda_stream))
    e1.record(st)
    torch.cuda.synchronize()
    if rep:
        ms.append(e0.elapsed_time(e1))
P = perm.cpu().numpy()
sample = np.arange(0, k, max(1, k // 2000))
hp = np.empty((sample.size, n), np.int32)
hs = np.empty(sample.size, np.int32)
Ps = np.ascontiguousarray(post.cpu().numpy()[sample])
_lib.check(_lib.lib.qldpc_osd_order_host(_lib.ptr(Ps), sample.size, n, _lib.ptr(hp), _lib.ptr(hs), 0))
print(json.dumps({"code": code, "p": p, "B": B, "osd_shots": k, "ms": sorted(ms), "ms_med": float(np.median(ms)),
                  "host_fallback": int((tie.cpu().numpy() < 0).sum()),
                  "equal_host_on_sample": bool(np.array_equal(P[sample], hp)),
                  "perm_sha": hashlib.sha256(P.tobytes()).hexdigest()[:16],
                  "lib": os.path.basename(_lib.LIB_PATH)}), flush=True)
