"""Where the device reliability order's near-ties sit, by OSD outcome: for
the non-converged shots of one configs[3]-style batch, the first near-tie
position (tiepos) of each shot against its status (0 = certified, 2 = left to
NumPy's order), and how many of its posteriors saturate the reliability key
(|LLR| > 36.7: 1 - 1/(1 + e^|LLR|) rounds to 1.0, so those keys tie exactly).
usage: python tools/osd_tie_stats.py CODE DEC SCHED ITERS P [B]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import _lib, codes, decoders, schedule, simulator  # noqa: E402

code, dec, sched, it, p = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), float(sys.argv[5])
B = int(sys.argv[6]) if len(sys.argv) > 6 else 65536
Hx, Hz = codes.load_code(code)
lx, _ = schedule.select_layers(Hx, Hz, sched)
lp, lr = schedule.pack_layers(lx, Hz.shape[0])
dev = torch.device("cuda", 0)
ch = simulator.DeviceChannel(Hx, Hz, dev, 1)
sy_z = ch.sample(p, B)[0]
r = decoders.decode_batch(Hz, sy_z, p / 3, it, algo=dec, want_post=True, layer_ptr=lp, layer_rows=lr)
bad = ((r.flags & _lib.FLAG_CONVERGED) == 0).nonzero().flatten()
k = int(bad.numel())
n = Hz.shape[1]
post = r.post.index_select(0, bad).contiguous()
syn = sy_z.index_select(0, bad).contiguous()
e = r.ehat.index_select(0, bad).contiguous()
h = _lib.code_for(Hz, 0)
perm = torch.empty((k, n), dtype=torch.int32, device=dev)
tie = torch.empty(k, dtype=torch.int32, device=dev)
status = torch.empty(k, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
_lib.check(_lib.lib.qldpc_osd_device_ordered(h.handle, k, syn.data_ptr(), post.data_ptr(), 0, e.data_ptr(),
                                             status.data_ptr(), perm.data_ptr(), tie.data_ptr(), st))
torch.cuda.synchronize()
s = status.cpu().numpy()
tp = tie.cpu().numpy()
sat = (post.abs() > 36.7).sum(1).cpu().numpy()
out = {"code": code, "p": p, "osd_shots": k, "status_hist": np.bincount(s, minlength=4).tolist()}
q = [0, 10, 25, 50, 75, 90, 100]
for v in (0, 2):
    m = s == v
    if m.any():
        out[f"status{v}"] = {"tiepos_pct": np.percentile(tp[m], q).astype(int).tolist(),
                             "saturated_pct": np.percentile(sat[m], q).astype(int).tolist()}
for T in (100, 200, 300, 400, 500, 600, 800):
    pred = tp < T
    out[f"tiepos<{T}"] = {"status2_caught": float((pred & (s == 2)).sum() / max(1, (s == 2).sum())),
                          "status0_flagged": float((pred & (s == 0)).sum() / max(1, (s == 0).sum()))}
for S in (400, 500, 520, 550, 600):
    pred = sat >= S
    out[f"saturated>={S}"] = {"status2_caught": float((pred & (s == 2)).sum() / max(1, (s == 2).sum())),
                              "status0_flagged": float((pred & (s == 0)).sum() / max(1, (s == 0).sum()))}
print(json.dumps(out))
