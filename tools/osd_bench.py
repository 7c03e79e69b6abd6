"""Device OSD alone on realistic inputs: the non-converged shots of one
simulate_p-style batch (device sampler, MS/BP decode with posteriors), then
qldpc_osd_device_ordered (device order + elimination) timed over repeats,
with the status histogram (2 = left to NumPy's order, 1 = IndexError case).
usage: python tools/osd_bench.py CODE DEC SCHED ITERS P [B] [ORDER] [REPS] [--worklog PATH]
--worklog: every OSD call's kernels (family names, resolved against the
rocprofv3 trace by tools/roofline_profile.py) with its shot count, the unit
of a counter profile (tools/gpu_run.sh roof-osd)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import _lib, codes, decoders, schedule, simulator  # noqa: E402

worklog = None
if "--worklog" in sys.argv:
    i = sys.argv.index("--worklog")
    worklog = sys.argv[i + 1]
    del sys.argv[i:i + 2]
code, dec, sched, it, p = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), float(sys.argv[5])
B = int(sys.argv[6]) if len(sys.argv) > 6 else 65536
order = int(sys.argv[7]) if len(sys.argv) > 7 else 0
reps = int(sys.argv[8]) if len(sys.argv) > 8 else 5
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
e0 = r.ehat.index_select(0, bad).contiguous()
h = _lib.code_for(Hz, 0)
perm = torch.empty((k, n), dtype=torch.int32, device=dev)
tie = torch.empty(k, dtype=torch.int32, device=dev)
status = torch.empty(k, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
times = []
for rep in range(reps + 1):
    e = e0.clone()
    torch.cuda.synchronize()
    t = time.perf_counter()
    _lib.check(_lib.lib.qldpc_osd_device_ordered(h.handle, k, syn.data_ptr(), post.data_ptr(), order, e.data_ptr(),
                                                 status.data_ptr(), perm.data_ptr(), tie.data_ptr(), st))
    torch.cuda.synchronize()
    if rep:
        times.append(time.perf_counter() - t)
if worklog:
    # one osd_order_kernel, one osd_block_kernel and one osd_kernel (the
    # column kernel's redo pass) per call (capi.cpp osd_device_impl)
    with open(worklog, "w") as f:
        json.dump({"unit": "osd_shot",
                   "launches": [{"kernel": kn, "half_shots": k, "iters": k}
                                for _ in range(reps + 1)
                                for kn in ("osd_order_kernel", "osd_block_kernel", "osd_kernel")
                                if kn != "osd_block_kernel" or not _lib.get_option("osd_column")]}, f)
hist = np.bincount(status.cpu().numpy(), minlength=4).tolist()
import hashlib  # noqa: E402
ehat_sha = hashlib.sha256(e.cpu().numpy().tobytes() + status.cpu().numpy().tobytes()).hexdigest()[:16]
t = float(np.median(times))
print(json.dumps({"code": code, "dec": dec, "sched": sched, "p": p, "B": B, "order": order,
                  "osd_shots": k, "sec": t, "osd_shots_per_s": k / t, "status_hist": hist, "ehat_sha": ehat_sha,
                  "lib": os.path.basename(_lib.LIB_PATH),
                  "kernel": "column" if _lib.get_option("osd_column") else "block"}))
