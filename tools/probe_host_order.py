"""Host NumPy reliability order throughput (osd_perms) at several thread
counts, on min-sum-like posteriors of LP118_2's width: the status-2 OSD shots
of configs[3] go through it.  usage: python tools/probe_host_order.py [rows]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import decoders  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 23000
rng = np.random.default_rng(1)
post = np.round(rng.normal(0, 8, (k, 1054)), 1) + 2.0      # quantised, tie-rich like MS posteriors
aff = len(os.sched_getaffinity(0))
out = {"rows": k, "cpu_count": os.cpu_count(), "affinity": aff}
for nt in (1, 4, 8, 16, 32):
    decoders.osd_perms(post[:512], nthreads=nt)
    t0 = time.perf_counter()
    decoders.osd_perms(post, nthreads=nt)
    out[f"sec_{nt}"] = round(time.perf_counter() - t0, 4)
t0 = time.perf_counter()
for r in range(200):
    np.argsort(post[r])
out["argsort_us_per_row"] = round((time.perf_counter() - t0) / 200 * 1e6, 2)
print(json.dumps(out), flush=True)
