"""Phase timing of one simulate_p batch on the device path (sample, decode X/Z,
OSD host order + GPU elimination, counters) for a config.
usage: python tools/prof_sim.py CODE DEC SCHED OSD ITERS P [B]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import _lib, codes, decoders, schedule, simulator  # noqa: E402

code, dec, sched, osd, it, p = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), float(sys.argv[6])
B = int(sys.argv[7]) if len(sys.argv) > 7 else 65536
Hx, Hz = codes.load_code(code)
lx, lz = schedule.select_layers(Hx, Hz, sched)
lpX, lrX = schedule.pack_layers(lx, Hz.shape[0])
lpZ, lrZ = schedule.pack_layers(lz, Hx.shape[0])
dev = torch.device("cuda", 0)
ch = simulator.DeviceChannel(Hx, Hz, dev, 1)
T = {}


def tick(name, t0):
    torch.cuda.synchronize()
    T[name] = T.get(name, 0.0) + time.perf_counter() - t0
    return time.perf_counter()


for rep in range(3):
    if rep == 1:
        T.clear()
    t = time.perf_counter()
    sy_z, sy_x, errX, errZ = ch.sample(p, B)
    t = tick("sample", t)
    rX = decoders.decode_batch(Hz, sy_z, p / 3, it, algo=dec, want_post=osd >= 0, layer_ptr=lpX, layer_rows=lrX)
    rZ = decoders.decode_batch(Hx, sy_x, p / 3, it, algo=dec, want_post=osd >= 0, layer_ptr=lpZ, layer_rows=lrZ)
    t = tick("decode", t)
    if osd >= 0:
        for r in (rX, rZ):
            T["osd_shots"] = T.get("osd_shots", 0) + int(((r.flags & _lib.FLAG_CONVERGED) == 0).sum())
        t = tick("osd_count", t)
        decoders.apply_osd_device_many([(Hz, sy_z, rX), (Hx, sy_x, rZ)], osd)
        t = tick("osd", t)
        T["osd_host_order_shots"] = T.get("osd_host_order_shots", 0) + rX.osd_host_order + rZ.osd_host_order
    c = ch.count(sy_z, sy_x, errX, errZ, rX.ehat, rZ.ehat, rX.iters, rZ.iters)
    t = tick("count", t)
T = {k: (v / 2 if k != "osd_shots" else v / 2) for k, v in T.items()}
print(json.dumps({"code": code, "dec": dec, "sched": sched, "osd": osd, "p": p, "B": B, "sec_per_batch": T}))
