"""cProfile of the host side of the device OSD path (apply_osd_device_many)
for one decode batch of a config: where the per-batch OSD time goes when few
shots need OSD. usage: python tools/prof_osd_path.py CODE DEC SCHED ITERS P [B]"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import codes, decoders, schedule, simulator  # noqa: E402

code, dec, sched, it, p = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), float(sys.argv[5])
B = int(sys.argv[6]) if len(sys.argv) > 6 else 262144
Hx, Hz = codes.load_code(code)
lx, lz = schedule.select_layers(Hx, Hz, sched)
lpX, lrX = schedule.pack_layers(lx, Hz.shape[0])
lpZ, lrZ = schedule.pack_layers(lz, Hx.shape[0])
ch = simulator.DeviceChannel(Hx, Hz, torch.device("cuda", 0), 1)


def batch():
    sy_z, sy_x, _, _ = ch.sample(p, B)
    rX = decoders.decode_batch(Hz, sy_z, p / 3, it, algo=dec, want_post=True, layer_ptr=lpX, layer_rows=lrX)
    rZ = decoders.decode_batch(Hx, sy_x, p / 3, it, algo=dec, want_post=True, layer_ptr=lpZ, layer_rows=lrZ)
    torch.cuda.synchronize()
    return [(Hz, sy_z, rX), (Hx, sy_x, rZ)]


for _ in range(2):                                    # warm-up (pinned buffers, thread pools)
    decoders.apply_osd_device_many(batch(), 0)
torch.cuda.synchronize()
items = batch()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
decoders.apply_osd_device_many(items, 0)
torch.cuda.synchronize()
pr.disable()
print(f"osd wall {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
