"""One simulate_p point (device pipeline), warm-up then timed: for kernel
traces of the end-to-end loop. usage: python tools/sim_one.py CODE DEC SCHED OSD ITERS P [SHOTS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import codes, simulator  # noqa: E402

code, dec, sched, osd, it, p = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), float(sys.argv[6])
shots = int(sys.argv[7]) if len(sys.argv) > 7 else 1 << 20
Hx, Hz = codes.load_code(code)
kw = dict(shots=shots, decType=dec, decIterations=it, decSchedule=sched, OSDorder=osd, verbose=False)
simulator.simulate_p(Hx, Hz, p, rngSeed=2, **kw)
t0 = time.perf_counter()
r = simulator.simulate_p(Hx, Hz, p, rngSeed=1, **kw)
dt = time.perf_counter() - t0
print(json.dumps({"code": code, "p": p, "shots": shots, "shots_per_s": shots / dt, "t0": t0, "sec": dt, **r}))
