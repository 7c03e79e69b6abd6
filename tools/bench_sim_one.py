"""One simulate_p point end to end (warm-up run, then a timed run), for
kernel traces of the simulator pipeline.
usage: python tools/bench_sim_one.py CODE DEC SCHED OSD ITERS P SHOTS"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import codes, simulator  # noqa: E402

code, dec, sched, osd, it, p, shots = sys.argv[1:8]
osd, it, p, shots = int(osd), int(it), float(p), int(shots)
Hx, Hz = codes.load_code(code)
kw = dict(shots=shots, decType=dec, decIterations=it, decSchedule=sched, OSDorder=osd, verbose=False)
simulator.simulate_p(Hx, Hz, p, rngSeed=2, **kw)
t0 = time.perf_counter()
r = simulator.simulate_p(Hx, Hz, p, rngSeed=1, **kw)
dt = time.perf_counter() - t0
print(json.dumps({"code": code, "dec": dec, "sched": sched, "osd": osd, "p": p, "shots": shots,
                  "t_start": t0, "sec": dt, "shots_per_s": shots / dt, **r}), flush=True)
