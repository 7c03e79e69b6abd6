"""Interleaved A/B of simulator.TAIL_DIV (smallest tapered tail batch) on one
simulate_p point. usage: python tools/ab_tail.py CODE DEC SCHED OSD ITERS P SHOTS DIV [DIV ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import codes, simulator  # noqa: E402

code, dec, sched, osd, it, p, shots = sys.argv[1:8]
divs = [int(x) for x in sys.argv[8:]]
osd, it, p, shots = int(osd), int(it), float(p), int(shots)
Hx, Hz = codes.load_code(code)
kw = dict(shots=shots, decType=dec, decIterations=it, decSchedule=sched, OSDorder=osd, verbose=False)
simulator.simulate_p(Hx, Hz, p, rngSeed=2, **kw)
for rnd in range(2):
    for dv in (divs if rnd == 0 else divs[::-1]):
        simulator.TAIL_DIV = dv
        t0 = time.perf_counter()
        r = simulator.simulate_p(Hx, Hz, p, rngSeed=1, **kw)
        dt = time.perf_counter() - t0
        print(json.dumps({"tail_div": dv, "round": rnd, "shots_per_s": shots / dt, "qBLER": r.get("qBLER")}), flush=True)
