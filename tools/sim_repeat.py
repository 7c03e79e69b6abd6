"""Repeat timed simulate_p calls for one config at several p (warm-up effects vs steady state).
usage: python tools/sim_repeat.py CODE DEC SCHED OSD ITERS SHOTS P [P ...]   (env SIM_BATCH = batch_size)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import codes, simulator  # noqa: E402

code, dec, sched, osd, it, shots = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
Hx, Hz = codes.load_code(code)
for p in map(float, sys.argv[7:]):
    ts = []
    for rep in range(3):
        t0 = time.perf_counter()
        simulator.simulate_p(Hx, Hz, p, shots=shots, decType=dec, decIterations=it, decSchedule=sched,
                             OSDorder=osd, rngSeed=1 + rep, verbose=False,
                             batch_size=int(os.environ["SIM_BATCH"]) if "SIM_BATCH" in os.environ else None)
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"code": code, "dec": dec, "sched": sched, "osd": osd, "p": p, "shots": shots,
                      "sec": ts, "shots_per_s": [shots / t for t in ts]}), flush=True)
