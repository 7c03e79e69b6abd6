"""End-to-end simulate_p throughput (device sampler + decode + OSD + counters)
for BASELINE.json configs[3] / configs[4] shapes on one GPU.

usage: python tools/bench_sim.py [shots] [CODE:DEC]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from qldpcsim_amd import codes, simulator  # noqa: E402


def main():
    shots = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    runs = [
        ("LP118_2", "MS", "L", 0, 50),      # configs[3]: MS layered + OSD-0
        ("LP118_2", "BP", "L", 4, 100),     # configs[4]: BP layered (+OSD 4: ignored by simulate)
        ("LP118_0", "MS", "F", -1, 50),
    ]
    only = sys.argv[2] if len(sys.argv) > 2 else None            # e.g. "LP118_2:MS"
    for code, dec, sched, osd, it in runs:
        if only and only != f"{code}:{dec}":
            continue
        Hx, Hz = codes.load_code(code)
        for p in (0.01, 0.02, 0.05, 0.1):
            simulator.simulate_p(Hx, Hz, p, shots=shots, decType=dec, decIterations=it,
                                 decSchedule=sched, OSDorder=osd, rngSeed=2, verbose=False)  # warm-up: same batches (sizes every pinned slot)
            t0 = time.perf_counter()
            r = simulator.simulate_p(Hx, Hz, p, shots=shots, decType=dec, decIterations=it,
                                     decSchedule=sched, OSDorder=osd, rngSeed=1,
                                     verbose=False)
            dt = time.perf_counter() - t0
            qbler = 1. - (r["decSuccessExact"] + r["decSuccessDegen"]) / shots
            print(json.dumps({"code": code, "decType": dec, "sched": sched, "OSDorder": osd, "p": p,
                              "shots": shots, "shots_per_s": shots / dt, "qBLER": qbler, **r}), flush=True)


if __name__ == "__main__":
    main()
