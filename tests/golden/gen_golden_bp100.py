"""100-iteration BP golden vectors (the BASELINE iteration count) from the
UNMODIFIED reference decoders: configs[4] (LP118_2, BP layered, p-sweep
[0.01, 0.02, 0.05, 0.1]) with 8 channel shots per p and half, and configs[2]
(LP118_0, BP flooding and layered) with 8 shots at p = 0.06 and 0.12, plus
arbitrary syndromes (never converging) — so the BP parity tests pin
full-length decodes, not only <= 30 iterations. Same method as gen_golden.py
(stub-package import, settrace capture of the final posteriors; build
container only). Writes tests/golden/bp_LP118_2_it100.npz and
tests/golden/bp_LP118_0_it100.npz.

Usage:  python tests/golden/gen_golden_bp100.py     (8 procs)
"""
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as g  # noqa: E402


def build_cases():
    cases = []
    seed = 20261016

    def add(**kw):
        nonlocal seed
        seed += 1
        kw.setdefault("osd", -1)
        kw["seed"] = seed
        kw["id"] = 20000 + len(cases)
        cases.append(kw)

    for half in ("X", "Z"):
        for p in (0.01, 0.02, 0.05, 0.1):
            for part in range(2):                          # 2 x 4 shots per (half, p)
                add(algo="BP", code="LP118_2", half=half, sched="L", kind="channel",
                    p_phys=p, shots=4, max_iter=100)
    for sched in ("F", "L"):
        for p in (0.06, 0.12):                             # 0.12: mostly full 100-iteration decodes
            for part in range(2):
                add(algo="BP", code="LP118_0", half="X", sched=sched, kind="channel",
                    p_phys=p, shots=4, max_iter=100)
    for half in ("X", "Z"):                                # arbitrary syndromes: never converge
        add(algo="BP", code="LP118_2", half=half, sched="L", kind="random", p_phys=0.05, shots=2,
            max_iter=100)
    return cases


def main():
    cases = build_cases()
    if len(sys.argv) > 1:                                  # timing probe: first N cases
        cases = cases[: int(sys.argv[1])]
    results = {}
    with Pool(int(os.environ.get("GOLDEN_PROCS", "8"))) as pool:
        for case, arrs in pool.imap_unordered(g.run_case, cases):
            results[case["id"]] = (case, arrs)
            print(f"[{len(results)}/{len(cases)}] {case['code']} {case['half']} {case['sched']} "
                  f"p={case['p_phys']} it={case['max_iter']} iters={arrs['iters'].tolist()}", flush=True)
    groups = {}
    for cid in sorted(results):
        case, arrs = results[cid]
        groups.setdefault(f"bp_{case['code']}_it100", []).append((case, arrs))
    for key, items in groups.items():
        out = {}
        meta = []
        for i, (case, arrs) in enumerate(items):
            meta.append(case)
            for name, a in arrs.items():
                out[f"c{i}_{name}"] = a
        out["cases_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        np.savez_compressed(os.path.join(HERE, f"{key}.npz"), **out)
        print("wrote", key, len(items), "cases")


if __name__ == "__main__":
    main()
