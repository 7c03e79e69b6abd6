"""Golden vectors for the BASELINE.json decoder configurations on LP118_2
(configs[3]: MS layered + OSD-0; configs[4]: BP layered over the p-sweep),
from the UNMODIFIED reference decoders — a supplement to gen_golden.py, same
method (stub-package import, settrace capture of the final posteriors; build
container only). Writes tests/golden/bp_LP118_2.npz and ms_LP118_2_osd.npz.

Usage:  python tests/golden/gen_golden_configs.py     (≈ 2-4 minutes, 8 procs)
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
    seed = 20260101

    def add(**kw):
        nonlocal seed
        seed += 1
        kw.setdefault("osd", -1)
        kw["seed"] = seed
        kw["id"] = 10000 + len(cases)
        cases.append(kw)

    for half in ("X", "Z"):
        for sched in ("L", "F"):
            for p in (0.01, 0.02, 0.05, 0.1):              # configs[4] p-sweep
                add(algo="BP", code="LP118_2", half=half, sched=sched, kind="channel",
                    p_phys=p, shots=2, max_iter=30)
            add(algo="BP", code="LP118_2", half=half, sched=sched, kind="random",
                p_phys=0.05, shots=1, max_iter=2)
        # configs[3]: MS layered + OSD-0 on the shots that do not converge
        add(algo="MS", code="LP118_2", half=half, sched="L", kind="channel", p_phys=0.1,
            shots=2, max_iter=5, osd=0)
        add(algo="MS", code="LP118_2", half=half, sched="L", kind="random", p_phys=0.05,
            shots=1, max_iter=3, osd=0)
    return cases


def main():
    cases = build_cases()
    weight = lambda c: (100 if c["osd"] >= 0 else 1) * c["shots"] * c["max_iter"]  # noqa: E731
    results = {}
    with Pool(int(os.environ.get("GOLDEN_PROCS", "8"))) as pool:
        for case, arrs in pool.imap_unordered(g.run_case, sorted(cases, key=weight, reverse=True)):
            results[case["id"]] = (case, arrs)
            print(f"[{len(results)}/{len(cases)}] {case['algo']} {case['half']} {case['sched']} "
                  f"{case['kind']} p={case['p_phys']} it={case['max_iter']} osd={case['osd']} "
                  f"iters={arrs['iters'].tolist()}", flush=True)
    groups = {}
    for cid in sorted(results):
        case, arrs = results[cid]
        key = f"{case['algo'].lower()}_{case['code']}" + ("_osd" if case["osd"] >= 0 else "")
        groups.setdefault(key, []).append((case, arrs))
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
