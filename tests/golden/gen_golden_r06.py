"""Round-6 golden vectors: BASELINE.json configs[0] at its own setting, from
the UNMODIFIED reference decoders (same method as gen_golden.py: stub-package
import, settrace capture of the final posteriors; build container only).

* ms_steane_cfg0.npz — Steane [[7,1,3]], MS flooding, 50 iterations,
  depolarizing p = 0.01 (prior p/3, simulator.py:278-282), 1000 channel shots
  per half (configs[0]'s shot count), in 8 parts of 125. decoders.py:110-182.

Usage:  python tests/golden/gen_golden_r06.py   (8 procs, seconds)
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
    seed = 20261018
    for half in ("X", "Z"):
        for part in range(8):
            seed += 1
            cases.append(dict(group="ms_steane_cfg0", algo="MS", code="steane", half=half, sched="F",
                              kind="channel", p_phys=0.01, shots=125, max_iter=50, osd=-1, seed=seed,
                              id=60000 + len(cases)))
    return cases


def main():
    cases = build_cases()
    results = {}
    with Pool(int(os.environ.get("GOLDEN_PROCS", "8"))) as pool:
        for case, arrs in pool.imap_unordered(g.run_case, cases):
            results[case["id"]] = (case, arrs)
            print(f"[{len(results)}/{len(cases)}] {case['group']} {case['half']} p={case['p_phys']} "
                  f"nonzero syndromes={int(arrs['syn'].any(axis=1).sum())} max iters={int(arrs['iters'].max())}",
                  flush=True)
    items = [results[c] for c in sorted(results)]
    out, meta = {}, []
    for i, (case, arrs) in enumerate(items):
        meta.append(case)
        for name, a in arrs.items():
            out[f"c{i}_{name}"] = a
    out["cases_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "ms_steane_cfg0.npz"), **out)
    print("wrote ms_steane_cfg0", len(items), "cases")


if __name__ == "__main__":
    main()
