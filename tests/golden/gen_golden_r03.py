"""Round-3 golden vectors: every BASELINE config pinned to the UNMODIFIED
reference decoders at the config's own settings (same method as
gen_golden.py: stub-package import, settrace capture of the final
posteriors; build container only). Three files:

* ms_LP118_0_headline.npz — the exact headline workload (BASELINE.json
  metric): LP118_0, MS flooding, 50 iterations, uniform random syndromes
  (never satisfiable: rank H = 232 < m = 240), prior 0.05/3; 64 shots per
  half. decoders.py:110-182.
* ms_LP118_2_osd50.npz — configs[3]'s setting: LP118_2, MS layered,
  50 iterations, channel p = 0.1; per half 80 shots, of which the
  non-converged ones also carry the reference's OSD-0 and OSD-1 estimates
  (`ehat_osd0`, `ehat_osd1`, decoders.py:179-180 -> OSDdec :299-370, called
  with the reference's own posteriors exactly as MS_decoder does).
* bp_LP118_2_it100_long.npz — configs[4]'s decoder at the two p where long
  decodes happen: LP118_2, BP layered, 100 iterations, channel p = 0.1 and
  0.05, 64 shots per (p, half). decoders.py:189-290.

Usage:  python tests/golden/gen_golden_r03.py [headline|osd|bp ...]   (8 procs)
"""
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as g  # noqa: E402


def build_cases(which):
    cases = []
    seed = 20261017

    def add(**kw):
        nonlocal seed
        seed += 1
        kw.setdefault("osd", -1)
        kw["seed"] = seed
        kw["id"] = 30000 + len(cases)
        cases.append(kw)

    for half in ("X", "Z"):
        for part in range(8):                               # 8 x 8 = 64 shots per half
            add(group="ms_LP118_0_headline", algo="MS", code="LP118_0", half=half, sched="F",
                kind="random", p_phys=0.05, shots=8, max_iter=50)
    for half in ("X", "Z"):
        for part in range(8):                               # 8 x 10 = 80 channel shots per half
            add(group="ms_LP118_2_osd50", algo="MS", code="LP118_2", half=half, sched="L",
                kind="channel", p_phys=0.1, shots=10, max_iter=50, osd_orders=[0, 1])
    for p in (0.1, 0.05):
        for half in ("X", "Z"):
            for part in range(8):                           # 8 x 8 = 64 shots per (p, half)
                add(group="bp_LP118_2_it100_long", algo="BP", code="LP118_2", half=half,
                    sched="L", kind="channel", p_phys=p, shots=8, max_iter=100)
    keep = {"headline": "ms_LP118_0_headline", "osd": "ms_LP118_2_osd50",
            "bp": "bp_LP118_2_it100_long"}
    groups = {keep[w] for w in which} if which else set(keep.values())
    return [c for c in cases if c["group"] in groups]


def run(case):
    """One case: the reference decoder per shot (gen_golden.run_case), then,
    for OSD cases, the reference OSDdec on every non-converged shot with the
    decoder's own final posteriors (what MS_decoder does at :179-180)."""
    orders = case.get("osd_orders")
    c, arrs = g.run_case({k: v for k, v in case.items() if k != "osd_orders"})
    c = dict(c, **({"osd_orders": orders} if orders else {}))
    if not orders:
        return c, arrs
    dec = g.ref_decoders()
    H, _ = g.half_inputs(case["code"], case["half"], case["sched"])
    syn = arrs["syn"].astype(int)
    conv = np.array([np.array_equal(syn[k], (H.astype(np.int64) @ arrs["ehat"][k].astype(np.int64)) % 2)
                     for k in range(syn.shape[0])])
    arrs["conv"] = conv.astype(np.uint8)
    for o in orders:
        e_o = arrs["ehat"].copy()
        for k in np.flatnonzero(~conv):
            e = arrs["ehat"][k].astype(np.int8)
            e_o[k] = np.asarray(dec.OSDdec(H, e, syn[k], arrs["post"][k], o)).astype(np.uint8)
        arrs[f"ehat_osd{o}"] = e_o
    return c, arrs


def main():
    cases = build_cases(sys.argv[1:])
    weight = lambda c: c["shots"] * c["max_iter"] * (20 if c["algo"] == "BP" else 1) * \
        (40 if c.get("osd_orders") else 1) * (2 if c["p_phys"] >= 0.1 else 1)  # noqa: E731
    results = {}
    with Pool(int(os.environ.get("GOLDEN_PROCS", "8"))) as pool:
        for case, arrs in pool.imap_unordered(run, sorted(cases, key=weight, reverse=True)):
            results[case["id"]] = (case, arrs)
            extra = f" conv={arrs['conv'].tolist()}" if "conv" in arrs else ""
            print(f"[{len(results)}/{len(cases)}] {case['group']} {case['half']} p={case['p_phys']} "
                  f"iters={arrs['iters'].tolist()}{extra}", flush=True)
    groups = {}
    for cid in sorted(results):
        case, arrs = results[cid]
        groups.setdefault(case["group"], []).append((case, arrs))
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
