"""Summary of tools/stall_profile.sh: per library build, the decode kernel's
SQ wave-state counters per half-shot iteration (quad-cycles, MI355X_MICROARCH.md:
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES) and instruction counts.

usage: python tools/stall_summary.py TAG   (reads gpurun_out/stall_TAG/<lib>/p*/)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
from kernel_counters import short  # noqa: E402


def main():
    tag = sys.argv[1]
    D = os.path.join("gpurun_out", f"stall_{tag}")
    out = {"config": open(os.path.join(D, "config.txt")).read().strip(), "libs": {}}
    for lib in sorted(os.listdir(D)):
        ld = os.path.join(D, lib)
        if not os.path.isdir(ld):
            continue
        res = {}
        for k in (1, 2):
            wl = json.load(open(os.path.join(ld, f"p{k}.work.json")))["launches"]
            kern = wl[0]["kernel"]
            its = sum(x["iters"] for x in wl if x["kernel"] == kern)
            tot = defaultdict(float)
            for fn in glob.glob(os.path.join(ld, f"p{k}", "**", "*counter_collection.csv"), recursive=True):
                with open(fn) as f:
                    for row in csv.DictReader(f):
                        if short(row["Kernel_Name"]) == kern:
                            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            # the bench's warm-up launches run the same work: counters cover
            # warmup + timed launches of the worklog (both recorded)
            res["kernel"] = kern
            res[f"half_shot_iterations_p{k}"] = its
            for c, v in tot.items():
                res[c] = v
        it1, it2 = res.get("half_shot_iterations_p1"), res.get("half_shot_iterations_p2")
        per = {}
        for c, v in res.items():
            if c.startswith("SQ_"):
                d = it1 if c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                 "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                                 "SQ_ACTIVE_INST_SCA") else it2
                per[c] = v / d if d else None
        wc = per.get("SQ_WAVE_CYCLES")
        shares = {c: per[c] / wc for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                                          "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA")
                  if wc and per.get(c) is not None}
        out["libs"][lib] = {"kernel": res.get("kernel"), "per_half_shot_iteration": per,
                            "share_of_wave_cycles": shares}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
