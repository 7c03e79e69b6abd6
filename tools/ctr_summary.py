"""Summarise gpu_counters.sh passes: per-kernel counter means over dispatches,
plus derived unit utilisations.

usage: python tools/ctr_summary.py gpurun_out/ctr_TAG [kernel-substr] [--json OUT]

Derived figures (MI355X: 256 CUs in 8 XCDs, 4 SIMDs per CU; SQ counters are
summed over the chip, GRBM_GUI_ACTIVE over the 8 XCDs):
  cycles      = GRBM_GUI_ACTIVE / 8                      (kernel duration, GPU clocks)
  valu_busy   = SQ_ACTIVE_INST_VALU * 4 / 1024 / cycles  (a wave64 VALU op holds its
                SIMD 4 cycles; the counter ticks once per instruction)
  lds_busy    = SQ_LDS_IDX_ACTIVE / 256 / cycles         (LDS array cycles per CU)
  lds_conflict_share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  per_wave_iter_* = instruction counts per wave per decoder iteration, given
                --work HALFSHOTS ITERS (one wave decodes one half-shot)
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def summarise(d, ks="qldpc", work=None):
    vals = defaultdict(list)
    for fn in glob.glob(d + "/p*/*counter_collection.csv"):
        for row in csv.DictReader(open(fn)):
            if ks in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"counters": mean}
    if "GRBM_GUI_ACTIVE" in mean:
        cyc = mean["GRBM_GUI_ACTIVE"] / 8
        out["cycles"] = cyc
        if "SQ_ACTIVE_INST_VALU" in mean:
            out["valu_busy"] = mean["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / cyc
        if "SQ_LDS_IDX_ACTIVE" in mean:
            out["lds_busy"] = mean["SQ_LDS_IDX_ACTIVE"] / 256 / cyc
    if mean.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict_share"] = mean.get("SQ_LDS_BANK_CONFLICT", 0.0) / mean["SQ_LDS_IDX_ACTIVE"]
    if work:
        hs, it = work
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if k in mean:
                out["per_wave_iter_" + k[9:].lower()] = mean[k] / (hs * it)
    return out


def main():
    argv = sys.argv[1:]
    work = None
    if "--work" in argv:
        i = argv.index("--work")
        work = (float(argv[i + 1]), float(argv[i + 2]))
        del argv[i:i + 3]
    jpath = None
    if "--json" in argv:
        i = argv.index("--json")
        jpath = argv[i + 1]
        del argv[i:i + 2]
    d = argv[0]
    ks = argv[1] if len(argv) > 1 else "qldpc"
    out = summarise(d, ks, work)
    for k in sorted(out["counters"]):
        print(f"{k:28s} {out['counters'][k]:16.4g}")
    for k in sorted(out):
        if k != "counters":
            print(f"{k:28s} {out[k]:16.4g}")
    if jpath:
        out["source"] = d
        out["kernel_filter"] = ks
        with open(jpath, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
