"""Per-kernel counter summary of an arbitrary program profiled by
tools/gpu_profile_program.sh (kernels that have no bench.py work units: the
OSD order / elimination kernels, the channel sampler, the outcome counters).

usage: python tools/kernel_counters.py TAG [gpurun_out/kprof_TAG]
writes profiles/<TAG>_kernels.json: for every kernel of the trace pass
  calls, mean_duration_ns (kernel-trace --stats);
  per_dispatch: waves, VALU / LDS / SALU instructions per wave, LDS-array
      cycles, bank-conflict share, HBM bytes (2 x FETCH_SIZE + WRITE_SIZE,
      MI355X_MICROARCH.md gfx950 correction, KiB -> bytes);
  busy: valu = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x cycles), lds =
      SQ_LDS_IDX_ACTIVE / (256 CUs x cycles), cycles = GRBM_GUI_ACTIVE / 8;
  hbm_gbs: HBM bytes per dispatch / mean duration (peak 8000).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)


def short(name):
    """'void qldpc::osd_block_kernel<17, 8, 2>(qldpc::OsdArgs)' -> 'osd_block_kernel<17, 8, 2>'."""
    m = re.search(r"qldpc::(?:\(anonymous namespace\)::)?([A-Za-z0-9_]+<[^()]*>|[A-Za-z0-9_]+)\(", name)
    if m:
        return m.group(1)
    m = re.match(r"(?:void )?([A-Za-z0-9_:]+)", name)          # library kernels: the qualified name only
    return m.group(1) if m else name


def pass_counters(pass_dir):
    """{kernel: {counter: sum}}, {kernel: dispatches}."""
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for fn in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                per[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id", row.get("Correlation_Id")))
    return per, {k: len(v) for k, v in disp.items()}


def main():
    tag = sys.argv[1]
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", f"kprof_{tag}")
    stats = {}
    for fn in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                stats[short(row["Name"])] = (float(row["AverageNs"]), int(row["Calls"]))
    c = defaultdict(dict)
    nd = {}
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        if not os.path.isdir(p):
            continue
        per, disp = pass_counters(p)
        for k, vals in per.items():
            c[k].update(vals)
            nd[k] = disp[k]
    import bench
    from qldpcsim_amd import _lib
    out = {"tag": tag, "program": open(os.path.join(d, "cmd.txt")).read().strip()
           if os.path.exists(os.path.join(d, "cmd.txt")) else None,
           "note": "tools/gpu_profile_program.sh + tools/kernel_counters.py; one rocprofv3 --pmc pass per "
                   "counter set; FETCH_SIZE doubled (gfx950), KiB -> bytes", "kernels": []}
    for k in sorted(c, key=lambda k: -(stats.get(k, (0, 0))[0] * stats.get(k, (0, 0))[1])):
        v, n = c[k], max(nd.get(k, 1), 1)
        ent = {"kernel": k, "code_sha256": bench.kernel_code_sha(_lib.LIB_PATH, k)}
        if k in stats:
            ent["mean_duration_ns"], ent["calls"] = stats[k]
            ent["total_ms"] = stats[k][0] * stats[k][1] / 1e6
        w = v.get("SQ_WAVES", 0.0)
        pd = {"dispatches_counted": n}
        if w:
            pd["waves"] = w / n
            for cn, key in (("SQ_INSTS_VALU", "valu_insts_per_wave"), ("SQ_INSTS_LDS", "lds_insts_per_wave"),
                            ("SQ_INSTS_SALU", "salu_insts_per_wave")):
                if cn in v:
                    pd[key] = v[cn] / w
        if "SQ_LDS_IDX_ACTIVE" in v:
            pd["lds_cycles"] = v["SQ_LDS_IDX_ACTIVE"] / n
            if v["SQ_LDS_IDX_ACTIVE"]:
                pd["lds_conflict_share"] = v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            pd["hbm_bytes"] = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024 / n
        ent["per_dispatch"] = pd
        if v.get("GRBM_GUI_ACTIVE"):
            cyc = v["GRBM_GUI_ACTIVE"] / 8.0
            ent["busy"] = {"valu": v.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / 1024 / cyc,
                           "lds": v.get("SQ_LDS_IDX_ACTIVE", 0.0) / 256 / cyc}
        if "hbm_bytes" in pd and ent.get("mean_duration_ns"):
            ent["hbm_gbs"] = pd["hbm_bytes"] / ent["mean_duration_ns"]
            ent["hbm_frac"] = ent["hbm_gbs"] / bench.HBM_PEAK_GBS
        out["kernels"].append(ent)
    path = os.path.join(ROOT, "profiles", f"{tag}_kernels.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
