"""Summarise tools/gpu_profile_roofline.sh runs into profiles/<TAG>_roofline.json,
the per-unit counter profile bench.py prices its roofline with.

usage: python tools/roofline_profile.py TAG [gpurun_out/roof_TAG]

For every profiled config (a subdirectory holding trace/, p1..pN/ rocprofv3
outputs and the bench --worklog of each run) and every decode kernel in it:
  per_half_shot_iteration: SQ_INSTS_VALU, SQ_LDS_IDX_ACTIVE (LDS-array cycles),
      SQ_INSTS_LDS, SQ_INSTS_SALU, SQ_LDS_BANK_CONFLICT, SQ_WAVE_CYCLES (quad),
      summed over the kernel's dispatches / the executed half-shot iterations
      the worklog records for those dispatches;
  per_half_shot: HBM bytes = 2 x FETCH_SIZE (gfx950 half-count correction,
      MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both KiB -> bytes;
  busy: valu = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x cycles), lds =
      SQ_LDS_IDX_ACTIVE / (256 CUs x cycles), cycles = GRBM_GUI_ACTIVE / 8 XCDs
      (the profiled run's own clock, for cross-checking bench.py's frac);
  mean_duration_ns: the kernel-trace --stats average of the trace pass.
Each counter comes from its own --pmc pass; units from that pass's worklog.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)


def kernel_match(row_name, kernel):
    return ("::" + kernel + "(") in row_name


def counters(pass_dir, kernel):
    """{counter: summed value over the kernel's dispatches}, dispatch count."""
    per = defaultdict(float)
    disp = set()
    for fn in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if not kernel_match(row["Kernel_Name"], kernel):
                    continue
                per[row["Counter_Name"]] += float(row["Counter_Value"])
                disp.add(row.get("Dispatch_Id", row.get("Correlation_Id", len(disp))))
    return dict(per), len(disp)


def work(worklog, kernel):
    with open(worklog) as f:
        L = [x for x in json.load(f)["launches"] if x["kernel"] == kernel]
    return len(L), sum(x["half_shots"] for x in L), sum(x["iters"] for x in L)


def stats(trace_dir, kernel):
    for fn in glob.glob(os.path.join(trace_dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if kernel_match(row["Name"], kernel):
                    return float(row["AverageNs"]), int(row["Calls"])
    return None, 0


def resolve(trace_dir, family):
    """Full kernel name for a worklog entry: a family name without template
    arguments (tools/osd_bench.py) is looked up in the trace's kernel names."""
    if "<" in family:
        return family
    for fn in glob.glob(os.path.join(trace_dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                nm = row["Name"]
                for tail in ("<", "("):
                    i = nm.find("::" + family + tail)
                    if i >= 0:
                        j = nm.find("(", i)
                        return nm[i + 2:j]
    return family


def summarise_config(d):
    with open(os.path.join(d, "trace.work.json")) as f:
        wl = json.load(f)
    kernels = sorted({x["kernel"] for x in wl["launches"]})
    unit = wl.get("unit", "half_shot_iteration")
    meta = {}
    if os.path.exists(os.path.join(d, "config.txt")):
        meta["bench_args"] = open(os.path.join(d, "config.txt")).read().strip()
    out = []
    for fam in kernels:
        k = resolve(os.path.join(d, "trace"), fam)
        c = {}
        ok = True
        for p in sorted(glob.glob(os.path.join(d, "p*"))):
            if not os.path.isdir(p):
                continue
            vals, nd = counters(p, k)
            nl, hs, it = work(p + ".work.json", fam)
            if nd != nl:
                print(f"{p}: {nd} dispatches of {k} but the worklog has {nl}", file=sys.stderr)
                ok = False
            for name, v in vals.items():
                c[name] = (v, hs, it)
        if not ok or not c:
            continue
        per_it = lambda n: c[n][0] / c[n][2]            # noqa: E731
        per_hs = lambda n: c[n][0] / c[n][1]            # noqa: E731
        import bench
        from qldpcsim_amd import _lib
        ent = {"kernel": k, **meta, "code_sha256": bench.kernel_code_sha(_lib.LIB_PATH, k),
               **({"unit": unit + " (per_half_shot_iteration and per_half_shot are per " + unit + ")"}
                  if unit != "half_shot_iteration" else {}),
               "per_half_shot_iteration": {
                   "valu_insts": per_it("SQ_INSTS_VALU"),
                   "lds_cycles": per_it("SQ_LDS_IDX_ACTIVE"),
                   "lds_insts": per_it("SQ_INSTS_LDS"),
                   "salu_insts": per_it("SQ_INSTS_SALU"),
                   "lds_bank_conflict_cycles": per_it("SQ_LDS_BANK_CONFLICT"),
                   "wave_quad_cycles": per_it("SQ_WAVE_CYCLES")},
               "per_half_shot": {
                   "hbm_fetch_bytes": 2 * 1024 * per_hs("FETCH_SIZE"),
                   "hbm_write_bytes": 1024 * per_hs("WRITE_SIZE")}}
        ent["per_half_shot"]["hbm_bytes"] = ent["per_half_shot"]["hbm_fetch_bytes"] + \
            ent["per_half_shot"]["hbm_write_bytes"]
        # VALU issue cycles by instruction class (MI355X_MICROARCH.md: a wave64
        # 32-bit VALU op issues over 2 cycles on a SIMD-32; float64 add / mul /
        # fma at half rate, 4; transcendentals 8 (f32) / 16 (f64, v_rcp_f64))
        cls = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
               "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_FMA_F32",
               "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32"]
        if all(k in c for k in cls):
            pc = {k[len("SQ_INSTS_VALU_"):].lower(): per_it(k) for k in cls}
            tot = per_it("SQ_INSTS_VALU")
            pc["other"] = tot - sum(pc.values())     # moves, bit ops, compares, f64 min/max if unclassified
            f64 = pc["add_f64"] + pc["mul_f64"] + pc["fma_f64"]
            ent["per_half_shot_iteration"]["valu_classes"] = pc
            ent["per_half_shot_iteration"]["valu_cycles"] = (2 * tot + 2 * f64 + 14 * pc["trans_f64"] +
                                                              6 * pc["trans_f32"])
            # the unclassified remainder holds float64 min / max / compares
            # (v_min_f64 & co. have no class counter): upper bound = all of it
            # at the float64 rate
            ent["per_half_shot_iteration"]["valu_cycles_hi"] = \
                ent["per_half_shot_iteration"]["valu_cycles"] + 2 * max(pc["other"], 0.0)
        # LDS path cycles (MI355X_MICROARCH.md §LDS): SQ_LDS_IDX_ACTIVE counts the
        # array cycles; a store also moves its address and data VGPRs to the
        # LDS at 2 cycles per source dword, which for ds_write_b32 / b64 is 2
        # cycles more than its array cycles (4 vs 2, 6 vs 4): path = array +
        # 2 x stores (a lower bound for 12- / 16-byte stores)
        if "SQ_INSTS_LDS_STORE" in c:
            pi = ent["per_half_shot_iteration"]
            pi["lds_store_insts"] = per_it("SQ_INSTS_LDS_STORE")
            pi["lds_load_insts"] = per_it("SQ_INSTS_LDS_LOAD")
            pi["lds_store_bytes"] = 64 * per_it("SQ_INSTS_LDS_STORE_BANDWIDTH")
            pi["lds_load_bytes"] = 64 * per_it("SQ_INSTS_LDS_LOAD_BANDWIDTH")
            pi["lds_path_cycles"] = pi["lds_cycles"] + 2 * pi["lds_store_insts"]
        # the SQ pass's own dispatches: busy fractions at its measured clock
        v, hs, it = c["GRBM_GUI_ACTIVE"]
        cyc = v / 8.0
        ent["busy"] = {"valu": c["SQ_ACTIVE_INST_VALU"][0] * 4 / 1024 / cyc,
                       "lds": c["SQ_LDS_IDX_ACTIVE"][0] / 256 / cyc,
                       "lds_conflict_share": c["SQ_LDS_BANK_CONFLICT"][0] / max(c["SQ_LDS_IDX_ACTIVE"][0], 1.0)}
        ns, calls = stats(os.path.join(d, "trace"), k)
        ent["mean_duration_ns"] = ns
        ent["trace_calls"] = calls
        tnl, ths, tit = work(os.path.join(d, "trace.work.json"), fam)
        if ns:
            # clock implied by the SQ pass's cycles at the trace pass's duration, per unit of work
            ent["clock_ghz"] = (cyc / it) / (ns * tnl / tit)
            ent["trace_units_per_call"] = {"half_shots": ths / tnl, "half_shot_iterations": tit / tnl}
        out.append(ent)
    return out


def main():
    tag = sys.argv[1]
    d = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", f"roof_{tag}")
    import bench
    from qldpcsim_amd import _lib
    doc = {"tag": tag, "device_code_sha256": bench.device_code_sha(_lib.LIB_PATH),
           "note": "tools/gpu_profile_roofline.sh + tools/roofline_profile.py; one rocprofv3 --pmc pass "
                   "per counter set; FETCH_SIZE doubled (gfx950), KiB -> bytes",
           "kernels": []}
    for cfg in sorted(glob.glob(os.path.join(d, "*", "trace.work.json"))):
        doc["kernels"] += summarise_config(os.path.dirname(cfg))
    path = os.path.join(ROOT, "profiles", f"{tag}_roofline.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
