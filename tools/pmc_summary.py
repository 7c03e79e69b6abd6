"""Summarise rocprofv3 outputs for profiles/.

usage: python tools/pmc_summary.py <round-tag> <code> <batch> <kernel-substr>
  reads gpurun_out/prof_<tag>/*kernel_stats.csv, gpurun_out/pmc_fetch[_<tag>]/*counter_collection.csv,
  gpurun_out/pmc_write[_<tag>]/*counter_collection.csv; writes profiles/<tag>_kernel_stats.csv and
  profiles/<tag>_pmc.json (HBM bytes per decode launch).

Counter handling (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
it is doubled (for this kernel's byte-wide syndrome loads the factor is
uncalibrated; the doubled value matches the 251.7 MB of syndromes read to 5%).
Each counter comes from its own --pmc pass.
"""
import csv
import glob
import json
import os
import shutil
import sys


def per_launch(path, counter, kernel):
    vals = []
    for fn in glob.glob(path):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == counter and kernel in row["Kernel_Name"]:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    tag, code, batch, kernel = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    root = os.path.join(os.path.dirname(__file__), "..")
    out = os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    for fn in glob.glob(os.path.join(root, "gpurun_out", f"prof_{tag}", "*kernel_stats.csv")):
        shutil.copy(fn, os.path.join(out, f"{tag}_kernel_stats.csv"))
    def pmc_dir(kind):
        d = os.path.join(root, "gpurun_out", f"pmc_{kind}_{tag}")
        return d if os.path.isdir(d) else os.path.join(root, "gpurun_out", f"pmc_{kind}")
    fetch = per_launch(os.path.join(pmc_dir("fetch"), "*counter_collection.csv"), "FETCH_SIZE", kernel)
    write = per_launch(os.path.join(pmc_dir("write"), "*counter_collection.csv"), "WRITE_SIZE", kernel)
    if not fetch or not write:
        raise SystemExit("no PMC rows for kernel " + kernel)
    f = sum(fetch) / len(fetch) * 1024 * 2
    w = sum(write) / len(write) * 1024
    d = {"code": code, "batch": batch, "kernel": kernel,
         "fetch_size_kib_raw": sum(fetch) / len(fetch), "write_size_kib_raw": sum(write) / len(write),
         "fetch_bytes_corrected": f, "write_bytes": w, "hbm_bytes_per_launch": f + w,
         "note": "FETCH_SIZE x1024 x2 (gfx950 half-count correction) + WRITE_SIZE x1024, "
                 "mean over launches, separate --pmc passes"}
    with open(os.path.join(out, f"{tag}_pmc.json"), "w") as fo:
        json.dump(d, fo, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
