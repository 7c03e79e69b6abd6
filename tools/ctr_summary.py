"""Summarise gpu_counters.sh passes: per-kernel counter totals (mean over dispatches).
usage: python tools/ctr_summary.py gpurun_out/ctr_TAG [kernel-substr]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
ks = sys.argv[2] if len(sys.argv) > 2 else "qldpc"
vals = defaultdict(list)
for fn in glob.glob(d + "/p*/*counter_collection.csv"):
    for row in csv.DictReader(open(fn)):
        if ks in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")
