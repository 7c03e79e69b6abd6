"""GPU idle gaps of the timed simulate_p run in a tools/bench_sim_one.py
kernel trace (gpu_run.sh sim3trace): the run is the second half of the
trace's channel_sample_kernel launches (warm-up and timed runs sample the
same batches); busy = union of kernel and copy intervals.
usage: python tools/pipeline_gaps.py TRACE_DIR [MIN_GAP_MS]"""
import csv
import glob
import json
import os
import sys


def rows(d, pat):
    out = []
    for fn in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name") or r.get("Direction") or "copy"
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return out


def main():
    d = sys.argv[1]
    min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
    kern = rows(d, "*kernel_trace.csv")
    copies = rows(d, "*memory_copy_trace.csv")
    samp = sorted(s for s, _, n in kern if "channel_sample_kernel" in n)
    t0 = samp[len(samp) // 2]
    ev = sorted(x for x in kern + copies if x[0] >= t0)
    t1 = max(e for _, e, _ in ev)
    busy, gaps = 0, []
    cur_s, cur_e, last = ev[0][0], ev[0][1], ev[0][2]
    for s, e, n in ev[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            if (s - cur_e) / 1e6 >= min_gap:
                gaps.append({"ms": round((s - cur_e) / 1e6, 2), "after": last[:60], "before": n[:60]})
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        last = n if e >= cur_e else last
    busy += cur_e - cur_s
    win = (t1 - t0) / 1e6
    by = {}
    for s, e, n in ev:
        k = n.split("(")[0][-60:]
        by[k] = by.get(k, 0) + (e - s) / 1e6
    top = sorted(by.items(), key=lambda x: -x[1])[:8]
    print(json.dumps({"window_ms": round(win, 1), "busy_ms": round(busy / 1e6, 1),
                      "busy_frac": round(busy / 1e6 / win, 3),
                      "gap_ms_total": round(sum(g["ms"] for g in gaps), 1), "gaps": gaps,
                      "time_by_name_ms": {k: round(v, 1) for k, v in top}}, indent=1))


if __name__ == "__main__":
    main()
