#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output: per-kernel launch stats and PMC counters (per dispatch mean).

usage: prof_summary.py <rocprof output dir> [...] [--emit OUT.json --kernel k_trace --workload c2]
--emit writes the per-launch HBM bytes of every dispatch whose name contains --kernel (all template
instantiations pooled), combining FETCH_SIZE and WRITE_SIZE from separate --pmc passes, for bench.py's
roofline.traffic.
FETCH_SIZE is reported doubled (gfx950 counts 128-B requests as 64 B for wide streams:
MI355X_MICROARCH.md §HBM); WRITE_SIZE as read.
"""
import collections
import csv
import glob
import json
import os
import sys


def short(n):
    n = n.replace("sptr::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def emit(dirs, kernel, out_path, workload):
    per = collections.defaultdict(list)  # counter -> per-dispatch values for matching kernels
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            vals = collections.defaultdict(float)
            for r in csv.DictReader(open(f)):
                if kernel in r["Kernel_Name"]:
                    vals[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            for (_, c), v in vals.items():
                per[c].append(v)
    mean = {c: sum(v) / len(v) for c, v in per.items() if v}
    fetch = 2.0 * mean.get("FETCH_SIZE", 0.0) * 1024.0
    write = mean.get("WRITE_SIZE", 0.0) * 1024.0
    res = {"workload": workload, "kernel": kernel, "dispatches": {c: len(v) for c, v in per.items()},
           "fetch_bytes_per_launch_x2": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (calibrated for 16-B/lane streams only); "
                   "Infinity-Cache hits are counted by these memory-side counters; mean over all dispatches of "
                   "every instantiation of the kernel"}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


def main():
    if "--emit" in sys.argv:
        a = sys.argv[1:]
        out = a[a.index("--emit") + 1]
        kernel = a[a.index("--kernel") + 1] if "--kernel" in a else "k_trace"
        wl = a[a.index("--workload") + 1] if "--workload" in a else "c2"
        dirs = [x for i, x in enumerate(a) if not x.startswith("--") and (i == 0 or not a[i - 1].startswith("--"))]
        emit(dirs, kernel, out, wl)
        return
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            print(f"== {f}")
            for r in csv.DictReader(open(f)):
                print(f"  {short(r['Name']):48s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:10.2f} "
                      f"pct={float(r['Percentage']):6.2f}")
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            print(f"== {f}")
            agg = collections.defaultdict(lambda: collections.defaultdict(float))
            dispatches = collections.defaultdict(set)
            dur = {}
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                dispatches[k].add(r["Dispatch_Id"])
                dur[(k, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            for k, v in agg.items():
                n = len(dispatches[k])
                t = sum(x for (kk, _), x in dur.items() if kk == k) / n
                out = {c: val / n for c, val in v.items()}
                if "FETCH_SIZE" in out:
                    out["FETCH_SIZE_x2_GBps"] = 2 * out["FETCH_SIZE"] * 1024 / t / 1e9
                if "WRITE_SIZE" in out:
                    out["WRITE_GBps"] = out["WRITE_SIZE"] * 1024 / t / 1e9
                if "GRBM_GUI_ACTIVE" in out:
                    out["clock_GHz"] = out["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
                print(f"  {k:48s} n={n:3d} t_us={t*1e6:9.1f} " + " ".join(f"{c}={x:.4g}" for c, x in sorted(out.items())))


if __name__ == "__main__":
    main()
