#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output: per-kernel launch stats and PMC counters (per dispatch mean).

usage: prof_summary.py <rocprof output dir> [...] [--emit OUT.json --kernel k_trace --workload c2]
--emit writes the per-launch HBM bytes of every dispatch whose name contains --kernel (a comma list:
any of them; all template
instantiations pooled), combining FETCH_SIZE and WRITE_SIZE from separate --pmc passes, for bench.py's
roofline.traffic.
FETCH_SIZE is reported doubled (gfx950 counts 128-B requests as 64 B for wide streams:
MI355X_MICROARCH.md §HBM); WRITE_SIZE as read.
"""
import collections
import csv
import datetime
import glob
import json
import os
import sys


def _now():
    """UTC collection time; bench.py cites the newest emitted file by this field."""
    return datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def short(n):
    n = n.replace("sptr::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


# position of the visit-count flag C among each kernel's template arguments
_COUNT_ARG = {"k_trace": 1, "k_trace_dyn": 1, "k_trace_wp": 1, "k_trace_pm": 0, "k_shadow": 1, "k_shadow_dyn": 0}


def _is_count_variant(name):
    """The instrumented (C = true) visit-count instantiation of a trace / shadow kernel runs only in
    bench.py's untimed counting pass and is left out of the per-launch means."""
    if "<" not in name:
        return False
    base = name.replace("sptr::", "").split("<", 1)[0].split()[-1]
    pos = _COUNT_ARG.get(base)
    args = [a.strip() for a in name.split("<", 1)[1].split(">", 1)[0].split(",")]
    return pos is not None and len(args) > pos and args[pos] == "true"


def emit(dirs, kernel, out_path, workload):
    per = collections.defaultdict(list)  # counter -> per-dispatch values for matching kernels
    dur = []
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            vals = collections.defaultdict(float)
            for r in csv.DictReader(open(f)):
                if any(k in r["Kernel_Name"] for k in kernel.split(",")) and not _is_count_variant(r["Kernel_Name"]):
                    vals[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
                    if r["Counter_Name"] == "SQ_INSTS_VALU":
                        dur.append((r["Dispatch_Id"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
            for (_, c), v in vals.items():
                per[c].append(v)
    mean = {c: sum(v) / len(v) for c, v in per.items() if v}
    if "SQ_INSTS_VALU" in mean:  # SQ pass: VALU wave-instructions per launch (bench.py valu_issue_frac)
        d = dict(dur)
        t = sum(d.values()) / max(1, len(d))
        res = {"workload": workload, "collected": _now(), "kernel": kernel, "dispatches": len(per["SQ_INSTS_VALU"]),
               "valu_per_launch": mean["SQ_INSTS_VALU"], "counters_per_launch": mean,
               "profiled_launch_us": t * 1e6,
               "valu_issue_frac_profiled": mean["SQ_INSTS_VALU"] / t / (256 * 4 * 0.5 * 2.4e9) if t else None,
               "note": "SQ_INSTS_VALU counts wave-instructions; peak issue 256 CU x 4 SIMD x 0.5/cycle x 2.4 GHz "
                       "(MI355X_MICROARCH.md: a wave issues a VALU instruction over 2 cycles); the visit-count "
                       "instantiation of the untimed pass is excluded"}
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
        return
    fetch = 2.0 * mean.get("FETCH_SIZE", 0.0) * 1024.0
    write = mean.get("WRITE_SIZE", 0.0) * 1024.0
    res = {"workload": workload, "collected": _now(), "kernel": kernel, "dispatches": {c: len(v) for c, v in per.items()},
           "fetch_bytes_per_launch_x2": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (calibrated for 16-B/lane streams only); "
                   "Infinity-Cache hits are counted by these memory-side counters; mean over the dispatches of "
                   "every instantiation of the kernel except the visit-count one of the untimed pass"}
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
