#!/usr/bin/env python3
"""Recompute a bench line's roofline from the committed rocprofv3 kernel statistics of the same session:
the timed-path instantiations (kCount = false) of the trace kernels (k_trace, k_trace_pm, k_trace_wp,
k_trace_dyn) pooled over their launches, and of the shadow kernels (k_shadow, k_shadow_dyn).
achieved = the line's bytes_per_launch / pooled average duration; frac = achieved / peak.

    usage: tools/recompute_roofline.py profiles/<tag>_bench_<wl>.json profiles/<tag>_kernel_stats_<wl>.csv
"""
import csv
import json
import re
import sys

# position of the kCount template argument per kernel
COUNT_ARG = {"k_trace_pm": 0, "k_trace": 1, "k_trace_wp": 1, "k_trace_dyn": 1, "k_shadow": 1, "k_shadow_dyn": 0}


def pooled(rows, family):
    calls, total = 0, 0.0
    for r in rows:
        m = re.search(r"sptr::(k_\w+)<([^>]*)>", r["Name"])
        if not m or m.group(1) not in COUNT_ARG or not m.group(1).startswith(family):
            continue
        if family == "k_trace" and m.group(1).startswith("k_shadow"):
            continue
        args = [a.strip() for a in m.group(2).split(",")]
        if args[COUNT_ARG[m.group(1)]] != "false":  # the instrumented (visit-count) pass
            continue
        calls += int(r["Calls"])
        total += float(r["TotalDurationNs"])
    return (total / calls * 1e-3, calls) if calls else (None, 0)


def recompute(bench_path, stats_path):
    line = json.loads(open(bench_path).read().splitlines()[-1])
    rows = list(csv.DictReader(open(stats_path)))
    out = {}
    for key, family in (("roofline", "k_trace"), ("shadow_roofline", "k_shadow")):
        r = line.get(key)
        if not r:
            continue
        avg_us, calls = pooled(rows, family)
        achieved = r["bytes_per_launch"] / (avg_us * 1e-6) / 1e9
        out[key] = {"line_frac": r["frac"], "line_avg_launch_us": r["avg_launch_us"], "stats_avg_launch_us": round(avg_us, 2),
                    "stats_launches": calls, "frac": round(achieved / r["peak"], 4),
                    "rel_diff": round(abs(achieved / r["peak"] - r["frac"]) / r["frac"], 4)}
    return out


if __name__ == "__main__":
    print(json.dumps(recompute(sys.argv[1], sys.argv[2]), indent=1))
