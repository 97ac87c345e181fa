#!/usr/bin/env python3
"""Recompute a bench line's roofline from the committed rocprofv3 kernel statistics of the same session:
the timed-path instantiations (kCount = false) of the trace kernels (k_trace, k_trace_pm, k_trace_wp,
k_trace_dyn) pooled over their launches, and of the shadow kernels (k_shadow, k_shadow_dyn).
achieved = the line's bytes_per_launch / pooled average duration; frac = achieved / peak.
With a third file (the kernel statistics of a one-stream run, launch mode 2) the line's roofline_serial
fractions are recomputed the same way.  step_roofline: bytes_per_step = the sum of its per-kernel bytes,
frac = bytes_per_step / ms_per_step / peak.

With --trace <kernel trace csv> (the same run's rocprofv3 run_kernel_trace.csv) and a line whose roofline
carries busy_us_per_launch (pixel lanes: two launch chains whose trace launches overlap), the trace
launches' busy time — the union of their dispatch intervals — per launch is recomputed from the
dispatch timestamps and priced the way the line prices it.

    usage: tools/recompute_roofline.py profiles/<tag>_bench_<wl>.json profiles/<tag>_kernel_stats_<wl>.csv
                                       [profiles/<tag>_kernel_stats_<wl>_serial.csv] [--trace <trace csv>]
"""
import csv
import json
import re
import sys

# position of the kCount template argument per kernel
COUNT_ARG = {"k_trace_pm": 0, "k_trace": 1, "k_trace_wp": 1, "k_trace_dyn": 1, "k_shadow": 1, "k_shadow_dyn": 0,
             "k_bounce": None, "k_bounce01": None}  # (no count instantiations: the visit-count pass fuses nothing)
FAMILY = {"k_trace": ("k_trace", "k_bounce"), "k_shadow": ("k_shadow",)}


def _timed(name, family):
    """The timed-path (kCount = false) instantiation of a kernel of `family`, by its demangled name."""
    m = re.search(r"sptr::(k_\w+)<([^>]*)>", name)
    if not m or m.group(1) not in COUNT_ARG or not m.group(1).startswith(FAMILY[family]):
        return False
    pos = COUNT_ARG[m.group(1)]
    if pos is None:
        return True
    args = [a.strip() for a in m.group(2).split(",")]
    return args[pos] == "false"  # (true: the instrumented visit-count pass)


def pooled(rows, family):
    calls, total = 0, 0.0
    for r in rows:
        if _timed(r["Name"], family):
            calls += int(r["Calls"])
            total += float(r["TotalDurationNs"])
    return (total / calls * 1e-3, calls) if calls else (None, 0)


def busy_per_launch(trace_rows, family="k_trace"):
    """(union of the timed-path dispatch intervals of `family` / their count in us, count)."""
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in trace_rows if _timed(r["Kernel_Name"], family))
    if not iv:
        return None, 0
    busy, lo, hi = 0, iv[0][0], iv[0][1]
    for b, e in iv[1:]:
        if b > hi:
            busy += hi - lo
            lo, hi = b, e
        else:
            hi = max(hi, e)
    busy += hi - lo
    return busy / len(iv) * 1e-3, len(iv)


def _one(r, rows, family, peak):
    avg_us, calls = pooled(rows, family)
    achieved = r["bytes_per_launch"] / (avg_us * 1e-6) / 1e9
    return {"line_frac": r["frac"], "line_avg_launch_us": r["avg_launch_us"], "stats_avg_launch_us": round(avg_us, 2),
            "stats_launches": calls, "frac": round(achieved / peak, 4),
            "rel_diff": round(abs(achieved / peak - r["frac"]) / r["frac"], 4)}


def recompute(bench_path, stats_path, serial_stats_path=None, trace_path=None):
    line = json.loads(open(bench_path).read().splitlines()[-1])
    rows = list(csv.DictReader(open(stats_path)))
    out = {}
    for key, family in (("roofline", "k_trace"), ("shadow_roofline", "k_shadow")):
        r = line.get(key)
        if r:
            out[key] = _one(r, rows, family, r["peak"])
    r = line.get("roofline")
    if r and trace_path and r.get("busy_us_per_launch"):
        busy_us, n = busy_per_launch(list(csv.DictReader(open(trace_path))))
        frac = r["bytes_per_launch"] / (busy_us * 1e-6) / 1e9 / r["peak"]
        out["roofline"].update({"line_busy_us_per_launch": r["busy_us_per_launch"], "trace_busy_us_per_launch": round(busy_us, 2),
                                "trace_launches": n, "frac_busy": round(frac, 4),
                                "rel_diff_busy": round(abs(frac - r["frac"]) / r["frac"], 4)})
    ser = line.get("roofline_serial")
    if ser and serial_stats_path:
        srows = list(csv.DictReader(open(serial_stats_path)))
        for key, family in (("trace", "k_trace"), ("shadow", "k_shadow")):
            if ser.get(key):
                out["roofline_serial." + key] = _one(ser[key], srows, family, line["roofline"]["peak"])
    st = line.get("step_roofline")
    if st:
        total = sum(st["bytes_by_kernel"].values())
        frac = total / (st["ms_per_step"] * 1e-3) / 1e9 / st["peak"]
        out["step_roofline"] = {"line_frac": st["frac"], "frac": round(frac, 4), "bytes_per_step": total,
                                "rel_diff": round(abs(frac - st["frac"]) / max(1e-12, st["frac"]), 4)}
    return out


if __name__ == "__main__":
    argv = sys.argv[1:]
    trace = None
    if "--trace" in argv:
        i = argv.index("--trace")
        trace = argv[i + 1]
        del argv[i:i + 2]
    print(json.dumps(recompute(*argv[:3], trace_path=trace) if len(argv) >= 2 else {}, indent=1))
