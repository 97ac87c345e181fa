#!/usr/bin/env python3
"""Summarise tools/calibrate_fetch.sh: per access shape, FETCH_SIZE bytes per launch against the known
distinct bytes the launch reads (and the raw TCC_EA0_RDREQ / _32B request counts when collected).
gather_cal runs the six modes in order, each as one warm-up + 2 measured launches of k_read."""
import collections
import csv
import glob
import json
import os
import sys

MODES = ["stream", "line", "half", "node", "tri", "r16"]
PER_MODE = 3  # warm-up + 2 launches


def per_dispatch(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_read" in r["Kernel_Name"]:
                vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(vals)
    out = {}
    for m, name in enumerate(MODES):
        chunk = ids[m * PER_MODE:(m + 1) * PER_MODE][1:]
        if not chunk:
            continue
        keys = set().union(*(vals[i].keys() for i in chunk))
        out[name] = {k: sum(vals[i][k] for i in chunk) / len(chunk) for k in keys}
    return out


def main():
    d = sys.argv[1]
    times = {}
    for line in open(os.path.join(d, "cal_time.jsonl")):
        r = json.loads(line)
        times[r["mode"]] = r
    fetch = per_dispatch(os.path.join(d, "cal_fetch"))
    req = per_dispatch(os.path.join(d, "cal_req")) if os.path.isdir(os.path.join(d, "cal_req")) else {}
    res = {}
    for m in MODES:
        if m not in times:
            continue
        known = times[m]["known_bytes"]
        e = {"known_bytes": known, "useful_GBps": times[m]["useful_GBps"], "us_per_launch": times[m]["us_per_launch"]}
        if m in fetch and "FETCH_SIZE" in fetch[m]:
            fb = fetch[m]["FETCH_SIZE"] * 1024.0
            e["fetch_size_bytes"] = fb
            e["known_over_fetch_size"] = known / fb if fb else None  # the factor to apply to FETCH_SIZE
        if m in req:
            e["requests"] = req[m]
            n = times[m]["known_bytes"] / {"stream": 16, "line": 128, "half": 64, "node": 64, "tri": 48, "r16": 16}[m]
            e["rdreq_per_access"] = {k: v / n for k, v in req[m].items()}
        res[m] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
