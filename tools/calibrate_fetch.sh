#!/usr/bin/env bash
# FETCH_SIZE calibration on the GPU box (tools/micro/gather_cal.hip): launch times, then FETCH_SIZE
# and the raw TCC read-request counters in passes of their own.  Output: gpurun_out/<tag>/cal_*.
#   usage: tools/calibrate_fetch.sh <tag>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1; mkdir -p "$out"
timeout -k 10 120 tools/micro/gather_cal all 5 > "$out/cal_time.jsonl"
cat "$out/cal_time.jsonl"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/cal_fetch" -o run -- tools/micro/gather_cal all 2 \
  > "$out/cal_fetch.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d "$out/cal_req" -o run -- \
  tools/micro/gather_cal all 2 > "$out/cal_req.log" 2>&1 || echo "raw request counters unavailable (rc=$?)"
python3 tools/calibrate_fetch.py "$out" > "$out/cal_summary.json"
cat "$out/cal_summary.json"
