#!/usr/bin/env bash
# like gpu_ab_multi.sh, with the bench's serial (one-stream) pass: ms/step, overlapped and serial trace
# fractions, trace and shadow launch averages.  usage: tools/gpu_ab_full.sh <tag> <wl> <reps> spec...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; out=gpurun_out/$1; mkdir -p $out
wl=$2; reps=$3; shift 3
for i in $(seq 1 $reps); do for spec in tree "$@"; do
  lib=${spec%%:*}; extra=""; [[ "$spec" == *:* ]] && extra=$(echo "${spec#*:}" | tr '=' ' ')
  L=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so; [ "$lib" = tree ] || L=$GRAFT_REPO_ROOT/$lib
  n=full_${wl}_${i}_$(echo "$spec" | tr '/: =' '____')
  SPTR_LIB=$L timeout -k 10 240 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive $extra > $out/$n.json 2>$out/$n.err
  python3 - "$out/$n.json" "$wl $spec" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1]); r = d["roofline"]; s = d.get("shadow_roofline") or {}
rs = d.get("roofline_serial") or {}
print(sys.argv[2], "ms", d["ms_per_step"], "frac", r.get("frac"), "trace_us", r.get("avg_launch_us"), "shadow_us", s.get("avg_launch_us"),
      "serial_ms", rs.get("ms_per_step"), "serial_frac", (rs.get("trace") or {}).get("frac"), "serial_trace_us", (rs.get("trace") or {}).get("avg_launch_us"),
      "serial_shadow_us", (rs.get("shadow") or {}).get("avg_launch_us"))
PY
done; done
