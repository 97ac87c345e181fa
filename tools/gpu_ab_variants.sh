#!/usr/bin/env bash
# A/B of library variants (tools/build_variants.sh) on one GPU box, alternating: for each repetition and
# each variant (tree = the in-tree library), one bench line per workload spec.  A spec is a workload name
# with optional extra bench flags after colons, e.g. "c2" or "c2:--emulate-shards:8".
#   usage: tools/gpu_ab_variants.sh <tag> <reps> "<variant> ..." <spec> [<spec> ...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; reps=$2; vars=$3; shift 3
out=gpurun_out/$tag; mkdir -p "$out"
for i in $(seq 1 "$reps"); do
  for v in $vars; do
    L=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so; [ "$v" = tree ] || L=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so
    for spec in "$@"; do
      wl=${spec%%:*}; extra=""; [ "$spec" != "$wl" ] && extra=$(echo "${spec#*:}" | tr ':' ' ')
      f=$out/${wl}$(echo "$extra" | tr -d ' -')_${v}_$i.json
      SPTR_LIB=$L timeout -k 10 200 python3 bench.py --workload "$wl" $extra --steps 20 --warmup 3 --no-cpu-baseline \
        --no-interactive --no-serial-pass > "$f" 2> "$f.err"
      python3 -c "import json,sys;d=json.loads(open('$f').read().splitlines()[-1]);s=d['stage_ms_untimed_step'];print('$spec', '$v', d['ms_per_step'], 'rf', d['roofline_pass']['ms_per_step'], 'trace0', s['trace0'], 'shade0', s['shade0'], 'trace', s['trace'], 'ok', d['output_check']['identical'])"
    done
  done
done
