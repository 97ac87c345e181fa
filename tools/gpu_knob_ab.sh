#!/usr/bin/env bash
# Runtime-knob A/B (no rebuild): bench lines per "workload:flags" spec.  usage: tools/gpu_knob_ab.sh <tag> "c2:--tail-depth 4" ...
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift; mkdir -p $o
i=0
for spec in "$@"; do
  wl=${spec%%:*}; fl=${spec#*:}; i=$((i+1))
  timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass $fl \
    > $o/ab_$i.json 2> $o/ab_$i.err || { tail -5 $o/ab_$i.err; exit 3; }
  python3 -c "import json;d=json.loads(open('$o/ab_$i.json').read().splitlines()[-1]);print('$wl [$fl]',d['ms_per_step'],d['stage_ms_per_step'],'tail',d['tail_rays_per_step'],'handed',d.get('paths_handed_off_per_step'))"
done
