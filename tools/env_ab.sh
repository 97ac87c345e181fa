#!/usr/bin/env bash
# A/B timing of library environment knobs on one workload: stage timing per setting.
#   usage: tools/env_ab.sh <tag> <workload> "<name>:<VAR=V VAR2=V>" ...   ("<name>:" = no variable)
#   env: AB_FLAGS (extra bench flags, e.g. "--launch-mode 1")
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wl=$2; shift 2; mkdir -p $o
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  env $vars timeout -k 10 300 python3 bench.py --workload $wl --steps 5 --warmup 1 \
    --no-cpu-baseline --no-interactive --stage-timing ${AB_FLAGS:-} > $o/${wl}_$name.json 2> $o/${wl}_$name.err
  python3 -c "import json;d=json.loads(open('$o/${wl}_$name.json').read().splitlines()[-1]);print('$wl $name',d['ms_per_step'],d['stage_ms_per_step'])"
done
