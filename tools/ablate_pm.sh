#!/usr/bin/env bash
# Bounce-0 ablation on C2 (experiment build; images of ablated runs are wrong by design):
# SPTR_ABLATE 1 = constant environment, 2 = no primary traversal, 4 = misses add nothing.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SPTR_LIB=$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so
o=gpurun_out/${1:-abl}; mkdir -p $o
for a in 0 1 2 3 7; do
  SPTR_ABLATE=$a timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-interactive --stage-timing --steps 10 > $o/abl$a.json 2>$o/abl$a.err
  python3 -c "import json;d=json.loads(open('$o/abl$a.json').read().splitlines()[-1]);print('ablate $a',d['ms_per_step'],d['stage_ms_per_step'])"
done
