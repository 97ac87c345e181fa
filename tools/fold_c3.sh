#!/usr/bin/env bash
# Bounce-0 fold modes on the L2/HBM scenes (experiment build): SPTR_FOLD 0 path-major, 2 lane groups.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-foldc3}; mkdir -p $o
export SPTR_LIB=$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so
for wl in ${WLS:-c3 c5}; do
  for m in 0 2; do
    SPTR_FOLD=$m timeout -k 10 300 python3 bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --no-interactive --stage-timing > $o/${wl}_$m.json 2>$o/${wl}_$m.err
    python3 -c "import json;d=json.loads(open('$o/${wl}_$m.json').read().splitlines()[-1]);print('$wl fold=$m',d['ms_per_step'],d['stage_ms_per_step'])"
  done
done
