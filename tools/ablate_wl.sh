#!/usr/bin/env bash
# SPTR_ABLATE timing experiments on one workload (experiment build; the ablated images are wrong):
# 0 none, 1 constant environment, 2 primary rays skip traversal, 4 primary misses add no radiance.
#   usage: tools/ablate_wl.sh <tag> <workload> [bits ...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SPTR_LIB=$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so
o=gpurun_out/$1; wl=$2; shift 2; mkdir -p $o
for a in ${@:-0 1 2 4 7}; do
  SPTR_ABLATE=$a timeout -k 10 300 python3 bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --no-interactive \
    --stage-timing > $o/${wl}_abl$a.json 2>$o/${wl}_abl$a.err
  python3 -c "import json;d=json.loads(open('$o/${wl}_abl$a.json').read().splitlines()[-1]);print('$wl ablate=$a',d['ms_per_step'],d['stage_ms_per_step'])"
done
