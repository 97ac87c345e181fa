#!/usr/bin/env bash
# Tail depth x library variant A/B: tools/tail_var_ab.sh <tag> <workload> "<variant> ..." "<depth> ..."
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wl=$2; mkdir -p $o
for v in $3; do
  lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ "$v" = tree ] && lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
  for t in $4; do
    SPTR_LIB=$lib timeout -k 10 300 python3 bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline --no-interactive \
      --stage-timing --tail-depth $t > $o/${wl}_${v}_t$t.json 2> $o/${wl}_${v}_t$t.err
    python3 -c "import json;d=json.loads(open('$o/${wl}_${v}_t$t.json').read().splitlines()[-1]);print('$wl $v tail $t',d['ms_per_step'],d['stage_ms_per_step'])"
  done
done
