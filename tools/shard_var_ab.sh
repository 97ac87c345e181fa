#!/usr/bin/env bash
# Emulated-shard (per-rank work of a G-GPU run) timing per library variant.
#   usage: tools/shard_var_ab.sh <tag> <workload> "<variant> ..." "<G> ..."
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wl=$2; mkdir -p $o
for v in $3; do
  lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ "$v" = tree ] && lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
  for g in $4; do
    SPTR_LIB=$lib timeout -k 10 300 python3 bench.py --workload $wl --steps 20 --warmup 2 --no-cpu-baseline --no-interactive \
      --emulate-shards $g > $o/${wl}_${v}_g$g.json 2> $o/${wl}_${v}_g$g.err
    python3 -c "import json;d=json.loads(open('$o/${wl}_${v}_g$g.json').read().splitlines()[-1]);print('$wl $v G=$g',d['ms_per_step'],d['value'])"
  done
done
