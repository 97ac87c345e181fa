#!/usr/bin/env bash
# A/B timing of library variants (tools/build_variants.sh) on one workload: stage timing per variant.
#   usage: tools/variant_ab.sh <tag> <workload> <variant> ...   (variant "tree": the in-tree library)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wl=$2; shift 2; mkdir -p $o
for v in "$@"; do
  lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ "$v" = tree ] && lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
  SPTR_LIB=$lib timeout -k 10 300 python3 bench.py --workload $wl --steps 5 --warmup 1 \
    --no-cpu-baseline --no-interactive --stage-timing > $o/${wl}_$v.json 2> $o/${wl}_$v.err
  python3 -c "import json;d=json.loads(open('$o/${wl}_$v.json').read().splitlines()[-1]);sc=d.get('scene',{});print('$wl $v',d['ms_per_step'],d['stage_ms_per_step'],{k:sc[k] for k in ('bvh_depth','bvh_width','lbvh_build_ms') if k in sc})"
done
