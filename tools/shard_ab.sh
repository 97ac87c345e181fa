#!/usr/bin/env bash
# Library variants (tools/build_variants.sh; "tree" = in-tree) over emulated C2 shard counts.
#   usage: tools/shard_ab.sh <tag> "<shard counts>" <variant> ...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; gs=$2; shift 2; mkdir -p $o
for g in $gs; do
  for v in "$@"; do
    lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ "$v" = tree ] && lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
    SPTR_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-interactive \
      --emulate-shards $g > $o/g${g}_$v.json 2>$o/g${g}_$v.err
    python3 -c "import json;d=json.loads(open('$o/g${g}_$v.json').read().splitlines()[-1]);print('G=$g $v',d['ms_per_step'])"
  done
done
