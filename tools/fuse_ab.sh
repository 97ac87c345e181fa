#!/usr/bin/env bash
# Fused-bounce threshold A/B (variants fb24 / fb30 vs the in-tree 2^26) over emulated C2 shards.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-fuse}; mkdir -p $o
for g in 1 2 4; do
  for v in tree fb30 fb24; do
    lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ "$v" = tree ] && lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
    SPTR_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-interactive --emulate-shards $g \
      > $o/g${g}_$v.json 2>$o/g${g}_$v.err
    python3 -c "import json;d=json.loads(open('$o/g${g}_$v.json').read().splitlines()[-1]);print('G=$g $v',d['ms_per_step'])"
  done
done
