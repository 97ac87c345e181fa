#!/usr/bin/env bash
# Emulated-shard C2 A/B over library variants: per-rank ms at G = 2, 4, 8.  usage: tools/gpu_shard_ab.sh <tag> <variant>...
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift; mkdir -p $o
for rep in 1 2; do
for v in "$@"; do
  for g in 2 4 8; do
    lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ -f $lib ] || lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
    SPTR_LIB=$lib timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 \
      --no-cpu-baseline --no-interactive --no-serial-pass --emulate-shards $g > $o/c2_${v}_g$g.json 2> $o/c2_${v}_g$g.err || { tail -5 $o/c2_${v}_g$g.err; exit 3; }
    python3 -c "import json;d=json.loads(open('$o/c2_${v}_g$g.json').read().splitlines()[-1]);print('c2 $v g$g rep$rep',d['ms_per_step'],'graph',d.get('graph_replay',{}).get('ms_per_step'),d['stage_ms_per_step'])"
  done
done
done
