#!/usr/bin/env bash
# C2 (and its emulated 8-way shard) A/B over library variants (tools/build_variants.sh).  usage: tools/gpu_variant_c2.sh <tag> <variant>...
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift; mkdir -p $o
for rep in 1 2; do
for v in "$@"; do
  for sh in 0 8; do
    ex=""; [ $sh = 8 ] && ex="--emulate-shards 8"
    SPTR_LIB=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 \
      --no-cpu-baseline --no-interactive --no-serial-pass --stage-timing $ex > $o/c2_${v}_g$sh.json 2> $o/c2_${v}_g$sh.err || { tail -5 $o/c2_${v}_g$sh.err; exit 3; }
    python3 -c "import json;d=json.loads(open('$o/c2_${v}_g$sh.json').read().splitlines()[-1]);print('c2 $v g$sh rep$rep',d['ms_per_step'],d['stage_ms_per_step'])"
  done
done
done
