#!/usr/bin/env bash
# Tail-depth sweep (first bounce traced path per thread) on emulated shards.
#   usage: tools/tail_sweep.sh <tag> <workload> "<shard counts>" "<depths>"
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wl=$2; mkdir -p $o
for g in $3; do
  for t in $4; do
    timeout -k 10 200 python3 bench.py --workload $wl --steps 20 --warmup 2 --no-cpu-baseline --no-interactive \
      --emulate-shards $g --tail-depth $t > $o/${wl}_g${g}_t$t.json 2>$o/${wl}_g${g}_t$t.err
    python3 -c "import json;d=json.loads(open('$o/${wl}_g${g}_t$t.json').read().splitlines()[-1]);print('$wl G=$g tail=$t',d['ms_per_step'])"
  done
done
