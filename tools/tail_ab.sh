#!/usr/bin/env bash
# Runtime A/B of the path-per-thread tail depth (bench.py --tail-depth) per workload.
#   usage: tools/tail_ab.sh <tag> <workload> <depth> ...   (depth 0 = library default)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wl=$2; shift 2; mkdir -p $o
for t in "$@"; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline --no-interactive --stage-timing \
    --tail-depth $t > $o/${wl}_tail$t.json 2> $o/${wl}_tail$t.err
  python3 -c "import json;d=json.loads(open('$o/${wl}_tail$t.json').read().splitlines()[-1]);print('$wl tail $t',d['ms_per_step'],d['stage_ms_per_step'])"
done
