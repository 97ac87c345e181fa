#!/usr/bin/env bash
# The default bench line (20 timed steps after 3 warmup) of each workload, citing the committed
# counter summaries: tag, workload...  Output: gpurun_out/<tag>/bench_<wl>.json
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
for wl in "$@"; do
  echo "[$(date +%T)] bench $wl"
  timeout -k 10 420 python3 bench.py --workload "$wl" > "$out/bench_$wl.json" 2> "$out/bench_$wl.err"
  python3 -c "import json;d=json.loads(open('$out/bench_$wl.json').read().splitlines()[-1]);print('$wl', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
