#!/usr/bin/env bash
# Sweep the BVH leaf-range size for the given workload: tools/leaf_sweep.sh <workload> <leaf> [<leaf> ...]
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/leaf
wl=$1; shift
for lf in "$@"; do
  timeout -k 10 300 python3 bench.py --workload "$wl" --steps 3 --warmup 1 --no-cpu-baseline --leaf-size "$lf" \
    > "gpurun_out/leaf/${wl}_$lf.json" 2>/dev/null
  python3 -c "import json;d=json.loads(open('gpurun_out/leaf/${wl}_$lf.json').read().splitlines()[-1]);print('$wl',$lf,d['value'],d['stage_ms_per_step'],d['roofline']['per_ray'])"
done
