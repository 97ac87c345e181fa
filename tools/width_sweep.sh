#!/usr/bin/env bash
# A/B the BVH width on the given workloads: tools/width_sweep.sh <workload> ...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/width
for wl in "$@"; do
  for w in 2 4; do
    timeout -k 10 300 python3 bench.py --workload "$wl" --steps 3 --warmup 1 --no-cpu-baseline --bvh-width "$w" \
      > "gpurun_out/width/${wl}_$w.json" 2>/dev/null
    python3 -c "import json;d=json.loads(open('gpurun_out/width/${wl}_$w.json').read().splitlines()[-1]);print('$wl',$w,d['value'],d['stage_ms_per_step'],d['roofline']['per_ray'],d['scene']['traversed_nodes'],d['scene']['leaf_size'])"
  done
done
