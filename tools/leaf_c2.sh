#!/usr/bin/env bash
# C2 trace-time sweep over BVH leaf size and width (LDS-staged default scene).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-leaf}; mkdir -p $o
for cfg in "--leaf-size 1" "--leaf-size 2" "--leaf-size 4" "--leaf-size 8" "--leaf-size 16" "--bvh-width 4 --leaf-size 2" "--bvh-width 4 --leaf-size 4" "--bvh-width 4 --leaf-size 8"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-interactive --stage-timing --steps 10 $cfg > $o/$tag.json 2>$o/$tag.err
  python3 -c "import json;d=json.loads(open('$o/$tag.json').read().splitlines()[-1]);print('$cfg',d['ms_per_step'],d['stage_ms_per_step'],d['roofline']['per_ray'])"
done
