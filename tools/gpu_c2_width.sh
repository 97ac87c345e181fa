#!/usr/bin/env bash
# C2 with the wide BVH (branch-free unified walk from LDS) vs the BVH2 default
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; out=gpurun_out/$1; mkdir -p $out
for spec in ${SPECS:-"0 0" "4 1" "4 2" "4 4" "4 8" "0 0"}; do set -- $spec
  timeout -k 10 200 python3 bench.py --workload c2 --steps 10 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass --bvh-width $1 --leaf-size $2 --stage-timing > $out/c2_w$1_l$2.json 2>/dev/null
  python3 -c "import json;d=json.loads(open('$out/c2_w$1_l$2.json').read().splitlines()[-1]);print('w=$1 l=$2', d['ms_per_step'], d['stage_ms_per_step'])"
done
