#!/usr/bin/env bash
# Sweep resident blocks per CU (SPTR_MAX_BLOCKS_PER_CU) for the given workloads.
set -euo pipefail
# the SPTR_ABLATE / SPTR_MAX_BLOCKS_PER_CU knobs exist only in experiment builds:
#   tools/build_variants.sh "knobs:-DSPTR_EXPERIMENT_KNOBS"   (on the CPU, before the GPU call)
export SPTR_LIB=${SPTR_LIB:-$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/occ
for wl in "$@"; do
  for b in 4 5 6 7 8; do
    SPTR_MAX_BLOCKS_PER_CU=$b timeout -k 10 300 python3 bench.py --workload "$wl" --steps 3 --warmup 1 --no-cpu-baseline \
      > "gpurun_out/occ/${wl}_$b.json" 2>/dev/null
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/occ/${wl}_$b.json').read().splitlines()[-1]);print('$wl',$b,d['value'],d['stage_ms_per_step'])"
  done
done
