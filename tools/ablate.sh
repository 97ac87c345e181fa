#!/usr/bin/env bash
# Timing experiments on one GPU (images of the ablated runs are wrong): SPTR_ABLATE bits of the
# bounce-0 trace (see k_trace), leaf size / BVH width, and emulated multi-GPU shards.
set -euo pipefail
# the SPTR_ABLATE / SPTR_MAX_BLOCKS_PER_CU knobs exist only in experiment builds:
#   tools/build_variants.sh "knobs:-DSPTR_EXPERIMENT_KNOBS"   (on the CPU, before the GPU call)
export SPTR_LIB=${SPTR_LIB:-$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-exp}
mkdir -p $o
show() { python3 -c "import json,sys; d=json.loads(open('$1').read().splitlines()[-1]); print('$2', d['ms_per_step'], d['value'], d.get('stage_ms_per_step'))"; }
for a in 0 1 2 4 7; do
  SPTR_ABLATE=$a timeout -k 10 200 python3 bench.py --no-cpu-baseline --stage-timing > $o/abl$a.json 2>$o/abl$a.err
  show $o/abl$a.json "ablate=$a"
done
for l in 2 4 16; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --leaf-size $l > $o/leaf$l.json 2>$o/leaf$l.err
  show $o/leaf$l.json "leaf=$l"
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline --bvh-width 4 > $o/w4.json 2>$o/w4.err
show $o/w4.json "width=4"
for g in 1 2 4 8; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --emulate-shards $g > $o/shard$g.json 2>$o/shard$g.err
  show $o/shard$g.json "shards=$g"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace -o run -- \
  python3 bench.py --no-cpu-baseline --steps 3 > $o/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace8 -o run -- \
  python3 bench.py --no-cpu-baseline --steps 3 --emulate-shards 8 > $o/trace8.log 2>&1
echo done
