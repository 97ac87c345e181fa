#!/usr/bin/env bash
# Cull-head A/B: GPU suite on the in-tree library (k_cull heads direct RECULL calls), then C2 and the
# 8-way C2 shard alternating with variants/nohead (k_frame_dyn ahead of k_cull).
#   usage: tools/gpu_head_ab.sh <tag>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -60 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
lib() { [ "$1" = tree ] && echo $GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so || echo $GRAFT_REPO_ROOT/variants/$1/libsptr_hip.so; }
for rep in 1 2; do
  for v in tree nohead; do
    for g in 8 1; do
      ex=""; [ $g = 8 ] && ex="--emulate-shards 8"
      SPTR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-interactive $ex \
        > $o/c2_g${g}_${v}_$rep.json 2> $o/c2_g${g}_${v}_$rep.err
      python3 -c "import json;d=json.loads(open('$o/c2_g${g}_${v}_$rep.json').read().splitlines()[-1]);print('g$g $v $rep',d['ms_per_step'],d['output_check']['identical'] if 'output_check' in d else '')"
    done
  done
done
