#!/usr/bin/env bash
# k_miss A/B: GPU suite on the in-tree library (deferred misses by k_miss beside k_shade), then C5 and C3
# bench lines alternating with variants/nomiss (k_shade makes them).   usage: tools/gpu_miss_ab.sh <tag>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -60 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
lib() { [ "$1" = tree ] && echo $GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so || echo $GRAFT_REPO_ROOT/variants/$1/libsptr_hip.so; }
for rep in 1 2; do
  for wl in c5 c3; do
    for v in tree nomiss; do
      SPTR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-interactive \
        > $o/${wl}_${v}_$rep.json 2> $o/${wl}_${v}_$rep.err
      python3 -c "import json;d=json.loads(open('$o/${wl}_${v}_$rep.json').read().splitlines()[-1]);print('$wl $v $rep',d['ms_per_step'],d['output_check']['identical'],d.get('stage_ms_untimed_step'))"
    done
  done
done
