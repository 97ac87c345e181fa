#!/usr/bin/env bash
# Deferred-tail A/B: GPU suite on the in-tree library, then C5 / C3 bench lines alternating the in-tree
# library (deferred tail) with variants/nodefer (the r06 sequence) and variants/deferl2 (C3 defers too).
#   usage: tools/gpu_defer_ab.sh <tag>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -60 $o/pytest_gpu.log; exit 1; }
tail -2 $o/pytest_gpu.log
run() {  # workload variant rep
  lib=$GRAFT_REPO_ROOT/variants/$2/libsptr_hip.so; [ "$2" = tree ] && lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
  SPTR_LIB=$lib timeout -k 10 300 python3 bench.py --workload $1 --steps 20 --warmup 3 --no-cpu-baseline --no-interactive \
    > $o/$1_$2_$3.json 2> $o/$1_$2_$3.err
  python3 -c "import json;d=json.loads(open('$o/$1_$2_$3.json').read().splitlines()[-1]);print('$1 $2 $3',d['ms_per_step'],d.get('stage_ms_untimed_step'))"
}
for rep in 1 2; do
  for v in tree nodefer; do run c5 $v $rep; done
  for v in tree deferl2; do run c3 $v $rep; done
done
