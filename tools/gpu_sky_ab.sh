#!/usr/bin/env bash
# A/B of library variants on C5 (bench lines alternating), after the overlap parity tests on each variant.
#   usage: tools/gpu_sky_ab.sh <tag> <variant> ...   ("tree": the in-tree library)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift; mkdir -p $o
lib() { [ "$1" = tree ] && echo $GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so || echo $GRAFT_REPO_ROOT/variants/$1/libsptr_hip.so; }
for v in "$@"; do
  [ "$v" = tree ] && continue
  SPTR_LIB=$(lib $v) timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "overlapped or many_lights or straggler" > $o/pytest_$v.log 2>&1 || { tail -30 $o/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $o/pytest_$v.log)"
done
for rep in 1 2; do
  for v in "$@"; do
    SPTR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --workload ${WL:-c5} --steps 20 --warmup 3 --no-cpu-baseline --no-interactive \
      > $o/${WL:-c5}_${v}_$rep.json 2> $o/${WL:-c5}_${v}_$rep.err
    python3 -c "import json;d=json.loads(open('$o/${WL:-c5}_${v}_$rep.json').read().splitlines()[-1]);print('$v $rep',d['ms_per_step'],d.get('stage_ms_untimed_step'))"
  done
done
