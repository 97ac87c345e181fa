#!/usr/bin/env bash
# alternate bench runs of the tree library and a reference library on one workload: tag, ref.so, wl, reps
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; out=gpurun_out/$1; mkdir -p $out
for i in $(seq 1 ${4:-3}); do for lib in tree "$2"; do
  L=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so; [ "$lib" = tree ] || L=$GRAFT_REPO_ROOT/$lib
  SPTR_LIB=$L timeout -k 10 200 python3 bench.py --workload $3 --steps 10 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass > $out/$3_${i}_$(basename $lib).json 2>/dev/null
  python3 -c "import json;d=json.loads(open('$out/$3_${i}_$(basename $lib).json').read().splitlines()[-1]);print('$3 $lib', d['ms_per_step'])"
done; done
