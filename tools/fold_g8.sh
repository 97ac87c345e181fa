#!/usr/bin/env bash
# Bounce-0 mode at small per-rank batches (experiment build): SPTR_FOLD 0 (path-major + k_sky for the
# culled pixels) vs 2 (lane groups) vs the library's choice, on emulated C2 shards.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SPTR_LIB=$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so
o=gpurun_out/${1:-foldg8}; mkdir -p $o
for g in 4 8; do
  for m in auto 0 2; do
    if [ $m = auto ]; then unset SPTR_FOLD; else export SPTR_FOLD=$m; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-interactive --emulate-shards $g > $o/g${g}_$m.json 2>$o/g${g}_$m.err
    python3 -c "import json;d=json.loads(open('$o/g${g}_$m.json').read().splitlines()[-1]);print('G=$g fold=$m',d['ms_per_step'])"
  done
done
