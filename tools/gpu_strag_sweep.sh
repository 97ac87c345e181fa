#!/usr/bin/env bash
# Straggler hand-off sweep on C5: variants x lane thresholds (2 repetitions).  usage: tools/gpu_strag_sweep.sh <tag> <variant>...
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift; mkdir -p $o
for rep in 1 2; do
for v in "$@"; do
  for n in 4 8 12; do
    SPTR_LIB=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so timeout -k 10 300 python3 bench.py --workload c5 --steps 10 --warmup 2 \
      --no-cpu-baseline --no-interactive --no-serial-pass --stragglers $n > $o/c5_${v}_s$n.json 2> $o/c5_${v}_s$n.err || { tail -5 $o/c5_${v}_s$n.err; exit 3; }
    python3 -c "import json;d=json.loads(open('$o/c5_${v}_s$n.json').read().splitlines()[-1]);print('c5 $v s$n rep$rep',d['ms_per_step'],'handed',d['paths_handed_off_per_step'])"
  done
done
done
