#!/usr/bin/env bash
# alternate bench runs of the tree library and several variant libraries on one workload:
#   tag, workload, reps, spec...   spec = lib[:bench args] (lib: "tree" or a path from the repo root;
#   bench args with '=' or ',' for spaces, e.g. tree:--tail-depth=4,--pixel-lanes=1)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; out=gpurun_out/$1; mkdir -p $out
wl=$2; reps=$3; shift 3
specs=("$@"); [ ${#specs[@]} -gt 0 ] || specs=(tree)
for i in $(seq 1 $reps); do for spec in tree "${specs[@]}"; do
  lib=${spec%%:*}; extra=""; [[ "$spec" == *:* ]] && extra=$(echo "${spec#*:}" | tr '=,' '  ')
  L=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so; [ "$lib" = tree ] || L=$GRAFT_REPO_ROOT/$lib
  n=${wl}_${i}_$(echo "$spec" | tr '/: =,' '_____')
  SPTR_LIB=$L timeout -k 10 200 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass $extra > $out/$n.json 2>$out/$n.err
  python3 -c "import json;d=json.loads(open('$out/$n.json').read().splitlines()[-1]);print('$wl $spec', d['ms_per_step'])"
done; done
