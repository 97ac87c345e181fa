#!/usr/bin/env bash
# alternate bench runs of this tree and of older trees unpacked under variants/ (each with its own
# bench.py, package and built library): tag, workload, reps, dir... (dir: a path from the repo root)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; out=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $out
wl=$2; reps=$3; shift 3
for i in $(seq 1 $reps); do for d in . "$@"; do
  n=${wl}_${i}_$(echo "$d" | tr '/.' '__')
  (cd "$GRAFT_REPO_ROOT/$d" && timeout -k 10 200 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass > $out/$n.json 2>$out/$n.err)
  python3 -c "import json;d=json.loads(open('$out/$n.json').read().splitlines()[-1]);print('$wl $d', d['ms_per_step'], d.get('stage_ms_untimed_step'))"
done; done
