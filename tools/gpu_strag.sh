#!/usr/bin/env bash
# Straggler hand-off session: its parity tests, then C5 (and C3) A/B: library default vs off vs 64/32 lanes.
#   usage: tools/gpu_strag.sh <tag>
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread \
  -k "straggler or overlapped or multibatch or tail_depth or launch_graph" > $o/pytest_strag.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|handed" $o/pytest_strag.log | head -30
[ $rc -eq 0 ] || exit $rc
for wl in c5; do
  for v in -1 0 64 32 8; do
    timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass \
      --stragglers $v > $o/${wl}_s$v.json 2> $o/${wl}_s$v.err || { tail -5 $o/${wl}_s$v.err; exit 3; }
    python3 -c "import json;d=json.loads(open('$o/${wl}_s$v.json').read().splitlines()[-1]);print('$wl stragglers $v',d['ms_per_step'],d['stage_ms_per_step'],'handed',d['paths_handed_off_per_step'],'rays',d['rays_per_step'])"
  done
done
