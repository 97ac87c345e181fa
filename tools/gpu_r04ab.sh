#!/usr/bin/env bash
# r04 A/B session: the graph-capture tests (their failure text), then the work-distribution variants
# (tools/build_variants.sh) on C2, C3, C5.  usage: tools/gpu_r04ab.sh <tag>
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread \
  -k "multibatch or many_calls or launch_graph or overlapped" > $o/pytest_graph.log 2>&1
grep -E "PASS|FAIL|Error|capture_error" $o/pytest_graph.log | head -30
for wl in c2 c3 c5; do
  for v in tree base nopm nosky notq; do
    lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ "$v" = tree ] && lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
    SPTR_LIB=$lib timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive \
      --no-serial-pass --stage-timing > $o/${wl}_$v.json 2> $o/${wl}_$v.err || { tail -5 $o/${wl}_$v.err; exit 3; }
    python3 -c "import json;d=json.loads(open('$o/${wl}_$v.json').read().splitlines()[-1]);print('$wl $v',d['ms_per_step'],d['stage_ms_per_step'])"
  done
done
