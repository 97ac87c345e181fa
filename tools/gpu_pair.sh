#!/usr/bin/env bash
# Two-rays-per-lane trace variants: bit-identity against the default build, then C5 / C3 timing.
#   usage: tools/gpu_pair.sh <tag> <variant>...
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift; mkdir -p $o
timeout -k 10 300 python3 tools/micro/render_dump.py $o/base.npz > $o/dump_base.log 2>&1 || { tail -5 $o/dump_base.log; exit 2; }
for v in "$@"; do
  SPTR_LIB=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so timeout -k 10 300 python3 tools/micro/render_dump.py $o/$v.npz > $o/dump_$v.log 2>&1 || { tail -5 $o/dump_$v.log; exit 2; }
  python3 tools/micro/compare_dumps.py $o/base.npz $o/$v.npz || exit 3
done
for rep in 1 2; do
for v in base "$@"; do
  lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ -f $lib ] || lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
  for wl in c5 c3; do
    SPTR_LIB=$lib timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass \
      > $o/${wl}_$v.json 2> $o/${wl}_$v.err || { tail -5 $o/${wl}_$v.err; exit 4; }
    python3 -c "import json;d=json.loads(open('$o/${wl}_$v.json').read().splitlines()[-1]);print('$wl $v rep$rep',d['ms_per_step'],d['stage_ms_per_step'],'handed',d.get('paths_handed_off_per_step'))"
  done
done
done
