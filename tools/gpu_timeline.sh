#!/usr/bin/env bash
# kernel-trace timeline of one timed step (the last complete render call) of a workload, plus a bench line
#   usage: tools/gpu_timeline.sh <tag> <workload> [bench flags...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; wl=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive "$@" > $out/bench_$wl.json 2> $out/bench_$wl.err
python3 -c "import json;d=json.loads(open('$out/bench_$wl.json').read().splitlines()[-1]);print('$wl', d['ms_per_step'], d.get('stage_ms_per_step'), d['roofline'].get('avg_launch_us'), (d.get('shadow_roofline') or {}).get('avg_launch_us'), d.get('roofline_serial',{}).get('ms_per_step'))"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tl_$wl -o run -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-interactive --no-serial-pass "$@" > $out/tl_$wl.log 2>&1
python3 tools/timeline.py $out/tl_$wl/run_kernel_trace.csv > $out/timeline_$wl.txt; cat $out/timeline_$wl.txt
