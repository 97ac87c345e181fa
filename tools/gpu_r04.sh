#!/usr/bin/env bash
# Round-4 GPU session step: the GPU suite and the C5/C3/C2 bench lines.  usage: tools/gpu_r04.sh <tag> [pytest -k expr]
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1; mkdir -p $out
sel=${2:-}
if [ -n "$sel" ]; then
  SPTR_PARITY_LOG=$out/parity timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$sel" > $out/pytest_gpu.log 2>&1
else
  SPTR_PARITY_LOG=$out/parity timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
fi
rc=$?
tail -25 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for wl in c5 c3 c2; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-interactive > $out/bench_$wl.json 2> $out/bench_$wl.err || exit 3
  python3 -c "import json;d=json.loads(open('$out/bench_$wl.json').read().splitlines()[-1]);r=d['roofline'];print('$wl',d['ms_per_step'],d['value'],'trace',r['avg_launch_us'],r['frac'],'hist',r.get('visit_hist_log2'),'serial',json.dumps(d.get('roofline_serial')),'step',d.get('step_roofline',{}).get('frac'),'graph',d.get('graph_replay'),'stages',d['stage_ms_per_step'])"
done
# the 8-way C2 per-rank cost (one GPU rendering shard 0 of 8): direct launches vs the graph replay pass
timeout -k 10 300 python3 bench.py --workload c2 --emulate-shards 8 --steps 20 --warmup 3 --no-cpu-baseline --no-interactive > $out/bench_c2_g8.json 2> $out/bench_c2_g8.err || exit 4
python3 -c "import json;d=json.loads(open('$out/bench_c2_g8.json').read().splitlines()[-1]);print('c2 g8',d['ms_per_step'],'render',d['render_ms'],'graph',d.get('graph_replay'),'stages',d['stage_ms_per_step'])"
