set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r01e
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r01e/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r01e/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r01e/pytest_gpu.log
for wl in c2 c5; do for t in 1 2 3 6; do
  timeout -k 10 300 python3 bench.py --workload $wl --tail-depth $t --no-cpu-baseline --stage-timing > gpurun_out/r01e/bench_${wl}_t$t.json 2>gpurun_out/r01e/bench_${wl}_t$t.err
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r01e/bench_${wl}_t$t.json').read().splitlines()[-1]); print('$wl t=$t', d['value'], d['ms_per_step'], d['stage_ms_per_step'], d['tail_rays_per_step'])"
done; done
