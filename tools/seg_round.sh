# Quick GPU check: the GPU test suite, then bench lines for the given workloads (default c2 c3).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-quick}; shift || true; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
for wl in ${@:-c2 c3}; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_$wl.json 2>$out/bench_$wl.err
  python3 -c "import json;d=json.loads(open('$out/bench_$wl.json').read().splitlines()[-1]);print('$wl',d['ms_per_step'],d['value'],d['tail_rays_per_step'])"
done
