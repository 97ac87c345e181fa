# Wavefront batch size sweep (paths per batch) on one GPU, per workload.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-wave}; mkdir -p $out
for wl in ${WLS:-c2 c3 c5}; do for wp in ${WPS:-16777216 33554432 67108864 134217728}; do
  f=$out/${wl}_w$wp
  timeout -k 10 200 python3 bench.py --workload $wl --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --wave-paths $wp > $f.json 2>$f.err
  python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('$wl wp=$wp',d['ms_per_step'],d['value'],d['tail_rays_per_step'])"
done; done
