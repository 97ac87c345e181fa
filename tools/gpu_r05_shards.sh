#!/usr/bin/env bash
# r05: GPU suite, interactive legs, and the strong-scaling rehearsal (per-rank work of G-GPU runs) of C2
# and C4 with a kernel trace of the 8-way C2 shard.  usage: tools/gpu_r05_shards.sh <tag> [--no-tests]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; out=gpurun_out/$tag; mkdir -p $out
if [ "${2:-}" != "--no-tests" ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
  tail -1 $out/pytest_gpu.log
fi
echo "[$(date +%T)] interactive"
timeout -k 10 600 python3 -c "
import sys, json; sys.path.insert(0,'.')
import bench
for r in bench.interactive(200): print(json.dumps(r))
" > $out/interactive.txt 2>&1
cut -c1-170 $out/interactive.txt
echo "[$(date +%T)] shards"
for spec in "c2 20" "c4 4"; do set -- $spec; wl=$1; st=$2
  for g in 1 2 4 8; do
    f=$out/${wl}_g$g
    timeout -k 10 300 python3 bench.py --workload $wl --steps $st --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass --emulate-shards $g > $f.json 2>$f.err
    python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('$wl g=$g',d['ms_per_step'],d['value'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/st8 -o run -- python3 bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline --no-interactive --no-serial-pass --emulate-shards 8 > $out/st8.log 2>&1
python3 tools/prof_summary.py $out/st8 > $out/st8_summary.txt; head -12 $out/st8_summary.txt
echo "[$(date +%T)] done"
