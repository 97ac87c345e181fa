#!/usr/bin/env bash
# Strong-scaling rehearsal on one GPU (per-rank work of G-GPU runs, bench.py --emulate-shards G) for C2 and C4,
# the 8-way C2 shard with two pixel lanes forced, and a kernel trace of the 8-way C2 shard.
#   usage: tools/gpu_shards.sh <tag>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; out=gpurun_out/$tag; mkdir -p $out
for spec in "c2 20" "c4 4"; do set -- $spec; wl=$1; st=$2
  for g in 1 2 4 8; do
    f=$out/${wl}_g$g
    timeout -k 10 300 python3 bench.py --workload $wl --steps $st --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass --emulate-shards $g > $f.json 2>$f.err
    python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('$wl g=$g',d['ms_per_step'],d['value'],d['pixel_lanes']['active'])"
  done
done
for rep in 1 2; do
  f=$out/c2_g8_lanes2_$rep
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass --emulate-shards 8 --pixel-lanes 2 > $f.json 2>$f.err
  python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('c2 g=8 lanes=2',d['ms_per_step'],d['value'])"
  f=$out/c2_g8_$rep
  timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass --emulate-shards 8 > $f.json 2>$f.err
  python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('c2 g=8 auto',d['ms_per_step'],d['value'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/st8 -o run -- python3 bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline --no-interactive --no-serial-pass --emulate-shards 8 > $out/st8.log 2>&1
python3 tools/prof_summary.py $out/st8 > $out/st8_summary.txt; head -14 $out/st8_summary.txt
echo "[$(date +%T)] done"
