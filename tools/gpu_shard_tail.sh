#!/usr/bin/env bash
# emulated C2 shards: tail-depth sweep (alternating) and one line with the graph-replay leg
#   usage: tools/gpu_shard_tail.sh <tag> <G> <reps> <tail depths...>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; G=$2; reps=$3; shift 3; out=gpurun_out/$tag; mkdir -p $out
for i in $(seq 1 $reps); do for t in "$@"; do
  f=$out/c2_g${G}_t${t}_$i
  timeout -k 10 200 python3 bench.py --workload c2 --steps 20 --warmup 2 --no-cpu-baseline --no-interactive --no-serial-pass --emulate-shards $G --tail-depth $t > $f.json 2>$f.err
  python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('c2 g=$G tail=$t',d['ms_per_step'],d['render_ms'])"
done; done
f=$out/c2_g${G}_graph
timeout -k 10 200 python3 bench.py --workload c2 --steps 20 --warmup 2 --no-cpu-baseline --no-interactive --emulate-shards $G > $f.json 2>$f.err
python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('c2 g=$G default',d['ms_per_step'],'graph',d.get('graph_replay'))"
