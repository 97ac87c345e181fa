# Strong-scaling rehearsal on one GPU: per-rank work of a G-GPU C2 run (--emulate-shards G),
# the tail-depth policy at G=8, and a kernel trace of the G=8 shard (launch gaps).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-shards}; mkdir -p $out
for wl in ${WLS:-c2}; do for g in ${GS:-1 2 4 8}; do for t in ${TS:-0}; do
  f=$out/${wl}_g${g}_t$t
  timeout -k 10 200 python3 bench.py --workload $wl --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --emulate-shards $g --tail-depth $t > $f.json 2>$f.err
  python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('$wl g=$g t=$t',d['ms_per_step'],d['value'],d['tail_rays_per_step'])"
done; done; done
[ -n "${NOPROF:-}" ] || timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/st8 -o run -- python3 bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline --emulate-shards 8 > $out/st8.log 2>&1
