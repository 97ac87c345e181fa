#!/usr/bin/env bash
# Quick GPU check after a kernel change: GPU test suite, C2 bench line, emulated shard sweep with a
# kernel trace of the 8-way shard.  Output: gpurun_out/<tag>/.   usage: tools/gpu_quick.sh <tag>
#   env: GS (shard counts, default "2 4 8"), WLS (workloads of the sweep, default c2), SHARD_STEPS
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-interactive --steps 20 --warmup 2 > $out/bench_c2.json 2> $out/bench_c2.err
python3 -c "import json;d=json.loads(open('$out/bench_c2.json').read().splitlines()[-1]);print('c2',d['ms_per_step'],d['value'],d['stage_ms_per_step'])"
for wl in ${WLS:-c2}; do
  for g in ${GS:-2 4 8}; do
    timeout -k 10 200 python3 bench.py --workload $wl --steps ${SHARD_STEPS:-20} --warmup 2 --no-cpu-baseline --no-interactive \
      --emulate-shards $g > $out/shard_${wl}_$g.json 2>$out/shard_${wl}_$g.err
    python3 -c "import json;d=json.loads(open('$out/shard_${wl}_$g.json').read().splitlines()[-1]);print('shard $wl $g',d['ms_per_step'],d['value'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/st1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-interactive > $out/st1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/st8 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate-shards 8 > $out/st8.log 2>&1
python3 tools/prof_summary.py $out/st1 > $out/summary_st1.txt
python3 tools/trace_gaps.py $(ls $out/st8/*kernel_trace.csv | head -1) > $out/gaps8.txt
tail -3 $out/gaps8.txt
