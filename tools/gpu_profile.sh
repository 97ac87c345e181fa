#!/usr/bin/env bash
# One GPU-box session: bench lines + rocprofv3 kernel stats + separate FETCH_SIZE / WRITE_SIZE PMC
# passes for the given workloads.  Every GPU step has its own time limit and the steps are chained,
# so the first failure ends the script.  Output: gpurun_out/<tag>/.
#   usage: tools/gpu_profile.sh <tag> <workload> [<workload> ...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
for wl in "$@"; do
  echo "[$(date +%T)] bench $wl"
  timeout -k 10 420 python3 bench.py --workload "$wl" --steps 5 --warmup 1 > "$out/bench_$wl.json" 2> "$out/bench_$wl.err"
  tail -1 "$out/bench_$wl.json"
  echo "[$(date +%T)] rocprof stats $wl"
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats_$wl" -o run -- \
    python3 bench.py --workload "$wl" --steps 3 --warmup 1 --no-cpu-baseline > "$out/stats_$wl.log" 2>&1
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[$(date +%T)] pmc $c $wl"
    timeout -k 10 420 rocprofv3 --pmc "$c" --output-format csv -d "$out/pmc_${c}_$wl" -o run -- \
      python3 bench.py --workload "$wl" --steps 1 --warmup 0 --no-cpu-baseline > "$out/pmc_${c}_$wl.log" 2>&1
  done
  python3 tools/prof_summary.py "$out/stats_$wl" "$out/pmc_FETCH_SIZE_$wl" "$out/pmc_WRITE_SIZE_$wl" > "$out/summary_$wl.txt"
  python3 tools/prof_summary.py "$out/pmc_FETCH_SIZE_$wl" "$out/pmc_WRITE_SIZE_$wl" --emit "$out/pmc_${wl}_trace.json" \
    --kernel k_trace --workload "$wl" > /dev/null
done
echo "[$(date +%T)] done"
