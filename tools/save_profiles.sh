#!/usr/bin/env bash
# Copy one tools/gpu_round.sh session's summaries from gpurun_out/<run>/ into profiles/<tag>_* (the
# tracked evidence bench.py's roofline reads: r*_pmc_<wl>_trace.json, r*_sq_<wl>_trace.json).
#   usage: tools/save_profiles.sh <run> <tag> <workload> ...
set -euo pipefail
cd "$(dirname "$0")/.."
run=gpurun_out/$1; tag=$2; shift 2
for wl in "$@"; do
  tail -1 $run/bench_$wl.json > profiles/${tag}_bench_$wl.json
  [ -f $run/bench_${wl}_stages.json ] && tail -1 $run/bench_${wl}_stages.json > profiles/${tag}_bench_${wl}_stages.json
  cp $run/summary_$wl.txt profiles/${tag}_summary_$wl.txt
  cp $run/stats_$wl/run_kernel_stats.csv profiles/${tag}_kernel_stats_$wl.csv
  cp $run/stats_$wl/run_kernel_trace.csv profiles/${tag}_kernel_trace_$wl.csv
  [ -f $run/stats_${wl}_serial/run_kernel_stats.csv ] && cp $run/stats_${wl}_serial/run_kernel_stats.csv profiles/${tag}_kernel_stats_${wl}_serial.csv
  for k in trace shadow; do
    [ -f $run/pmc_${wl}_$k.json ] && cp $run/pmc_${wl}_$k.json profiles/${tag}_pmc_${wl}_$k.json
    [ -f $run/sq_${wl}_$k.json ] && cp $run/sq_${wl}_$k.json profiles/${tag}_sq_${wl}_$k.json
  done
  [ -f $run/sq_$wl.txt ] && cp $run/sq_$wl.txt profiles/${tag}_sq_$wl.txt
  true
done
ls profiles/${tag}_*
