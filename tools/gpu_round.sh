#!/usr/bin/env bash
# One GPU-box session: GPU tests (optional), bench lines, rocprofv3 kernel trace + stats, and separate
# FETCH_SIZE / WRITE_SIZE PMC passes per workload.  Every GPU step has its own time limit and the
# steps are chained (set -e), so the first failure ends the script.  Output: gpurun_out/<tag>/.
#   usage: tools/gpu_round.sh <tag> [--tests] [--sq] <workload> [<workload> ...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
tests=0; sq=0; benchflags=${BENCHFLAGS:-}
while [ $# -gt 0 ] && [ "${1#--}" != "$1" ]; do
  case $1 in --tests) tests=1 ;; --sq) sq=1 ;; esac
  shift
done
if [ $tests = 1 ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1 || { tail -40 "$out/pytest_gpu.log"; exit 1; }
  tail -2 "$out/pytest_gpu.log"
fi
# Per workload the counter passes run first and their summaries are emitted into profiles/ (on the
# box), so that the bench line that follows cites this session's counters (bench.py picks the
# newest summary by its collection time); tools/save_profiles.sh copies them into the tracked tree.
for wl in "$@"; do
  echo "[$(date +%T)] rocprof kernel trace + stats $wl"
  # (no untimed one-stream / one-chain passes: the statistics pool only launches run as the timed steps run)
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats_$wl" -o run -- \
    python3 bench.py --workload "$wl" --steps 3 --warmup 1 --no-cpu-baseline --no-interactive --no-serial-pass $benchflags > "$out/stats_$wl.log" 2>&1
  if [ "$wl" = c3 ] || [ "$wl" = c5 ]; then  # the launches alone: one stream, nothing overlapped (roofline_serial)
    echo "[$(date +%T)] rocprof kernel trace + stats $wl, launch mode 2"
    timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats_${wl}_serial" -o run -- \
      python3 bench.py --workload "$wl" --steps 3 --warmup 1 --no-cpu-baseline --no-interactive --launch-mode 2 > "$out/stats_${wl}_serial.log" 2>&1
  fi
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[$(date +%T)] pmc $c $wl"
    timeout -s KILL 300 rocprofv3 --pmc "$c" --output-format csv -d "$out/pmc_${c}_$wl" -o run -- \
      python3 bench.py --workload "$wl" --steps 1 --warmup 0 --no-cpu-baseline --no-interactive > "$out/pmc_${c}_$wl.log" 2>&1
  done
  python3 tools/prof_summary.py "$out/stats_$wl" "$out/pmc_FETCH_SIZE_$wl" "$out/pmc_WRITE_SIZE_$wl" > "$out/summary_$wl.txt"
  for k in trace shadow; do
    kn=k_$k; [ $k = trace ] && kn=k_trace,k_bounce  # (the fused bounce launches count as trace launches)
    python3 tools/prof_summary.py "$out/pmc_FETCH_SIZE_$wl" "$out/pmc_WRITE_SIZE_$wl" --emit "$out/pmc_${wl}_$k.json" \
      --kernel $kn --workload "$wl" > /dev/null
    cp "$out/pmc_${wl}_$k.json" "profiles/${tag}_pmc_${wl}_$k.json"
  done
  if [ $sq = 1 ]; then
    echo "[$(date +%T)] pmc SQ $wl"
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$out/pmc_SQ_$wl" -o run -- \
      python3 bench.py --workload "$wl" --steps 1 --warmup 0 --no-cpu-baseline --no-interactive > "$out/pmc_SQ_$wl.log" 2>&1
    python3 tools/prof_summary.py "$out/pmc_SQ_$wl" > "$out/sq_$wl.txt"
    for k in trace shadow; do
      kn=k_$k; [ $k = trace ] && kn=k_trace,k_bounce
      python3 tools/prof_summary.py "$out/pmc_SQ_$wl" --emit "$out/sq_${wl}_$k.json" --kernel $kn --workload "$wl" > /dev/null
      cp "$out/sq_${wl}_$k.json" "profiles/${tag}_sq_${wl}_$k.json"
    done
  fi
  echo "[$(date +%T)] bench $wl"
  timeout -k 10 420 python3 bench.py --workload "$wl" $benchflags > "$out/bench_$wl.json" 2> "$out/bench_$wl.err"
  tail -1 "$out/bench_$wl.json"
  echo "[$(date +%T)] bench $wl --stage-timing"
  timeout -k 10 420 python3 bench.py --workload "$wl" --stage-timing --no-cpu-baseline --no-interactive \
    > "$out/bench_${wl}_stages.json" 2> "$out/bench_${wl}_stages.err"
done
echo "[$(date +%T)] done"
