#!/usr/bin/env bash
# Wait-state and cache counters of one workload's kernels, one rocprofv3 --pmc pass per counter group.
#   usage: tools/c5_counters.sh <tag> <workload>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wl=$2; mkdir -p $o
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $o/cnt_${wl}_$n -o run -- \
    python3 bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline --no-interactive > $o/cnt_${wl}_$n.log 2>&1
  python3 tools/prof_summary.py $o/cnt_${wl}_$n | grep -E "k_trace|k_shadow|k_tail|k_shade" > $o/cnt_${wl}_$n.txt || true
  echo "== $n"; cat $o/cnt_${wl}_$n.txt
}
run wait SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU
run l2 TCC_HIT_sum TCC_MISS_sum
run l1 TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
