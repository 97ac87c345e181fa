#!/usr/bin/env bash
# Kernel-trace statistics and SQ issue / wait / LDS counters of one workload, one rocprofv3 pass per
# counter group (<= 8 SQ counters a pass).  usage: tools/gpu_counters.sh <tag> <workload> [bench flags...]
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; wl=$2; shift 2; mkdir -p $o
extra=("$@")
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats_$wl -o run -- \
  python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-interactive --no-serial-pass "${extra[@]}" > $o/stats_$wl.log 2>&1 || exit 1
python3 tools/prof_summary.py $o/stats_$wl > $o/summary_$wl.txt; head -14 $o/summary_$wl.txt
run() {  # name, counters...
  local n=$1; shift
  local cs=("$@")
  timeout -s KILL 120 rocprofv3 --pmc "${cs[@]}" --output-format csv -d $o/cnt_${wl}_$n -o run -- \
    python3 bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline --no-interactive --no-serial-pass "${extra[@]}" > $o/cnt_${wl}_$n.log 2>&1 || return 1
  python3 tools/prof_summary.py $o/cnt_${wl}_$n > $o/cnt_${wl}_$n.txt || true
  echo "== $n"; grep -E "k_trace|k_shade|k_bounce|k_shadow|k_sky|k_tail" $o/cnt_${wl}_$n.txt | grep -v '<true' | head -12
}
run issue SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD || exit 1
run wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD || exit 1
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_INSTS_VMEM_WR SQ_IFETCH SQ_INSTS_BRANCH || exit 1
run util SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES || true
