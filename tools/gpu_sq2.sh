#!/usr/bin/env bash
# One extra SQ counter pass (wait/active breakdown) on a workload.  usage: tools/gpu_sq2.sh <tag> <workload>
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA \
  --output-format csv -d $o/pmc_SQ2_$2 -o run -- python3 bench.py --workload $2 --steps 1 --warmup 0 --no-cpu-baseline --no-interactive --no-serial-pass > $o/pmc_SQ2_$2.log 2>&1
rc=$?; tail -3 $o/pmc_SQ2_$2.log
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $o/pmc_SQ2_$2 > $o/sq2_$2.txt; grep -E "k_trace|k_shadow|k_strag|k_sky|k_shade|k_tail" $o/sq2_$2.txt | cut -c1-400
