#!/usr/bin/env bash
# One GPU-box session: the GPU test suite (parity fractions logged to gpurun_out/<tag>/parity), then
# library-variant A/B timings (tools/variant_ab.sh) per workload.  A failing test does not stop the
# A/B runs; a crash, abort or timeout of any GPU step ends the script.
#   usage: tools/gpu_tests_ab.sh <tag> "<wl> <variant> ..." ["<wl> <variant> ..."]
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/$tag; mkdir -p "$out"
echo "[$(date +%T)] pytest -m gpu"
SPTR_PARITY_LOG=$out/parity timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$out/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for spec in "$@"; do
  set -- $spec
  echo "[$(date +%T)] A/B $*"
  bash tools/variant_ab.sh "$tag" "$@" || exit $?
done
echo "[$(date +%T)] done (pytest rc=$rc)"
