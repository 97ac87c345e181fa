#!/usr/bin/env bash
# k_sky for the thread-per-pixel bounce 0 (SPTR_PM_SKY): parity tests of the pixel-major paths, then C2 A/B.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -v --timeout 240 --timeout-method thread \
  -k "pixel_major or fold or golden or c2 or render_default or progressive or shards or graph" > $o/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAIL" $o/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_variant_c2.sh $(basename $o)_ab "$@"
