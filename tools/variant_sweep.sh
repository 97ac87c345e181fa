# A/B timing of build variants (tools/build_variants.sh) through SPTR_LIB, with per-stage timing.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-variants}; mkdir -p $out
for wl in ${WLS:-c2 c3 c5}; do for v in ${VS:-base}; do
  f=$out/${wl}_$v${SFX:-}
  SPTR_LIB=$PWD/variants/$v/libsptr_hip.so timeout -k 10 200 python3 bench.py --workload $wl --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --stage-timing ${EXTRA:-} > $f.json 2>$f.err
  python3 -c "import json;d=json.loads(open('$f.json').read().splitlines()[-1]);print('$wl $v ${EXTRA:-}',d['ms_per_step'],d['value'],d['stage_ms_per_step'])"
done; done
