#!/usr/bin/env bash
# r05 session: bit-identity of the current library against a reference build (render dumps), the GPU
# suite, and bench lines of the given workloads.  usage: tools/gpu_r05.sh <tag> <ref.so|-> [--tests] [wl ...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=$1; ref=$2; shift 2
out=gpurun_out/$tag; mkdir -p "$out"
if [ "$ref" != "-" ]; then
  echo "[$(date +%T)] render dumps"
  timeout -k 10 180 python3 tools/micro/render_dump.py "$out/dump_new.npz" > "$out/dump_new.log" 2>&1
  SPTR_LIB="$ref" timeout -k 10 180 python3 tools/micro/render_dump.py "$out/dump_ref.npz" > "$out/dump_ref.log" 2>&1
  python3 tools/micro/compare_dumps.py "$out/dump_ref.npz" "$out/dump_new.npz" | tee "$out/dump_cmp.txt" || true
fi
if [ "${1:-}" = "--tests" ]; then
  shift
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1 || { tail -40 "$out/pytest_gpu.log"; exit 1; }
  tail -2 "$out/pytest_gpu.log"
fi
for wl in "$@"; do
  echo "[$(date +%T)] bench $wl"
  timeout -k 10 300 python3 bench.py --workload "$wl" --steps 10 --warmup 2 --no-cpu-baseline --no-interactive \
    > "$out/bench_$wl.json" 2> "$out/bench_$wl.err"
  python3 - "$out/bench_$wl.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {}); s = d.get("shadow_roofline", {}) or {}
print(d["config"]["workload"], "ms/step", round(d["ms_per_step"], 3), "value", round(d["value"]), "frac", r.get("frac"),
      "trace_us", r.get("avg_launch_us"), "shadow", {k: s.get(k) for k in ("avg_launch_us", "launches_per_step", "frac", "salu_valu")})
PY
done
echo "[$(date +%T)] done"
