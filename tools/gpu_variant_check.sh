#!/usr/bin/env bash
# bit-identity of variant libraries against the tree library (render dumps of C2/C3/C5 and two mesh
# scenes).  usage: tools/gpu_variant_check.sh <tag> <lib> ...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 180 python3 tools/micro/render_dump.py $out/dump_tree.npz > $out/dump_tree.log 2>&1
for lib in "$@"; do
  n=$(echo $lib | tr '/' '_')
  SPTR_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 180 python3 tools/micro/render_dump.py $out/dump_$n.npz > $out/dump_$n.log 2>&1
  echo "== $lib"; python3 tools/micro/compare_dumps.py $out/dump_tree.npz $out/dump_$n.npz || true
done
