# Build occupancy-hint variants of libsptr_hip.so into variants/<tag>/ (A/B timing via SPTR_LIB).
#   usage: tools/build_variants.sh "tag:-DFLAG=V -DFLAG2=V" ...
set -euo pipefail
mkdir -p variants && ln -sfn ../include variants/include
cd "$(dirname "$0")/.."
for spec in "$@"; do
  tag=${spec%%:*}; defs=${spec#*:}
  d=variants/$tag; mkdir -p $d
  cp -r simple-path-tracer_amd/csrc simple-path-tracer_amd/host simple-path-tracer_amd/tools simple-path-tracer_amd/Makefile $d/ 2>/dev/null || true
  make -s -C $d -j8 libsptr_hip.so HIPCC="/opt/rocm/bin/hipcc $defs"
  echo "$tag: $d/libsptr_hip.so ($defs)"
done
