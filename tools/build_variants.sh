#!/usr/bin/env bash
# Build variants of libsptr_hip.so (occupancy hints, experiment knobs) for A/B timing via SPTR_LIB.
# Sources are built in /tmp; only the library lands in variants/<tag>/ (which travels to the GPU box).
#   usage: tools/build_variants.sh "tag:-DFLAG=V -DFLAG2=V" ...
set -euo pipefail
cd "$(dirname "$0")/.."
rm -rf variants && mkdir -p variants && ln -sfn ../include variants/include
for spec in "$@"; do
  tag=${spec%%:*}; defs=${spec#*:}
  b=/tmp/sptr_variant_build/$tag; rm -rf $b; mkdir -p $b variants/$tag
  cp -r simple-path-tracer_amd/csrc simple-path-tracer_amd/host simple-path-tracer_amd/tools simple-path-tracer_amd/Makefile $b/
  ln -sfn "$PWD/include" /tmp/sptr_variant_build/include
  make -s -C $b -j8 libsptr_hip.so HIPCC="/opt/rocm/bin/hipcc $defs"
  cp $b/libsptr_hip.so variants/$tag/
  echo "$tag: variants/$tag/libsptr_hip.so ($defs)"
done
