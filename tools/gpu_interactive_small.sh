#!/usr/bin/env bash
# interactive 1-spp frames of the L2/HBM scenes at small sizes, launch modes 0 / 1 (graph vs direct)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1
python3 -c "import sys; sys.path.insert(0,'simple-path-tracer_amd'); import workloads; workloads.write_hdr('/tmp/sky.hdr', workloads.synthetic_sky_equirect())"
for sz in "256 144" "512 288" "960 540"; do set -- $sz $1; for m in 0 1; do
  timeout -k 10 120 simple-path-tracer_amd/sptr_cli --scene sphere_mesh:1250:4000 --w $1 --h $2 --spp 200 --warmup 10 --launch-mode $m --json --out /dev/null | cut -c1-200
  timeout -k 10 120 simple-path-tracer_amd/sptr_cli --scene gltf:assets/rattan_dining_chair/scene.gltf --env /tmp/sky.hdr --w $1 --h $2 --spp 200 --warmup 10 --launch-mode $m --json --out /dev/null | cut -c1-200
done; done
