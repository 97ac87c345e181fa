#!/usr/bin/env bash
# 1-spp progressive frames of the default scene through sptr_cli at several sizes, launch modes 0/1/3,
# alternating: wall / p50 / device ms per frame.  usage: tools/gpu_interactive_modes.sh <tag> [reps]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; out=gpurun_out/$1; mkdir -p $out
for i in $(seq 1 ${2:-2}); do for wh in "640 360" "800 600" "1280 720" "1920 1080"; do set -- $wh; for m in 0 1 3; do
  timeout -k 10 120 simple-path-tracer_amd/sptr_cli --scene default --w $1 --h $2 --spp 400 --warmup 20 --launch-mode $m --json --out /dev/null > $out/im_${1}_${m}_$i.json 2>$out/im_${1}_${m}_$i.err
  python3 -c "import json;d=json.loads(open('$out/im_${1}_${m}_$i.json').read().splitlines()[-1]);print('$1x$2 mode $m', 'wall', d['ms_per_frame_wall'], 'p50', d['ms_per_frame_p50'], 'dev', d['ms_per_frame_device'])"
done; done; done
