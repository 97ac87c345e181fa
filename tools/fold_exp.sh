set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SPTR_LIB=$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so
o=gpurun_out/fold; mkdir -p $o
for cfg in "c4 4" "c4 2" "c4 1" "c2 1" "c2 2"; do set -- $cfg
  for m in 1 2; do
    SPTR_FOLD=$m timeout -k 10 200 python3 bench.py --workload $1 --emulate-shards $2 --steps 4 --warmup 1 --no-cpu-baseline --no-interactive --stage-timing > $o/$1_$2_$m.json 2>$o/$1_$2_$m.err
    python3 -c "import json;d=json.loads(open('$o/$1_$2_$m.json').read().splitlines()[-1]);print('$1 G=$2 fold=$m',d['ms_per_step'],d['stage_ms_per_step'])"
  done
done
