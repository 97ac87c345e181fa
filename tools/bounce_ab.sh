set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/variant_ab.sh ab15 c2 tree b4 b6 b7
o=gpurun_out/ab15; mkdir -p $o
for v in tree b6; do
  lib=$GRAFT_REPO_ROOT/variants/$v/libsptr_hip.so; [ "$v" = tree ] && lib=$GRAFT_REPO_ROOT/simple-path-tracer_amd/libsptr_hip.so
  SPTR_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-interactive --emulate-shards 8 > $o/s8_$v.json 2>$o/s8_$v.err
  python3 -c "import json;d=json.loads(open('$o/s8_$v.json').read().splitlines()[-1]);print('G8 $v',d['ms_per_step'])"
done
SPTR_NO_BOUNCE=1 SPTR_LIB=$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-interactive > $o/nb.json 2>$o/nb.err
python3 -c "import json;d=json.loads(open('$o/nb.json').read().splitlines()[-1]);print('G1 knobs no-bounce',d['ms_per_step'])"
SPTR_LIB=$GRAFT_REPO_ROOT/variants/knobs/libsptr_hip.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-interactive > $o/kb.json 2>$o/kb.err
python3 -c "import json;d=json.loads(open('$o/kb.json').read().splitlines()[-1]);print('G1 knobs bounce',d['ms_per_step'])"
