cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05h
timeout -k 10 600 python3 -c "
import sys, json; sys.argv=['x']; sys.path.insert(0,'.')
import bench
for r in bench.interactive(200): print(json.dumps(r))
" > gpurun_out/r05h/inter.txt 2>&1; cat gpurun_out/r05h/inter.txt
