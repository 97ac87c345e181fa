"""The multi-GPU data path's collective on the real backend: bench.gather_tiles over RCCL ("nccl"),
one rank on cuda:0 (the GPU box has one GPU; the N-rank schedule itself is covered over gloo by
tests/test_distributed_cpu.py).  Runs in a child process so that the process group lives and dies
with it."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import importlib.util, os, socket, sys
import torch, torch.distributed as dist
with socket.socket() as s:
    s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
spec = importlib.util.spec_from_file_location("bench", os.path.join(sys.argv[1], "bench.py"))
bench = importlib.util.module_from_spec(spec); spec.loader.exec_module(bench)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
send = torch.arange(4096, dtype=torch.int32, device="cuda")
gathered = torch.zeros(4096, dtype=torch.int32, device="cuda")
bench.gather_tiles(send, gathered, 1, 0)
torch.cuda.synchronize()
ok = bool(torch.equal(gathered, send))
print("backend", dist.get_backend(), "gather_ok", ok)
dist.destroy_process_group()
sys.exit(0 if ok else 1)
"""


@pytest.mark.gpu
def test_rccl_gather_tiles_one_rank():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "gather_ok True" in r.stdout
