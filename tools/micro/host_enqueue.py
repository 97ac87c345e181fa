"""Host time of one asynchronous render call (the library's enqueue of its launches) against the device
time of the call, for the C2 workload: the whole frame (two pixel lanes) and the 8-way shard (one chain).
  usage: python tools/micro/host_enqueue.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simple-path-tracer_amd"))
import sptr  # noqa: E402
import workloads  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
r = sptr.Renderer(0)
wl = workloads.WORKLOADS["c2"]
workloads.setup(r, wl)
cam = workloads.camera(wl)
stream = torch.cuda.current_stream().cuda_stream
for shards in (1, 8):
    def call():
        r.render(cam, wl.width, wl.height, spp=wl.spp, max_depth=wl.max_depth, shard_rank=0, shard_count=shards,
                 flags=sptr.SPTR_FRAME_RECULL | sptr.SPTR_FRAME_ASYNC, stream=stream)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    r.collect_stats()
    host = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        call()
        host.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    r.collect_stats()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        call()
    e1.record()
    torch.cuda.synchronize()
    r.collect_stats()
    host.sort()
    print(f"shards {shards}: host enqueue ms per call min {host[0]:.3f} median {host[10]:.3f} max {host[-1]:.3f}; "
          f"device ms per call {e0.elapsed_time(e1) / 20:.3f}", flush=True)
