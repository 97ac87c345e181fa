"""Device time per call of the 8-way C2 shard (and the whole frame) with the cull recomputed in the call
(SPTR_FRAME_RECULL: k_frame_dyn -> k_cull -> chain) and with the cached mask (k_frame_dyn -> chain), on a
torch side stream; 200 calls each, alternating twice.
  usage: python tools/micro/head_cost.py"""
import os
import sys

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
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    stream = st.cuda_stream
    for shards, n in ((8, 200), (1, 40)):
        for rep in range(2):
            for name, fl in (("recull", sptr.SPTR_FRAME_RECULL), ("cached", 0)):
                def call():
                    r.render(cam, wl.width, wl.height, spp=wl.spp, max_depth=wl.max_depth, shard_rank=0, shard_count=shards,
                             flags=fl | sptr.SPTR_FRAME_ASYNC, stream=stream)
                for _ in range(5):
                    call()
                st.synchronize()
                r.collect_stats()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(n):
                    call()
                e1.record(st)
                st.synchronize()
                r.collect_stats()
                print(f"shards {shards} {name} rep {rep}: {e0.elapsed_time(e1) / n * 1e3:.1f} us per call", flush=True)
