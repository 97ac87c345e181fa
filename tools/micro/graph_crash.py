"""Reproduction of the r06 host crash inside hipGraphLaunch (torch's HIP runtime): a two-lane call shape
captured and replayed in launch mode 3 (each lane context captures on the shared capture stream), then a
one-chain shape captured in launch mode 0 and replayed on a torch stream.  Prints "ok" when it survives.

    python tools/micro/graph_crash.py [--no-lanes-first] [--lib-stream]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simple-path-tracer_amd"))
import sptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--no-lanes-first", action="store_true")
ap.add_argument("--golden", action="store_true", help="the golden tests' calls in between")
ap.add_argument("--lib-stream", action="store_true", help="replay on the library's stream instead of a torch one")
a = ap.parse_args()
r = sptr.Renderer(0)
if not a.no_lanes_first:
    W, H = 3840, 2160
    sptr.setup_default(r, "default")
    cam = sptr.camera_lookat(aspect=W / H)
    r.set_wave_paths(1 << 25)
    r.set_launch_mode(3)
    for _ in range(3):
        r.render(cam, W, H, spp=16, flags=sptr.SPTR_FRAME_RECULL)
    r.set_launch_mode(0)
    r.set_wave_paths(0)
    print("lanes captured:", r.graph_info(), flush=True)
W, H = 1920, 1080
sptr.setup_default(r, "default_emitter")
cam = sptr.camera_lookat(aspect=W / H)
s = torch.cuda.Stream()
if a.golden:  # the calls test_gpu_golden.py makes before the crashing one
    r.render(cam, W, H, spp=64)
    for g in range(8):
        r.render(cam, W, H, spp=64, shard_rank=g, shard_count=8)
    sptr.setup_default(r, "default_emitter")
    for i in range(3):
        r.render(cam, W, H, spp=64, flags=sptr.SPTR_FRAME_RECULL | sptr.SPTR_FRAME_ASYNC, stream=s.cuda_stream)
        r.tiles_device()
    r.collect_stats()
    print("two lanes on the torch stream", r.graph_info(), flush=True)
    sptr.setup_default(r, "default_emitter")
r.set_pixel_lanes(1)
for i in range(3):
    r.render(cam, W, H, spp=64, flags=sptr.SPTR_FRAME_RECULL | sptr.SPTR_FRAME_ASYNC,
             stream=None if a.lib_stream else s.cuda_stream)
    print("call", i, r.graph_info(), flush=True)
r.collect_stats()
print("ok", flush=True)
r.close()
