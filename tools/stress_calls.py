#!/usr/bin/env python3
"""Many direct-launch render calls in one process (cross-stream fork/join dependencies per call):
the runtime must not accumulate state across calls.   usage: tools/stress_calls.py N [launch_mode]"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "simple-path-tracer_amd"))
import sptr  # noqa: E402

n = int(sys.argv[1])
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 1
r = sptr.Renderer(0)
sptr.setup_default(r, "sphere_mesh", 60, 120)
r.set_launch_mode(mode)
W, H = 96, 64
cam = sptr.camera_lookat(aspect=W / H)
for i in range(n):
    r.render(cam, W, H, spp=4, frame_begin=1)
    if i % 500 == 0:
        print("call", i, flush=True)
print("done", n, flush=True)
