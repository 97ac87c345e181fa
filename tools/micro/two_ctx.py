"""Timing experiment: one rank's share of a frame (shard R of G) rendered as `lanes` interleaved
sub-shards (R + G*j of lanes*G) by as many contexts on one GPU concurrently (each with its own buffers
and streams), against one context rendering the whole share.  usage: two_ctx.py <wl> <G> <lanes...>"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "simple-path-tracer_amd"))
import sptr, workloads  # noqa: E402

wl = workloads.WORKLOADS[sys.argv[1]]
G = int(sys.argv[2])
lane_counts = [int(x) for x in sys.argv[3:]] or [2]
steps = int(os.environ.get("STEPS", "10"))
W, H = wl.width, wl.height
cam = workloads.camera(wl)
ctx = [sptr.Renderer(0) for _ in range(max(lane_counts))]
for r in ctx:
    workloads.setup(r, wl)
    r.set_launch_mode(int(os.environ.get("MODE", "1")))
F = sptr.SPTR_FRAME_ASYNC | sptr.SPTR_FRAME_RECULL


def go(lanes):
    for j in range(lanes):
        ctx[j].render(cam, W, H, spp=wl.spp, max_depth=wl.max_depth, shard_rank=j * G, shard_count=lanes * G, flags=F)


def run(lanes):
    for _ in range(2):
        go(lanes)
    for r in ctx:
        r.collect_stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        go(lanes)
    for r in ctx:
        r.collect_stats()
    return (time.perf_counter() - t0) / steps * 1e3


for rep in range(2):
    for lanes in [1] + lane_counts:
        print(wl.name, f"G={G}", f"lanes={lanes}", round(run(lanes), 3), "ms/step", flush=True)
