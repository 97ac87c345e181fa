#!/usr/bin/env python3
"""Benchmark: Mrays/s (+ Msamples/s) of the MI355X wavefront path tracer on BASELINE config C2.

Workload (BASELINE.json configs[1]): default scene + emissive sphere (diffuse, metal, dielectric and
emissive materials), 1920x1080, 64 spp, max depth 6, procedural sky, one directional sun; inputs
synthetic (the reference's own procedural scene — no datasets).  One "step" = one complete 64-spp
render of the frame: every rank renders its interleaved 32x32 tiles, resolves them, and the
resolved RGBA8 tiles are all-gathered over RCCL and unpacked into the 1920x1080 RGB8 image.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU, RCCL backend)

value = all ranks' rays (closest-hit + any-hit queries) / max-over-ranks wall time of K steps.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "simple-path-tracer_amd"))
import sptr  # noqa: E402

W, H, SPP, DEPTH, SCENE = 1920, 1080, 64, 6, "default_emitter"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


class _DevArray:
    """Zero-copy torch view of a device buffer owned by libsptr_hip."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes // 4,), "typestr": "<i4", "data": (ptr, False),
                                         "version": 3}


def trace_bytes(st, rays):
    """B_ray = 28 (path id + origin + dir) + 8 (t + prim id) + 64*nodes + 48*tris + 16*spheres."""
    return 36.0 * rays + 64.0 * st.node_visits + 48.0 * st.tri_tests + 16.0 * st.sphere_tests


def cpu_baseline(cam):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure, used only as the timed CPU baseline

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    P = oracle.Prepared(oracle.builtin_scene(SCENE), bvh=True)
    t0 = time.perf_counter()
    _, _, cnt = P.render(cam.as_array(), W, H, oracle.preset_materials(True), oracle.default_lights(),
                         frames=SPP, max_depth=DEPTH, threads=threads)
    dt = time.perf_counter() - t0
    rays = cnt["rays_closest"] + cnt["rays_shadow"]
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"full workload: {W}x{H} x {SPP} spp, {rays} rays in {dt:.2f} s "
                      f"(oracle C++ restatement + median-split BVH, std::thread over 32x32 tiles)",
            "msamples_per_s": round(cnt["samples"] / dt / 1e6, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--wave-paths", type=int, default=0)
    ap.add_argument("--leaf-size", type=int, default=0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)

    r = sptr.Renderer(local)
    if args.wave_paths:
        r.set_wave_paths(args.wave_paths)
    if args.leaf_size:
        r.set_leaf_size(args.leaf_size)
    sptr.setup_default(r, SCENE)
    cam = sptr.camera_lookat(aspect=W / H)
    ntx, nty = (W + 31) // 32, (H + 31) // 32
    tiles_per_rank = (ntx * nty + world - 1) // world
    send = torch.zeros(tiles_per_rank * 1024, dtype=torch.int32, device=dev)
    gathered = torch.zeros(world * tiles_per_rank * 1024, dtype=torch.int32, device=dev)
    image = torch.zeros(W * H * 3, dtype=torch.uint8, device=dev)

    def step(flags=0):
        st = r.render(cam, W, H, spp=SPP, max_depth=DEPTH, shard_rank=rank, shard_count=world, flags=flags)
        ptr, nbytes = r.tiles_device()
        local_tiles = torch.as_tensor(_DevArray(ptr, nbytes), device=dev)
        send[: local_tiles.numel()].copy_(local_tiles)
        if distributed:
            dist.all_gather_into_tensor(gathered, send)
        else:
            gathered.copy_(send)
        if rank == 0:
            torch.cuda.current_stream().synchronize()
            r.unpack_tiles(gathered.data_ptr(), world, tiles_per_rank, W, H, image.data_ptr())
        return st

    for _ in range(args.warmup):
        step()
    # untimed instrumented pass: BVH node / primitive fetch counts for the algorithmic-bytes model
    cnt = step(sptr.SPTR_FRAME_COUNT_VISITS)

    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [step(sptr.SPTR_FRAME_TIMING) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    rays = sum(s.rays_closest + s.rays_shadow for s in stats)
    samples = sum(s.samples for s in stats)
    t = torch.tensor([elapsed, float(rays), float(samples)], dtype=torch.float64, device=dev)
    if distributed:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, rays, samples = float(tmax[0]), float(tsum[1]), float(tsum[2])

    if rank == 0:
        ms_trace = sum(s.ms_trace for s in stats)
        launches = sum(s.trace_launches for s in stats)
        stage_ms = {k: round(sum(getattr(s, "ms_" + k) for s in stats) / len(stats), 3)
                    for k in ("raygen", "trace", "shade", "shadow", "accum")}
        # per-launch algorithmic bytes of the trace kernel (counted pass scaled to the timed steps)
        bytes_step = trace_bytes(cnt, cnt.rays_closest)
        avg_launch_s = (ms_trace / launches) * 1e-3
        bytes_launch = bytes_step / max(1, cnt.trace_launches or (launches / len(stats)))
        achieved = bytes_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "trace_pmc_bytes.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        line = {
            "metric": "Mrays/sec + Msamples/sec, default scene 1920x1080, 1/2/4/8 MI355X",
            "value": round(rays / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "msamples_per_s": round(samples / elapsed / 1e6, 2),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference's procedural default scene + emissive sphere; no datasets)",
            "config": {"workload": f"C2: default scene + emitter, {W}x{H}, {SPP} spp, depth {DEPTH}",
                       "scene": SCENE, "width": W, "height": H, "spp": SPP, "max_depth": DEPTH,
                       "parallelism": f"tile-sharded x{world} (interleaved 32x32 tiles) + RCCL all-gather"},
            "roofline": {"bound": "hbm", "kernel": "k_trace", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "bytes_per_launch": round(bytes_launch), "avg_launch_us": round(avg_launch_s * 1e6, 2),
                         "note": "algorithmic bytes per SURVEY 8(d); BVH/prims of this scene are LDS-staged"},
            "stage_ms_per_step": stage_ms,
            "rays_per_step": int(rays / args.steps),
            "visits": {"node": cnt.node_visits, "tri": cnt.tri_tests, "sphere": cnt.sphere_tests,
                       "closest_rays": cnt.rays_closest},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cam)
        print(json.dumps(line), flush=True)
    r.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
