#!/usr/bin/env python3
"""Benchmark: Mrays/s (+ Msamples/s) of the MI355X wavefront path tracer.

Default workload = BASELINE.json configs[1] (C2): default scene + emissive sphere (diffuse, metal,
dielectric and emissive materials), 1920x1080, 64 spp, max depth 6, procedural sky, one sun.
Inputs are synthetic (the reference's own procedural scene; no datasets).  --workload c1|c3|c4|c5
selects the other configurations (simple-path-tracer_amd/workloads.py); c5 is the HBM roofline run.

One "step" = one complete render of the frame at the workload's spp: every rank renders its
interleaved 32x32 tiles (the reference's tile schedule, src/GLRenderer.cpp:335-350) and resolves
them; the resolved RGBA8 tiles are gathered to rank 0 over RCCL and rank 0 unpacks them into the W x H
RGB8 image.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

`--gpus N` without a torch.distributed environment launches the N ranks itself: a child
`torch.distributed.run` of a fresh interpreter, started before this process touches the GPU (this
process only waits for it and exits with its code).  `--dry-run` runs the same rank launch, tile
schedule, gather and unpack on the CPU over gloo with a synthetic per-pixel pattern instead of
the renderer (a check of the multi-rank plumbing that needs no GPU).

value = all ranks' rays (closest-hit + any-hit queries, = the reference's rtcIntersect1 +
rtcOccluded1 calls) / max-over-ranks wall time of the K timed steps.  Work per rank shrinks as N
grows (fixed frame), so scaling is "strong".
"""
import argparse
import glob
import json
import math
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "simple-path-tracer_amd"))
import sptr  # noqa: E402
import workloads  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# VALU issue peak: a wave issues one VALU instruction per 2 cycles on its SIMD (MI355X_MICROARCH.md),
# 256 CUs x 4 SIMDs x 0.5 x 2.4 GHz = 1.2288e12 wave-instructions/s
VALU_PEAK_WAVE_INSTR_PER_S = 256 * 4 * 0.5 * 2.4e9
# SURVEY.md §8(d) ray stream: path id 4 + origin 12 + dir 12 read, t 4 + prim 4 written.  A primary
# ray reads nothing (raygen is fused into the bounce-0 trace), so it is charged the 8 B it writes.
STREAM_READ_BYTES, STREAM_WRITE_BYTES = 28.0, 8.0
L2_BYTES_PER_XCD = 4 << 20  # MI355X: 4 MB L2 per XCD (MI355X_MICROARCH.md)
XCDS = 8
CPU_SAMPLE_SPP = {"c1": 4, "c2": 64, "c3": 128, "c4": 64, "c5": 64}  # ~1-4 s per run on 16 host threads
# experiment knobs of the library and the build (timing studies only); a bench line records any that
# is set, so a stray variable cannot silently change a measured number
KNOB_VARS = ("SPTR_LIB", "SPTR_ABLATE", "SPTR_MAX_BLOCKS_PER_CU")


class _DevArray:
    """Zero-copy torch view of a device buffer owned by libsptr_hip."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes // 4,), "typestr": "<i4", "data": (ptr, False),
                                         "version": 3}


def _latest_profile(pattern):
    """The newest committed counter summary: by its "collected" UTC time (tools/prof_summary.py
    --emit); files from before that field count as older, and among themselves go by name."""
    best = None
    for path in glob.glob(os.path.join(ROOT, "profiles", pattern)):
        with open(path) as f:
            data = json.load(f)
        key = (data.get("collected", ""), os.path.basename(path))
        if best is None or key > best[0]:
            best = (key, data, path)
    if best is None:
        return None, None
    return best[1], os.path.relpath(best[2], ROOT)


def roofline(cnt, stats, layout, wl_name, steps, samples):
    """Roofline of the dominant kernel, k_trace (all bounces; one template).

    Algorithmic bytes per ray, SURVEY.md §8(d): B_ray = 36 + 64 n_node + 48 n_tri + 16 n_sph with the
    visit counts taken from an instrumented pass over the same rays; primary rays (raygen fused, no
    input stream) are charged their 8 written bytes only.  Which of the node/primitive bytes are HBM
    bytes depends on where the scene lives:
      lds  scene staged in LDS (lds_bytes > 0): node/primitive fetches never leave the CU;
      l2   scene fits one XCD's 4 MB L2: one scene copy per XCD per launch (counting every visit as
           HBM bytes would report more than the peak on C3);
      hbm  larger scenes (C5, 1.1 GB > the 256 MB MALL): every visit counts, as in §8(d).
    Beside the modelled fraction: counter_frac = FETCH_SIZE x2 + WRITE_SIZE per launch (the latest
    profiles/r*_pmc_<wl>_trace.json) over the live launch time, and valu_issue_frac = SQ_INSTS_VALU per
    launch (profiles/r*_sq_<wl>_trace.json) over the live launch time and the 1.23e12/s issue peak."""
    launches = sum(s.trace_launches for s in stats)
    avg_launch_s = sum(s.ms_trace for s in stats) / max(1, launches) * 1e-3
    launches_per_step = max(1, launches // max(1, steps))
    traced = cnt.rays_closest - cnt.rays_tail  # closest-hit queries of k_trace (the rest run in k_tail)
    primary = min(traced, samples)  # one primary ray per pixel sample, all traced by k_trace
    stream = (STREAM_READ_BYTES + STREAM_WRITE_BYTES) * (traced - primary) + STREAM_WRITE_BYTES * primary
    node_b = layout["node_bytes"] / max(1, layout["num_nodes"]) if layout["num_nodes"] else 64.0
    scene = node_b * cnt.node_visits + 48.0 * cnt.tri_tests + 16.0 * cnt.sphere_tests
    lds = layout["lds_bytes"] > 0
    footprint = sum(layout[k] for k in ("node_bytes", "tri_bytes", "sphere_bytes", "prim_ref_bytes"))
    residency = "lds" if lds else ("l2" if footprint <= L2_BYTES_PER_XCD else "hbm")
    hbm_alg = stream + {"lds": 0.0, "l2": XCDS * footprint * launches_per_step, "hbm": scene}[residency]
    per_launch = hbm_alg / launches_per_step
    achieved = per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    pmc, pmc_src = _latest_profile(f"r*_pmc_{wl_name}_trace.json")
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    sq, sq_src = _latest_profile(f"r*_sq_{wl_name}_trace.json")
    valu = sq.get("valu_per_launch") if sq else None
    out = {"bound": "hbm", "kernel": "k_trace", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": pmc_src,
           "counter_frac": round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 4) if traffic and avg_launch_s else None,
           "valu_issue_frac": round(valu / avg_launch_s / VALU_PEAK_WAVE_INSTR_PER_S, 4) if valu and avg_launch_s else None,
           "valu_source": sq_src,
           "bytes_per_launch": round(per_launch), "avg_launch_us": round(avg_launch_s * 1e6, 2),
           "launches_per_step": launches_per_step,
           "scene_in_lds": lds, "scene_residency": residency, "scene_bytes": int(footprint),
           "b_ray_full_gbs": round((stream + scene) / launches_per_step / avg_launch_s / 1e9, 1) if avg_launch_s else 0,
           "per_ray": {"nodes": round(cnt.node_visits / max(1, traced), 3),
                       "tris": round(cnt.tri_tests / max(1, traced), 3),
                       "spheres": round(cnt.sphere_tests / max(1, traced), 3)}}
    fr = {"hbm_model": out["frac"], "hbm_counters": out["counter_frac"], "valu_issue": out["valu_issue_frac"]}
    known = {k: v for k, v in fr.items() if v is not None}
    out["binding"] = max(known, key=known.get) if known else None
    return out


def host_cpus():
    """What this process may use: hardware threads, the affinity mask, the cgroup CPU quota."""
    hw = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = hw
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = max(1, math.ceil(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    granted = min(aff, quota) if quota else aff
    return {"hardware_concurrency": hw, "affinity": aff, "cgroup_quota_cpus": quota, "granted": granted,
            "model": model}


def cpu_baseline(wl, flat, cam):
    """The oracle (C++ restatement of the reference's CPU wavefront integrator, Embree semantics with
    its own binned-SAH BVH) on the host cores, on the same scene and camera: a reported baseline.
    Two runs: every CPU this process is granted, and one fewer (the reference's TBB policy,
    src/main.cpp:127-135)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure, used here only as the timed CPU baseline

    cpus = host_cpus()
    spp = min(wl.spp, CPU_SAMPLE_SPP.get(wl.name, 1))
    scene = {k: getattr(flat, k) for k in ("positions", "indices", "tri_geom_first", "spheres", "geom_material")}
    t0 = time.perf_counter()
    P = oracle.Prepared(scene, bvh=True)
    t_build = time.perf_counter() - t0
    faces = workloads.hdr_env_faces() if wl.hdr_env else None
    mats = oracle.preset_materials(wl.scene == "default_emitter")

    def run(threads):
        t0 = time.perf_counter()
        _, _, cnt = P.render(cam.as_array(), wl.width, wl.height, mats, oracle.default_lights(), frames=spp,
                             max_depth=wl.max_depth, threads=threads, env_faces=faces)
        dt = time.perf_counter() - t0
        rays = cnt["rays_closest"] + cnt["rays_shadow"]
        return rays, cnt["samples"], dt

    n_all = cpus["granted"]
    rays, samples, dt = run(n_all)
    res = {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": n_all, "kind": "port",
           "sample": f"{wl.width}x{wl.height} x {spp} spp of {wl.spp} ({'full workload' if spp == wl.spp else 'first spp'})"
                     f", {rays} rays in {dt:.2f} s (+{t_build:.2f} s BVH build); oracle/wf_oracle.cpp with a"
                     f" binned-SAH BVH, std::thread over 32x32 tiles with a dynamic tile counter",
           "msamples_per_s": round(samples / dt / 1e6, 3), "cpu": cpus}
    if n_all > 1:
        r1, s1, d1 = run(n_all - 1)
        res["cores_minus_1"] = {"cores": n_all - 1, "value": round(r1 / d1 / 1e6, 3),
                                "msamples_per_s": round(s1 / d1 / 1e6, 3),
                                "policy": "reference TBB policy: hardware_concurrency - 1 (src/main.cpp:127-135)"}
    return res


def interactive(steps):
    """The reference's own usage: 1 spp per render() call, progressive accumulation, RGB8 read back
    every frame, as GLRenderer::renderLoop drives a backend (src/GLRenderer.cpp:161-176).  Runs the C++
    harness (backends::HipBackend through the C ABI) as a child process."""
    cli = os.path.join(ROOT, "simple-path-tracer_amd", "sptr_cli")
    out = []
    for w, h in ((800, 600), (1920, 1080)):
        r = subprocess.run([cli, "--scene", "default", "--w", str(w), "--h", str(h), "--spp", str(steps),
                            "--warmup", "10", "--json", "--out", "/dev/null"], capture_output=True, text=True,
                           timeout=300)
        if r.returncode != 0:
            raise RuntimeError(f"sptr_cli failed: {r.stderr[-2000:]}")
        out.append(json.loads(r.stdout.strip().splitlines()[-1]))
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """One process per GPU: run this script under torch.distributed.run in a child process (this
    process has not touched the GPU and never does; it waits and returns the child's exit code)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def gather_tiles(send, gathered, world, rank):
    """Rank 0 collects every rank's resolved tiles (dist.gather: one point-to-point transfer per
    rank to rank 0).  On the fully connected xGMI mesh of an 8-GPU node the 7 transfers use 7
    different links at once; a ring all-gather would move the frame over one link per step, N-1
    steps in a row, and hand every rank a whole frame that only rank 0 uses."""
    dist.gather(send, list(gathered.chunk(world)) if rank == 0 else None, dst=0)


def dry_run(args, wl, world, rank):
    """CPU plumbing check of the multi-rank step (gloo): each rank packs its interleaved tiles of a
    synthetic per-pixel pattern with the product's host tile packing (the twin of the device
    resolve's tile layout), one gather to rank 0, which unpacks and compares with the whole pattern."""
    import numpy as np

    W, H = wl.width, wl.height
    yy, xx = np.mgrid[0:H, 0:W].astype(np.uint32)
    pattern = np.stack([(xx * 7 + yy) & 255, (xx ^ yy) & 255, (xx * 13 + yy * 5) & 255], -1).astype(np.uint8)
    tiles = sptr.pack_tiles(pattern, world, rank)
    gathered = torch.zeros(world * tiles.size, dtype=torch.int32)
    gather_tiles(torch.from_numpy(tiles.view(np.int32)), gathered, world, rank)
    mine = torch.tensor([float(((tiles >> 24) == 255).sum())], dtype=torch.float64)  # pixels inside the image
    dist.all_reduce(mine)
    if rank == 0:
        img = sptr.unpack_tiles(gathered.numpy().view(np.uint32), world, W, H)
        ok = bool(np.array_equal(img, pattern)) and int(mine.item()) == W * H
        print(json.dumps({"dry_run": True, "n_gpus": world, "world_size": dist.get_world_size(),
                          "backend": dist.get_backend(), "workload": wl.name, "tiles_per_rank": int(tiles.size // 1024),
                          "pixels_covered": int(mine.item()), "gather_ok": ok}), flush=True)
        if not ok:
            sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c2", choices=sorted(workloads.WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-interactive", action="store_true", help="skip the 1-spp progressive-frame leg")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo check of the rank launch + tile gather")
    ap.add_argument("--wave-paths", type=int, default=0)
    ap.add_argument("--leaf-size", type=int, default=0)
    ap.add_argument("--bvh-width", type=int, default=0, choices=[0, 2, 4])
    ap.add_argument("--tail-depth", type=int, default=0, help="first bounce traced path-per-thread (0 = library default)")
    ap.add_argument("--emulate-shards", type=int, default=0,
                    help="timing experiment on one GPU: render only shard 0 of G (the per-rank work of a G-GPU run); "
                         "the line is marked emulated and is not a G-GPU measurement")
    ap.add_argument("--integrator", default="wavefront", choices=["wavefront", "pathtracer"],
                    help="pathtracer: the reference's default CPU integrator semantics (PathTracer.cpp), "
                         "4 samples per frame; the headline metric is the wavefront integrator's")
    ap.add_argument("--stage-timing", action="store_true",
                    help="HIP events around every stage (default: around the k_trace launches only, which the "
                         "roofline needs; events between the other stages would add dispatch gaps)")
    args = ap.parse_args()
    wl = workloads.WORKLOADS[args.workload]
    W, H = wl.width, wl.height

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    distributed = world > 1
    if distributed and args.emulate_shards:
        print("bench.py: --emulate-shards is a one-GPU timing experiment; not allowed with several ranks",
              file=sys.stderr)
        sys.exit(2)

    if args.dry_run:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dry_run(args, wl, world, rank)
        dist.destroy_process_group()
        return

    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    dev = torch.device("cuda", local)

    r = sptr.Renderer(local)
    if args.wave_paths:
        r.set_wave_paths(args.wave_paths)
    if args.leaf_size:
        r.set_leaf_size(args.leaf_size)
    if args.bvh_width:
        r.set_bvh_width(args.bvh_width)
    if args.tail_depth:
        r.set_tail_depth(args.tail_depth)
    flat = workloads.setup(r, wl)
    layout, info = r.scene_layout(), r.scene_info()
    cam = workloads.camera(wl)
    shards = args.emulate_shards if args.emulate_shards else world
    shard = 0 if args.emulate_shards else rank
    tiles_per_rank = sptr.tiles_per_rank(W, H, shards)
    send = torch.zeros(tiles_per_rank * 1024, dtype=torch.int32, device=dev)
    gathered = torch.zeros(shards * tiles_per_rank * 1024, dtype=torch.int32, device=dev)
    image = torch.zeros(W * H * 3, dtype=torch.uint8, device=dev)

    # a real stream (torch's default is the legacy null stream, which the library's non-blocking
    # streams do not order against): render, copy, gather and unpack all run on it
    torch_stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(torch_stream)
    stream = torch_stream.cuda_stream

    integ = sptr.SPTR_INTEGRATOR_PATHTRACER if args.integrator == "pathtracer" else sptr.SPTR_INTEGRATOR_WAVEFRONT
    # PathTracer mode: a frame is 4 samples (setupPathTracer), so spp/4 frames give the same samples
    frames = max(1, wl.spp // 4) if args.integrator == "pathtracer" else wl.spp

    def step(flags=0):
        # every stage of a step is enqueued on torch's current stream, with no host synchronisation:
        # render (SPTR_FRAME_ASYNC) -> tile copy -> RCCL gather to rank 0 -> rank-0 unpack
        r.render(cam, W, H, spp=frames, max_depth=wl.max_depth, shard_rank=shard, shard_count=shards,
                 flags=flags | sptr.SPTR_FRAME_ASYNC, stream=stream, integrator=integ, samples_per_frame=4)
        ptr, nbytes = r.tiles_device()
        local_tiles = torch.as_tensor(_DevArray(ptr, nbytes), device=dev)
        send[: local_tiles.numel()].copy_(local_tiles)
        if distributed:
            gather_tiles(send, gathered, world, rank)
        else:
            gathered[: send.numel()].copy_(send)
        if rank == 0:
            r.unpack_tiles(gathered.data_ptr(), shards, tiles_per_rank, W, H, image.data_ptr(), stream=stream)

    for _ in range(args.warmup):
        step()
    r.collect_stats()
    # untimed instrumented pass: BVH node / primitive fetch counts for the algorithmic-bytes model
    step(sptr.SPTR_FRAME_COUNT_VISITS)
    cnt = r.collect_stats()
    # the timed call shape (its event flag differs from the warmup's) seen twice before timing: the
    # library captures a repeated shape into a launch graph on its second call, so the capture
    # happens here and every timed step replays it, as repeated renders of one frame do
    timing = sptr.SPTR_FRAME_TIMING if args.stage_timing else sptr.SPTR_FRAME_TIMING_TRACE
    for _ in range(2):
        step(timing)
    r.collect_stats()

    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timing)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = [r.collect_stats()]  # the K timed steps' counters and stage events, summed

    rays = sum(s.rays_closest + s.rays_shadow for s in stats)
    samples = sum(s.samples for s in stats)
    t = torch.tensor([elapsed, float(rays), float(samples)], dtype=torch.float64, device=dev)
    if distributed:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, rays, samples = float(tmax[0]), float(tsum[1]), float(tsum[2])
        # the gathered frame is the same bytes a 1-GPU render gives (tests/test_gpu_parity.py shard union)
        want = W * H * (frames * 4 if args.integrator == "pathtracer" else wl.spp) * args.steps
        assert int(tsum[2]) == want, (int(tsum[2]), want)

    if rank == 0:
        stage_ms = {k: round(sum(getattr(s, "ms_" + k) for s in stats) / args.steps, 3)
                    for k in (("trace0", "trace", "shade0", "shade", "shadow", "tail", "accum") if args.stage_timing
                              else ("trace0", "trace"))}
        knobs = {k: os.environ[k] for k in KNOB_VARS if os.environ.get(k)}
        line = {
            "metric": "Mrays/sec + Msamples/sec, default scene 1920x1080, 1/2/4/8 MI355X",
            "value": round(rays / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "msamples_per_s": round(samples / elapsed / 1e6, 2),
            "n_gpus": dist.get_world_size() if distributed else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (the reference's procedural scenes; no datasets)",
            "config": {"workload": wl.description, "scene": os.path.basename(wl.scene), "width": W, "height": H,
                       "spp": wl.spp, "max_depth": wl.max_depth,
                       "parallelism": f"tile-sharded x{world} (interleaved 32x32 tiles) + RCCL gather to rank 0"},
            "integrator": args.integrator,
            "world_size": world,
            "collective": ("RCCL gather of the RGBA8 tiles to rank 0 (point-to-point over xGMI), once per step" if distributed
                           else "none (1 rank)"),
            "roofline": roofline(cnt, stats, layout, wl.name, args.steps, samples),
            "stage_ms_per_step": stage_ms,
            "tail_rays_per_step": int(sum(s.rays_tail for s in stats) / args.steps),
            "rays_per_step": int(rays / args.steps),
            "scene": {"prims": info["prims"], "lbvh_nodes": info["nodes"], "bvh_depth": info["depth"],
                      "lbvh_build_ms": round(info["build_ms"], 3), "leaf_size": layout["leaf_size"],
                      "bvh_width": layout["bvh_width"], "traversed_nodes": layout["num_nodes"]},
            "cpu_baseline": None,
        }
        if knobs:
            line["experiment_knobs"] = knobs
        if args.emulate_shards:
            line["emulated"] = f"shard 0 of {shards} on one GPU: per-rank work of a {shards}-GPU run (not a multi-GPU value)"
        if args.integrator == "pathtracer":
            line["note"] = ("PathTracer-mode throughput (the reference's default CPU integrator semantics, path per "
                            "thread); not the headline wavefront metric; roofline fields describe no k_trace launch")
        if world == 1 and not args.no_interactive and not args.emulate_shards and args.integrator == "wavefront":
            line["interactive"] = interactive(200)
        if world == 1 and not args.no_cpu_baseline and args.integrator == "wavefront":
            line["cpu_baseline"] = cpu_baseline(wl, flat, cam)
        print(json.dumps(line), flush=True)
    r.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
