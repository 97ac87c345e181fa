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
# LDS aggregate read bandwidth with every CU streaming ds_read_b64/b128 (MI355X_MICROARCH.md §LDS, ~150 TB/s):
# the roof §8(d)'s node/primitive bytes are priced against for scenes staged in LDS
LDS_PEAK_GBS = 150000.0
# VALU issue peak: a wave issues one VALU instruction per 2 cycles on its SIMD (MI355X_MICROARCH.md),
# 256 CUs x 4 SIMDs x 0.5 x 2.4 GHz = 1.2288e12 wave-instructions/s
VALU_PEAK_WAVE_INSTR_PER_S = 256 * 4 * 0.5 * 2.4e9
# SURVEY.md §8(d) ray stream: path id 4 + origin 12 + dir 12 read, t 4 + prim 4 written (frac_s8d)
STREAM_READ_BYTES, STREAM_WRITE_BYTES = 28.0, 8.0
# the product's streams: hit record {t, prim} + slot/path id, ray origin + direction
# (two float4), throughput and radiance float4, four cubemap texels per environment lookup
HIT_RECORD_BYTES, RAY_READ_BYTES, THR_READ_BYTES, RAD_BYTES, ENV_TEXEL_BYTES = 12.0, 32.0, 16.0, 16.0, 64.0
L2_BYTES_PER_XCD = 4 << 20  # MI355X: 4 MB L2 per XCD (MI355X_MICROARCH.md)
XCDS = 8
CPU_SAMPLE_SPP = {"c1": 4, "c2": 64, "c3": 128, "c4": 64, "c5": 64}  # ~1-4 s per run on 16 host threads
# experiment knobs of the library and the build (timing studies only); a bench line records any that
# is set, so a stray variable cannot silently change a measured number
KNOB_VARS = ("SPTR_LIB", "SPTR_ABLATE", "SPTR_MAX_BLOCKS_PER_CU", "SPTR_OVERLAP", "SPTR_FUSE_FROM", "SPTR_SKY_BLOCKS",
             "SPTR_FOLD", "SPTR_NO_FUSE", "SPTR_NO_DYN", "SPTR_DYN_LDS", "SPTR_NO_BOUNCE")


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


def _residency(layout):
    footprint = sum(layout[k] for k in ("node_bytes", "tri_bytes", "sphere_bytes", "prim_ref_bytes"))
    res = "lds" if layout["lds_bytes"] > 0 else ("l2" if footprint <= L2_BYTES_PER_XCD else "hbm")
    return res, footprint


def _counter_fracs(wl_name, kernel, avg_launch_s, stream_read_per_launch):
    """counter_frac = HBM bytes per launch from FETCH_SIZE / WRITE_SIZE (the newest
    profiles/r*_pmc_<wl>_<kernel>.json) over the live launch time, with FETCH_SIZE calibrated per access
    shape (tools/micro/gather_cal.hip, profiles/r03b_fetch_calibration.json): a coalesced 16-B-per-lane
    stream is counted at half its bytes, a random 48/64-B gather (BVH nodes, triangles) at its bytes.  So
    traffic = FETCH_SIZE + (the launch's coalesced stream reads, from the model) / 2 + WRITE_SIZE;
    traffic_x2 (FETCH_SIZE doubled, the stream-only calibration of MI355X_MICROARCH.md) beside it.
    valu_issue_frac = SQ_INSTS_VALU per launch (profiles/r*_sq_<wl>_<kernel>.json) over the live launch
    time and the 1.23e12/s issue peak; salu_per_valu from the same SQ pass."""
    pmc, pmc_src = _latest_profile(f"r*_pmc_{wl_name}_{kernel}.json")
    traffic_x2 = pmc.get("hbm_bytes_per_launch") if pmc else None
    traffic = None
    if pmc and pmc.get("fetch_bytes_per_launch_x2") is not None:
        traffic = pmc["fetch_bytes_per_launch_x2"] / 2.0 + stream_read_per_launch / 2.0 + pmc["write_bytes_per_launch"]
    sq, sq_src = _latest_profile(f"r*_sq_{wl_name}_{kernel}.json")
    valu = sq.get("valu_per_launch") if sq else None
    salu = sq.get("counters_per_launch", {}).get("SQ_INSTS_SALU") if sq else None
    return {"traffic": traffic, "traffic_x2": traffic_x2, "traffic_source": pmc_src,
            "counter_frac": round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 4) if traffic and avg_launch_s else None,
            "valu_issue_frac": round(valu / avg_launch_s / VALU_PEAK_WAVE_INSTR_PER_S, 4) if valu and avg_launch_s else None,
            "salu_per_valu": round(salu / valu, 3) if salu and valu else None, "valu_source": sq_src}


def env_hbm_bytes(lookups, env_bytes, launches):
    """HBM bytes of cubemap lookups (4 texels, ENV_TEXEL_BYTES each): the faces (6 x size^2 float4, 25 MB
    at 512^2) stay in the 256 MB MALL, so a launch reads them from HBM at most once per XCD, as an
    L2-resident scene (_residency)."""
    return min(ENV_TEXEL_BYTES * lookups, XCDS * env_bytes * launches) if env_bytes else 0.0


def roofline(cnt, stats, layout, wl_name, steps, env_bytes=0):
    """Roofline of the dominant kernel, k_trace (all its launches: bounce 0 and the wavefront bounces
    before the path-per-thread tail; one template), with the fused bounce launches
    (k_bounce: the trace and the shading of a bounce in one launch, LDS scenes in batches of at most
    2^26 paths — the pixel lanes' chains and the sharded frames) counted as trace launches: they are the
    same traversal, and in those chains they hold most of the traversal time.

    cnt: the stats of one instrumented (SPTR_FRAME_COUNT_VISITS) step, used only for per-ray ratios (BVH
    visits, hit fraction); stats: the K timed steps (launch times, launch counts and the rays the trace
    launches traversed, all summed over the K steps), so every per-launch figure below is a ratio of
    two sums over the same launches and does not depend on K.

    Rays are those the trace launches actually traverse (the library's traced_primary / traced_bounce):
    camera rays of frustum-culled pixels are answered without a traversal and are not charged.
    Algorithmic HBM bytes per traversed ray: a camera ray reads nothing (raygen is fused)
    and writes a 12-B hit record (t, prim, path id) on a hit or its 16-B radiance on a miss; a later
    ray reads its 32-B origin/direction, writes a 12-B hit record on a hit or, on a miss, reads its
    throughput and read-modify-writes its radiance (48 B); a miss in a cubemap environment also reads 4
    texels (64 B).  Node/primitive bytes (64 n_node + 48 n_tri + 16 n_sph per ray, the visit counts of
    the instrumented pass) count as HBM bytes according to where the scene lives:
      lds  scene staged in LDS (lds_bytes > 0): node/primitive fetches never leave the CU;
      l2   scene fits one XCD's 4 MB L2: one scene copy per XCD per launch;
      hbm  larger scenes (C5, 1.1 GB > the 256 MB MALL): every visit counts, as in SURVEY.md §8(d).
    s8d: §8(d) taken literally (36 B per traversed ray and every visit charged, whatever the residency),
    priced against the roof those bytes actually stream from: HBM for l2/hbm scenes (frac_s8d), the LDS
    aggregate read bandwidth for LDS-staged scenes (s8d_lds_frac; no HBM fraction is given for them, since
    their node/primitive reads never reach HBM).
    Beside them: counter_frac / valu_issue_frac / salu_per_valu from the session's rocprofv3 passes."""
    launches = sum(s.trace_launches for s in stats)
    avg_launch_s = sum(s.ms_trace for s in stats) / max(1, launches) * 1e-3
    # the launches' busy time (union of their intervals): two pixel lanes' trace launches overlap, so each
    # launch's own duration includes the time it shares with the other lane's; the achieved rate divides
    # the bytes by the busy time (one chain: busy = the sum of the durations, the same figure)
    busy_s = sum(getattr(s, "ms_trace_busy", 0.0) for s in stats) * 1e-3
    eff_launch_s = busy_s / max(1, launches) if busy_s > 0 else avg_launch_s
    tp = sum(s.traced_primary for s in stats)
    tb = sum(s.traced_bounce for s in stats)
    tf = sum(getattr(s, "traced_fused", 0) for s in stats)  # bounce rays of k_bounce
    # visits and hit fractions per traversed ray, bounce 0 and later bounces (instrumented step)
    vp = [cnt.node_visits_primary, cnt.tri_tests_primary, cnt.sphere_tests_primary]
    vb = [cnt.node_visits - vp[0], cnt.tri_tests - vp[1], cnt.sphere_tests - vp[2]]
    pp = [v / max(1, cnt.traced_primary) for v in vp]
    pb = [v / max(1, cnt.traced_bounce) for v in vb]
    hp = getattr(cnt, "hits_primary", 0) / max(1, cnt.traced_primary)
    hb = getattr(cnt, "hits_bounce", 0) / max(1, cnt.traced_bounce)
    node_b = layout["node_bytes"] / max(1, layout["num_nodes"]) if layout["num_nodes"] else 64.0
    scene_p = node_b * pp[0] + 48.0 * pp[1] + 16.0 * pp[2]
    scene_b = node_b * pb[0] + 48.0 * pb[1] + 16.0 * pb[2]
    stream = (tp * (hp * HIT_RECORD_BYTES + (1.0 - hp) * RAD_BYTES)
              + tb * (RAY_READ_BYTES + hb * HIT_RECORD_BYTES + (1.0 - hb) * (THR_READ_BYTES + 2 * RAD_BYTES)))
    # fused bounce rays (k_bounce): the visit-count pass runs them as separate trace launches, so its
    # bounce hit fraction and visits per ray apply to them
    stream += tf * (hb * FUSED_HIT_BYTES + (1.0 - hb) * FUSED_MISS_BYTES)
    # the fused bounce-1 rays of k_bounce01 (LDS scenes: every fused chain starts with it) read a 12-B
    # bounce-0 hit record instead of a 48-B ray + throughput
    residency, footprint = _residency(layout)
    t01 = sum(list(getattr(s, "traced_by_depth", [0, 0]))[1] for s in stats) if residency == "lds" and tf else 0
    stream -= t01 * (RAY_READ_BYTES + THR_READ_BYTES - HIT_RECORD_BYTES)
    stream += env_hbm_bytes(tp * (1.0 - hp) + (tb + tf) * (1.0 - hb), env_bytes, launches)
    stream_read = (tb * (RAY_READ_BYTES + (1.0 - hb) * (THR_READ_BYTES + RAD_BYTES))
                   + tf * (RAY_READ_BYTES + THR_READ_BYTES + RAD_BYTES)
                   - t01 * (RAY_READ_BYTES + THR_READ_BYTES - HIT_RECORD_BYTES))  # coalesced reads
    scene = {"lds": 0.0, "l2": XCDS * footprint * launches, "hbm": scene_p * tp + scene_b * (tb + tf)}[residency]
    # straggler hand-off (hbm scenes): the rest of a handed-off ray's walk runs in k_strag, not in the
    # trace launch; its visits (counted in every call) are not the trace launch's bytes
    sv = [sum(list(getattr(s, "strag_visits", (0, 0, 0)))[i] for s in stats) for i in range(3)]
    strag_bytes = node_b * sv[0] + 48.0 * sv[1] + 16.0 * sv[2] if residency == "hbm" else 0.0
    scene -= strag_bytes
    per_launch = (stream + scene) / max(1, launches)
    achieved = per_launch / eff_launch_s / 1e9 if eff_launch_s > 0 else 0.0
    tbf = tb + tf
    s8d = ((STREAM_READ_BYTES + STREAM_WRITE_BYTES) * (tp + tbf) + 64.0 * (pp[0] * tp + pb[0] * tbf)
           + 48.0 * (pp[1] * tp + pb[1] * tbf) + 16.0 * (pp[2] * tp + pb[2] * tbf)) / max(1, launches)
    out = {"bound": "hbm", "kernel": "k_trace + k_bounce" if tf else "k_trace", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4)}
    out.update(_counter_fracs(wl_name, "trace", eff_launch_s, stream_read / max(1, launches)))
    if residency == "lds":
        out["s8d_lds_frac"] = round(s8d / eff_launch_s / 1e9 / LDS_PEAK_GBS, 4) if eff_launch_s else None
    else:
        out["frac_s8d"] = round(s8d / eff_launch_s / 1e9 / HBM_PEAK_GBS, 4) if eff_launch_s else None
    out.update({
        "busy_ms_per_step": round(busy_s * 1e3 / max(1, steps), 4),
        "busy_us_per_launch": round(eff_launch_s * 1e6, 2),
        "s8d_bytes_per_launch": round(s8d),
        "bytes_per_launch": round(per_launch), "stream_bytes_per_launch": round(stream / max(1, launches)),
        "scene_hbm_bytes_per_bounce_ray": round(scene_b) if residency == "hbm" else 0,
        "avg_launch_us": round(avg_launch_s * 1e6, 2),
        "launches_per_step": round(launches / max(1, steps), 3),
        "traversed_rays_per_launch": round((tp + tb + tf) / max(1, launches)),
        "fused_bounce_rays_per_step": round(tf / max(1, steps)),
        "handed_off": {"paths_per_launch": round(sum(getattr(s, "paths_handed_off", 0) for s in stats) / max(1, launches)),
                       "resumed_walk_bytes_per_launch": round(strag_bytes / max(1, launches))},
        "hit_fraction": {"primary": round(hp, 4), "bounce": round(hb, 4)},
        "scene_in_lds": residency == "lds", "scene_residency": residency, "scene_bytes": int(footprint),
        "per_ray": {"primary": {"nodes": round(pp[0], 3), "tris": round(pp[1], 3), "spheres": round(pp[2], 3)},
                    "bounce": {"nodes": round(pb[0], 3), "tris": round(pb[1], 3), "spheres": round(pb[2], 3)}}})
    # the instrumented step, per bounce: traversed rays and node visits per ray; per-ray visit histogram
    # (bin b: 2^(b-1) <= visits < 2^b)
    tbd, nbd = list(getattr(cnt, "traced_by_depth", [])), list(getattr(cnt, "nodes_by_depth", []))
    out["by_bounce"] = [{"bounce": d, "rays": int(tbd[d]), "nodes_per_ray": round(nbd[d] / tbd[d], 3)}
                        for d in range(len(tbd)) if tbd[d]]
    hist = list(getattr(cnt, "trace_visit_hist", []))
    if any(hist):
        out["visit_hist_log2"] = [int(x) for x in hist]
    if residency != "lds":
        out["overlap"] = ("launch durations include the time shared with the launches the library overlaps on "
                          "its second stream (k_sky beside bounce 0, k_shadow_dyn(d-1) beside bounce d; DESIGN.md §3)")
    fr = {"hbm_model": out["frac"], "hbm_counters": out["counter_frac"], "valu_issue": out["valu_issue_frac"]}
    known = {k: v for k, v in fr.items() if v is not None}
    out["binding"] = max(known, key=known.get) if known else None
    return out


# shadow task bytes: {origin, tfar} + {contrib, path id} read (32 B) and the radiance read-modify-write
# of an unoccluded task (32 B; charged to every task, an upper bound)
SHADOW_TASK_BYTES = 64.0


def shadow_roofline(cnt, stats, layout, wl_name, steps):
    """Roofline of the any-hit stage (k_shadow / k_shadow_dyn) where it runs as launches of its own (L2/HBM
    scenes; LDS scenes trace the shadow ray inside k_shade, and their line carries no shadow entry).  Per
    task: SHADOW_TASK_BYTES + 64 n_node + 48 n_tri with the instrumented pass's visits per any-hit query,
    HBM bytes per the scene residency as in roofline(); counters / VALU / SALU from the session's
    r*_pmc_<wl>_shadow.json / r*_sq_<wl>_shadow.json."""
    launches = sum(s.shadow_launches for s in stats)
    if not launches:
        return None
    avg_launch_s = sum(s.ms_shadow for s in stats) / launches * 1e-3
    tasks = sum(s.rays_shadow for s in stats)
    n_node = cnt.shadow_node_visits / max(1, cnt.rays_shadow)
    n_tri = cnt.shadow_prim_tests / max(1, cnt.rays_shadow)
    node_b = layout["node_bytes"] / max(1, layout["num_nodes"]) if layout["num_nodes"] else 64.0
    residency, footprint = _residency(layout)
    scene = {"lds": 0.0, "l2": XCDS * footprint * launches, "hbm": (node_b * n_node + 48.0 * n_tri) * tasks}[residency]
    per_launch = (SHADOW_TASK_BYTES * tasks + scene) / launches
    achieved = per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    out = {"bound": "hbm", "kernel": "k_shadow", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4)}
    out.update(_counter_fracs(wl_name, "shadow", avg_launch_s, 32.0 * tasks / launches))
    out.update({"bytes_per_launch": round(per_launch), "avg_launch_us": round(avg_launch_s * 1e6, 2),
                "launches_per_step": round(launches / max(1, steps), 3), "tasks_per_launch": round(tasks / launches),
                "per_task": {"nodes": round(n_node, 3), "tris": round(n_tri, 3)}, "scene_residency": residency,
                "ms_per_step": round(sum(s.ms_shadow for s in stats) / max(1, steps), 3)})
    hist = list(getattr(cnt, "shadow_visit_hist", []))
    if any(hist):
        out["visit_hist_log2"] = [int(x) for x in hist]
    return out


# k_shade per shaded hit: hit record (12) + ray origin/direction (32) + throughput (16) read, continuation
# ray (o, d, thr: 48) written, radiance read-modify-write (32)
SHADE_BYTES_PER_HIT = 12.0 + 32.0 + 16.0 + 48.0 + 32.0
# a bounce ray of the fused k_bounce (trace + shading in one launch, LDS scenes): its ray and throughput
# read once (48 B); a hit writes the continuation ray (48 B) and read-modify-writes the radiance (32 B,
# charged to every hit as for k_shade), a miss read-modify-writes the radiance (32 B); no hit record
FUSED_HIT_BYTES = 32.0 + 16.0 + 48.0 + 32.0
FUSED_MISS_BYTES = 32.0 + 16.0 + 32.0
SHADOW_TASK_WRITE_BYTES = 32.0  # a shadow task written by k_shade where the shadow ray has a launch of its own
ACCUM_BYTES_PER_PIXEL = 32.0 + 7.0  # accum read-modify-write; resolved RGBA8 tile + RGB8 image written


def step_roofline(cnt, stats, steps, ms_per_step, trace, shadow, pixels, spp, env_bytes=0):
    """Whole-step algorithmic HBM bytes over ms_per_step: every kernel of the step, not one launch.
      trace   the trace roofline's bytes per launch x its launches per step (traversed rays only)
      shadow  likewise for k_shadow(_dyn) (scenes whose shadow rays have launches of their own)
      shade   SHADE_BYTES_PER_HIT per hit of the wavefront trace launches (+ the shadow task written,
              where shadow rays have launches of their own)
      tail    k_tail keeps path state in registers: only its closest-hit rays' node/primitive bytes, for
              HBM scenes (the bounce rays' per-ray scene bytes)
      sky     culled camera samples: 4 cubemap texels (64 B) each with an HDR environment, up to one
              copy of the faces per XCD per k_sky launch (one per sample batch); the culled pixels'
              accum read-modify-write (32 B)
      accum   ACCUM_BYTES_PER_PIXEL per pixel + the 16-B radiance read of every traversed camera path
    This is a model of the bytes the algorithm must move, priced at the HBM peak; the measured step is
    latency-bound, so frac is well below 1."""
    tp = sum(s.traced_primary for s in stats) / steps
    tb = sum(s.traced_bounce for s in stats) / steps
    samples = sum(s.samples for s in stats) / steps
    tail_rays = sum(s.rays_tail for s in stats) / steps
    hp = getattr(cnt, "hits_primary", 0) / max(1, cnt.traced_primary)
    hb = getattr(cnt, "hits_bounce", 0) / max(1, cnt.traced_bounce)
    hits = tp * hp + tb * hb
    parts = {
        "trace": trace["bytes_per_launch"] * trace["launches_per_step"],
        "shadow": shadow["bytes_per_launch"] * shadow["launches_per_step"] if shadow else 0.0,
        "shade": hits * (SHADE_BYTES_PER_HIT + (SHADOW_TASK_WRITE_BYTES if shadow else 0.0)),
        "tail": tail_rays * trace.get("scene_hbm_bytes_per_bounce_ray", 0),
        "sky": env_hbm_bytes(samples - tp, env_bytes, sum(getattr(s, "waves", 1) for s in stats) / steps)
               + (samples - tp) / max(1, spp) * 32.0,
        "accum": pixels * ACCUM_BYTES_PER_PIXEL + tp * RAD_BYTES,
    }
    total = sum(parts.values())
    achieved = total / (ms_per_step * 1e-3) / 1e9 if ms_per_step > 0 else 0.0
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "bytes_per_step": round(total), "ms_per_step": round(ms_per_step, 4),
            "bytes_by_kernel": {k: round(v) for k, v in parts.items()}}


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
    harness (backends::HipBackend through the C ABI) as a child process: the default scene at 800x600
    and 1080p, and the L2/HBM scenes C3 (chair + HDR environment) and C5 (10M triangles) at 1080p; the
    1080p legs in launch mode 0 (graph replay where it pays, the default) and 1 (direct launches), and
    with HipBackend::Settings::lagged_readback (each render() returns the previous frame's image, read
    back beside the next frame's kernels: sptr_read_rgb8_lagged)."""
    import tempfile

    cli = os.path.join(ROOT, "simple-path-tracer_amd", "sptr_cli")
    out = []
    with tempfile.TemporaryDirectory() as d:
        sky = os.path.join(d, "sky.hdr")
        workloads.write_hdr(sky, workloads.synthetic_sky_equirect())
        c3, c5 = workloads.WORKLOADS["c3"], workloads.WORKLOADS["c5"]
        legs = [(["--scene", "default"], 800, 600, 0)]
        for mode in (0, 1):
            legs.append((["--scene", "default"], 1920, 1080, mode))
        for mode in (0, 1):
            legs.append((["--scene", c3.scene, "--env", sky], 1920, 1080, mode))
            legs.append((["--scene", f"sphere_mesh:{c5.p0}:{c5.p1}"], 1920, 1080, mode))
        legs += [(["--scene", "default", "--lagged"], 800, 600, 0), (["--scene", "default", "--lagged"], 1920, 1080, 0),
                 (["--scene", c3.scene, "--env", sky, "--lagged"], 1920, 1080, 0),
                 (["--scene", f"sphere_mesh:{c5.p0}:{c5.p1}", "--lagged"], 1920, 1080, 0)]
        for extra, w, h, mode in legs:
            r = subprocess.run([cli, *extra, "--w", str(w), "--h", str(h), "--spp", str(steps), "--warmup", "10",
                                "--launch-mode", str(mode), "--json", "--out", "/dev/null"], capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                raise RuntimeError(f"sptr_cli failed: {r.stderr[-2000:]}")
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            if rec["scene"].startswith("gltf:"):
                rec["scene"] = "c3 (gltf chair + synthetic HDR env)"
            elif rec["scene"].startswith("sphere_mesh"):
                rec["scene"] = "c5 (" + rec["scene"] + ")"
            out.append(rec)
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
    dist.barrier()
    t0 = time.perf_counter()
    tiles = sptr.pack_tiles(pattern, world, rank)  # stands in for the render + resolve of this rank's tiles
    t1 = time.perf_counter()
    gathered = torch.zeros(world * tiles.size, dtype=torch.int32)
    gather_tiles(torch.from_numpy(tiles.view(np.int32)), gathered, world, rank)
    img = sptr.unpack_tiles(gathered.numpy().view(np.uint32), world, W, H) if rank == 0 else None
    t2 = time.perf_counter()
    mine = torch.tensor([float(((tiles >> 24) == 255).sum())], dtype=torch.float64)  # pixels inside the image
    dist.all_reduce(mine)
    # the same per-step split the GPU line reports: max over ranks of render and of gather (+ unpack)
    tm = torch.tensor([(t1 - t0) * 1e3, (t2 - t1) * 1e3], dtype=torch.float64)
    dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    if rank == 0:
        ok = bool(np.array_equal(img, pattern)) and int(mine.item()) == W * H
        print(json.dumps({"dry_run": True, "n_gpus": world, "world_size": dist.get_world_size(),
                          "backend": dist.get_backend(), "workload": wl.name, "tiles_per_rank": int(tiles.size // 1024),
                          "pixels_covered": int(mine.item()), "gather_ok": ok,
                          "render_ms": round(float(tm[0]), 4), "gather_ms": round(float(tm[1]), 4),
                          "gather_bytes": int(world * tiles.size * 4) if world > 1 else 0}), flush=True)
        if not ok:
            sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(workloads.WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-interactive", action="store_true", help="skip the 1-spp progressive-frame leg")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo check of the rank launch + tile gather")
    ap.add_argument("--wave-paths", type=int, default=0)
    ap.add_argument("--leaf-size", type=int, default=0)
    ap.add_argument("--bvh-width", type=int, default=0, choices=[0, 2, 4])
    ap.add_argument("--split-refs", type=int, default=0, help="most references per split triangle (0 = library default, 1 = none)")
    ap.add_argument("--stragglers", type=int, default=-1,
                    help="straggler hand-off lane threshold (-1 = library default, 0 = off; HBM scenes)")
    ap.add_argument("--tail-depth", type=int, default=0, help="first bounce traced path-per-thread (0 = library default)")
    ap.add_argument("--pixel-lanes", type=int, default=0, choices=[0, 1, 2],
                    help="sptr_set_pixel_lanes: 0 automatic (default), 1 one launch chain, 2 two lanes")
    ap.add_argument("--launch-mode", type=int, default=0, choices=[0, 1, 2, 3],
                    help="0: replay captured launch graphs where they pay (default); 1: direct launches; 2: direct "
                         "launches on one stream, no overlap (timing studies); 3: graphs for every repeated shape")
    ap.add_argument("--no-serial-pass", action="store_true",
                    help="skip the untimed one-stream pass (launch mode 2) that times the trace / shadow launches "
                         "alone for scenes whose launches overlap")
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
    if args.split_refs:
        r.set_split_refs(args.split_refs)
    if args.stragglers >= 0:
        r.set_stragglers(args.stragglers)
    if args.tail_depth:
        r.set_tail_depth(args.tail_depth)
    if args.launch_mode:
        r.set_launch_mode(args.launch_mode)
    if args.pixel_lanes:
        r.set_pixel_lanes(args.pixel_lanes)
    # does the library's side stream run beside the render stream on this device (its own hardware
    # queue)?  Two 200-us one-wave spins, serial vs forked (sptr_overlap_probe)
    probe = r.overlap_probe()
    flat = workloads.setup(r, wl)
    layout, info = r.scene_layout(), r.scene_info()
    env_bytes = 6 * 512 * 512 * 16 if wl.hdr_env else 0  # workloads.hdr_env_faces(): 512^2 faces, float4 on the device
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

    def step(flags=0, ev=None):
        # every stage of a step is enqueued on torch's current stream, with no host synchronisation:
        # render (SPTR_FRAME_ASYNC) -> tile copy -> RCCL gather to rank 0 -> rank-0 unpack.  ev: three
        # timing events (render start, render + tile copy done, gather + unpack done) on that stream.
        if ev:
            ev[0].record()
        r.render(cam, W, H, spp=frames, max_depth=wl.max_depth, shard_rank=shard, shard_count=shards,
                 flags=flags | sptr.SPTR_FRAME_ASYNC, stream=stream, integrator=integ, samples_per_frame=4)
        ptr, nbytes = r.tiles_device()
        local_tiles = torch.as_tensor(_DevArray(ptr, nbytes), device=dev)
        src = local_tiles
        if local_tiles.numel() != send.numel():  # a rank with fewer tiles: padded to the common size
            send[: local_tiles.numel()].copy_(local_tiles)
            src = send
        if ev:
            ev[1].record()
        if distributed:
            gather_tiles(src, gathered, world, rank)
        elif shards > 1:  # --emulate-shards: shard 0's tiles in the gather buffer (the others stay 0)
            gathered[: src.numel()].copy_(src)
        tiles_in = gathered if shards > 1 else src  # one GPU, whole frame: unpacked in place
        if rank == 0:
            r.unpack_tiles(tiles_in.data_ptr(), shards, tiles_per_rank, W, H, image.data_ptr(), stream=stream)
        if ev:
            ev[2].record()
        return src

    # The timed steps are the calls a default caller makes: no stage-timing flag, so the library launches
    # them as it launches any render (launch mode 0: a captured graph where one replays faster, DESIGN.md
    # §6).  Every timed step recomputes the bounce-0 cull mask (SPTR_FRAME_RECULL): it is a per-camera
    # structure, and a renderer whose camera moves pays it every frame, so it is inside the timed step.
    # (--stage-timing: events around every stage inside the timed steps, a timing study, not a headline.)
    timed = sptr.SPTR_FRAME_RECULL | (sptr.SPTR_FRAME_TIMING if args.stage_timing else 0)
    for _ in range(args.warmup):
        step(timed)
    r.collect_stats()
    # untimed instrumented pass: BVH node / primitive fetch counts for the algorithmic-bytes model
    step(sptr.SPTR_FRAME_COUNT_VISITS)
    cnt = r.collect_stats()
    # the timed call shape seen twice right before timing (a graph, where mode 0 captures one, is captured
    # on the second call)
    for _ in range(2):
        step(timed)
    r.collect_stats()

    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        last_tiles = step(timed)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = [r.collect_stats()]  # the K timed steps' counters, summed

    # The last timed step's output against an untimed render of the same frame (default flags, the
    # library's own stream, synchronous: the call shape tests/test_gpu_golden.py checks against the oracle):
    # this rank's resolved tiles, and on one GPU the unpacked RGB8 image, byte for byte.
    tiles_timed = last_tiles.clone()
    image_timed = image.clone() if rank == 0 else None
    torch.cuda.synchronize()
    r.render(cam, W, H, spp=frames, max_depth=wl.max_depth, shard_rank=shard, shard_count=shards,
             integrator=integ, samples_per_frame=4)
    ref_ptr, ref_bytes = r.tiles_device()
    ref_tiles = torch.as_tensor(_DevArray(ref_ptr, ref_bytes), device=dev)
    n_cmp = min(ref_tiles.numel(), tiles_timed.numel())
    tile_words_differing = int((ref_tiles[:n_cmp] != tiles_timed[:n_cmp]).sum().item()) + \
        abs(ref_tiles.numel() - tiles_timed.numel())
    image_bytes_differing = None
    if rank == 0 and shards == 1:
        ref_rgb = torch.from_numpy(r.read_rgb8().reshape(-1)).to(dev)
        image_bytes_differing = int((ref_rgb != image_timed).sum().item())
    if distributed:  # every rank's differing tile words
        diff = torch.tensor([tile_words_differing], dtype=torch.int64, device=dev)
        dist.all_reduce(diff)
        tile_words_differing = int(diff.item())
    output_check = {"reference": "untimed render of the same frame, default flags, synchronous",
                    "identical": tile_words_differing == 0 and not image_bytes_differing,
                    "tile_words_differing": tile_words_differing, "image_bytes_differing": image_bytes_differing}

    # Launch durations for the roofline: an untimed pass of the same K steps in which the trace, fused-bounce
    # and shadow launches time themselves (SPTR_FRAME_TIMING_TRACE; such calls always run as direct launches).
    # Counts (rays, visits) are the same as the timed steps'; the durations are these launches' own.
    timing = (sptr.SPTR_FRAME_TIMING if args.stage_timing else sptr.SPTR_FRAME_TIMING_TRACE) | sptr.SPTR_FRAME_RECULL
    for _ in range(2):
        step(timing)
    r.collect_stats()
    torch.cuda.synchronize()
    tr0 = time.perf_counter()
    for i in range(args.steps):
        step(timing)
    torch.cuda.synchronize()
    rf_elapsed = time.perf_counter() - tr0
    stats_rf = [r.collect_stats()]

    # render / gather split of a step: an untimed pass of the same K steps with three torch events per step.
    # (The timed steps carry none: each event record between two launches idles the GPU for several
    # microseconds, r06: the 8-way C2 shard 0.478 ms/step with them, 0.458 without.)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for i in range(args.steps):
        step(timed, evs[i])
    torch.cuda.synchronize()
    r.collect_stats()
    render_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    gather_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps

    # one untimed step with events around every stage (the timed steps record them around the trace and
    # shadow launches only: each record between two launches idles the GPU for several microseconds)
    step(sptr.SPTR_FRAME_TIMING | sptr.SPTR_FRAME_RECULL)
    st_full = r.collect_stats()
    stage_full = {k: round(getattr(st_full, "ms_" + k), 3)
                  for k in ("total", "cull", "trace0", "trace", "shade0", "shade", "shadow", "tail", "accum")}

    # pixel lanes (sptr_set_pixel_lanes): the timed calls' two launch chains share the GPU, so their launch
    # durations include each other's time; an untimed pass of the same steps as one chain gives the
    # launches' own durations (roofline_one_chain)
    lanes_info = r.pixel_lanes_info()
    stats_one = None
    one_chain_pass = lanes_info["active"] and not args.no_serial_pass and args.integrator == "wavefront"
    if distributed:  # (its steps gather: every rank runs it or none)
        flag = torch.tensor([1 if one_chain_pass else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        one_chain_pass = bool(flag.item())
    if one_chain_pass:
        r.set_pixel_lanes(1)
        step(timing)
        r.collect_stats()
        torch.cuda.synchronize()
        to0 = time.perf_counter()
        for i in range(args.steps):
            step(timing)
        torch.cuda.synchronize()
        one_elapsed = time.perf_counter() - to0
        stats_one = [r.collect_stats()]
        r.set_pixel_lanes(args.pixel_lanes)

    # untimed one-stream pass (launch mode 2) for scenes whose launches overlap on the side streams: the
    # trace and shadow launches' own durations, with nothing beside them (roofline_serial)
    stats_serial = None
    residency = _residency(layout)[0]
    # the committed counter summaries (profiles/r*_pmc_<wl>_*.json) describe the workload's default line; an
    # emulated shard or a one-chain pass runs other launches, so they take no counter fractions
    prof = wl.name if not args.emulate_shards else f"{wl.name}_shard{args.emulate_shards}"
    if world == 1 and residency != "lds" and not args.no_serial_pass and args.launch_mode == 0 and \
            args.integrator == "wavefront":
        r.set_launch_mode(2)
        step(timing)
        r.collect_stats()
        torch.cuda.synchronize()
        ts0 = time.perf_counter()
        for i in range(args.steps):
            step(timing)
        torch.cuda.synchronize()
        serial_elapsed = time.perf_counter() - ts0
        stats_serial = [r.collect_stats()]
        r.set_launch_mode(0)

    # untimed pass of the same steps without stage events, launch mode 3: the call shape is captured
    # into a launch graph on its second call and replayed from then on (stage spans inside a graph would need
    # external event-record nodes, which torch's HIP 7.0 runtime refuses inside a capture: calls with
    # stage timing, like the timed steps above, run as direct launches)
    graph_replay = None
    if world == 1 and args.launch_mode == 0 and args.integrator == "wavefront" and not args.no_serial_pass:
        r.set_launch_mode(3)  # (mode 0 launches a large call with side-stream launches directly)
        for _ in range(2):
            step(sptr.SPTR_FRAME_RECULL)
        r.collect_stats()
        torch.cuda.synchronize()
        tg0 = time.perf_counter()
        for i in range(args.steps):
            step(sptr.SPTR_FRAME_RECULL)
        torch.cuda.synchronize()
        graph_elapsed = time.perf_counter() - tg0
        gst = r.collect_stats()
        g = r.graph_info()
        r.set_launch_mode(0)
        graph_replay = {"ms_per_step": round(graph_elapsed / args.steps * 1e3, 3),
                        "mrays_per_s": round((gst.rays_closest + gst.rays_shadow) / graph_elapsed / 1e6, 2),
                        "graph": {k: g[k] for k in ("valid", "nodes", "edges", "depth", "captures")},
                        "capture_error": g["capture_error"] or None}

    rays = sum(s.rays_closest + s.rays_shadow for s in stats)
    samples = sum(s.samples for s in stats)
    traced_p = sum(s.traced_primary for s in stats)
    t = torch.tensor([elapsed, float(rays), float(samples), float(traced_p), render_ms, gather_ms],
                     dtype=torch.float64, device=dev)
    per_rank_render = [render_ms]
    if distributed:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, rays, samples, traced_p = float(tmax[0]), float(tsum[1]), float(tsum[2]), float(tsum[3])
        render_ms, gather_ms = float(tmax[4]), float(tmax[5])
        allr = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(allr, t[4:5].clone())
        per_rank_render = [float(x.item()) for x in allr]
        # the gathered frame is the same bytes a 1-GPU render gives (tests/test_gpu_parity.py shard union)
        want = W * H * (frames * 4 if args.integrator == "pathtracer" else wl.spp) * args.steps
        assert int(tsum[2]) == want, (int(tsum[2]), want)

    if rank == 0:
        stage_ms = {k: round(sum(getattr(s, "ms_" + k) for s in stats_rf) / args.steps, 3)
                    for k in (("trace0", "trace", "shade0", "shade", "shadow", "tail", "accum", "cull")
                              if args.stage_timing else ("trace0", "trace", "shadow"))}
        knobs = {k: os.environ[k] for k in KNOB_VARS if os.environ.get(k)}
        if args.launch_mode:
            knobs["launch_mode"] = args.launch_mode
        if args.split_refs:
            knobs["split_refs"] = args.split_refs
        if args.stragglers >= 0:
            knobs["stragglers"] = args.stragglers
        if args.pixel_lanes:
            knobs["pixel_lanes"] = args.pixel_lanes
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
            "roofline": roofline(cnt, stats_rf, layout, prof, args.steps, env_bytes=env_bytes),
            "shadow_roofline": shadow_roofline(cnt, stats_rf, layout, prof, args.steps),
            # the launch durations above come from this untimed pass of the same steps
            "roofline_pass": {"flags": "SPTR_FRAME_TIMING_TRACE | SPTR_FRAME_RECULL (direct launches)",
                              "ms_per_step": round(rf_elapsed / args.steps * 1e3, 3)},
            "output_check": output_check,
            "overlap_probe": probe,
            "stage_ms_per_step": stage_ms,  # (the roofline pass's)
            # all stages of one untimed step, events around each (stage spans overlap on L2/HBM scenes)
            "stage_ms_untimed_step": stage_full,
            "cull_ms": stage_full["cull"],
            "cull_launches_per_step": sum(s.cull_launches for s in stats) / args.steps,
            "tail_rays_per_step": int(sum(s.rays_tail for s in stats) / args.steps),
            # paths the bounce traces handed to the straggler kernel (sptr_set_stragglers)
            "paths_handed_off_per_step": int(sum(s.paths_handed_off for s in stats) / args.steps),
            "rays_per_step": int(rays / args.steps),
            # queries answered without a traversal: the camera rays of frustum-culled pixels (all ranks)
            "culled_primary_per_step": int((samples - traced_p) / args.steps) if args.integrator == "wavefront" else 0,
            "traversed_rays_per_step": int((rays - (samples - traced_p if args.integrator == "wavefront" else 0)) / args.steps),
            # per step: max over ranks of render (+ tile copy) and of gather (+ rank-0 unpack), HIP events
            # (an untimed pass of the same steps)
            "render_ms": round(render_ms, 4),
            "gather_ms": round(gather_ms, 4),
            "gather_bytes": int(shards * tiles_per_rank * 4096) if distributed else 0,
            "render_ms_per_rank": [round(x, 4) for x in per_rank_render],
            "scene": {"prims": info["prims"], "lbvh_nodes": info["nodes"], "bvh_depth": info["depth"],
                      "lbvh_build_ms": round(info["build_ms"], 3), "leaf_size": layout["leaf_size"],
                      "bvh_width": layout["bvh_width"], "traversed_nodes": layout["num_nodes"],
                      "prim_refs": layout["num_prim_refs"]},
            "cpu_baseline": None,
        }
        if args.integrator == "wavefront":
            line["step_roofline"] = step_roofline(cnt, stats, args.steps, elapsed / args.steps * 1e3, line["roofline"],
                                                  line["shadow_roofline"], samples / max(1, args.steps) / wl.spp / world,
                                                  wl.spp, env_bytes=env_bytes)
        if stats_serial:
            rs = roofline(cnt, stats_serial, layout, wl.name, args.steps, env_bytes=env_bytes)
            ss = shadow_roofline(cnt, stats_serial, layout, wl.name, args.steps)
            line["roofline_serial"] = {
                "note": "untimed pass with every launch on one stream (launch mode 2): launch durations with nothing "
                        "beside them; the headline value is the overlapped run's",
                "ms_per_step": round(serial_elapsed / args.steps * 1e3, 3),
                "trace": {k: rs[k] for k in ("achieved", "frac", "avg_launch_us", "launches_per_step", "bytes_per_launch")},
                "shadow": {k: ss[k] for k in ("achieved", "frac", "avg_launch_us", "launches_per_step", "bytes_per_launch")}
                if ss else None}
        line["pixel_lanes"] = {"requested": lanes_info["requested"], "active": lanes_info["active"],
                               "note": "two lanes: the shard's even and odd tiles as two concurrent launch chains; "
                                       "each launch's duration (avg_launch_us) includes the other chain's time, so "
                                       "roofline.achieved divides the trace bytes by the trace launches' busy time "
                                       "(the union of their intervals over both lanes, busy_us_per_launch)"
                               if lanes_info["active"] else "one launch chain"}
        if stats_one:
            ro = roofline(cnt, stats_one, layout, wl.name + "_one_chain", args.steps, env_bytes=env_bytes)
            line["roofline_one_chain"] = {
                "note": "untimed pass of the same steps as one launch chain (sptr_set_pixel_lanes 1): the trace "
                        "launches' own durations; the headline value is the two-lane run's",
                "ms_per_step": round(one_elapsed / args.steps * 1e3, 3),
                "trace": {k: ro[k] for k in ("achieved", "frac", "avg_launch_us", "launches_per_step", "bytes_per_launch")}}
        if graph_replay:
            line["graph_replay"] = graph_replay
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
