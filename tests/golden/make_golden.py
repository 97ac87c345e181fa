#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference ships no tests, fixtures or golden images for this path and cannot be built here
(SURVEY.md §4, §8c), so these vectors come from the oracle restatement (oracle/wf_oracle.cpp):
they pin the oracle itself against regressions and are the shared expected values of the CPU and
GPU parity tests.  PARITY UNPINNED w.r.t. the reference binary.

Fixture plan: (i) wang_hash / rand01 streams, (ii) primary rays of a 64x48 image,
(iii) first-hit tables, (iv) 1-spp linear radiance at depth 1..6, (v) RGB8 of config C1
(default scene, 256x256, 4 spp, depth 6).

usage: python tests/golden/make_golden.py   (rewrites the .npz files next to this script)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

SEEDS = np.array([0, 1, 2, 61, 9781, 12345, 0x7FFFFFFF, 0x80000000, 0xDEADBEEF, 0xFFFFFFFF], np.uint32)


def camera_rays(cam, W, H, acc=1):
    d, _ = oracle.primary(cam, W, H, acc)
    rays = np.zeros((W * H, 8), np.float32)
    rays[:, 0:3] = cam[:3]
    rays[:, 3:6] = d.reshape(-1, 3)
    rays[:, 7] = np.inf
    return rays


def random_rays(n, seed):
    g = np.random.default_rng(seed)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = g.uniform((-5, 0, -6), (5, 3, 4), size=(n, 3))
    d = g.normal(size=(n, 3))
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = np.inf
    return rays


def main():
    # (i) RNG
    hashes = np.array([oracle.wang_hash(int(s)) for s in SEEDS], np.uint32)
    streams = np.stack([oracle.rand_stream(int(s), 16)[0] for s in SEEDS])
    states = np.stack([oracle.rand_stream(int(s), 16)[1] for s in SEEDS])
    np.savez_compressed(os.path.join(HERE, "rng.npz"), seeds=SEEDS, hashes=hashes, streams=streams, states=states)

    # (ii) primary rays, 64x48 at acc 1 and 5
    W, H = 64, 48
    cam = oracle.camera(aspect=W / H)
    d1, r1 = oracle.primary(cam, W, H, 1)
    d5, r5 = oracle.primary(cam, W, H, 5)
    np.savez_compressed(os.path.join(HERE, "primary.npz"), cam=cam, dirs1=d1, rng1=r1, dirs5=d5, rng5=r5)

    # (iii) first hits: camera rays + random rays, default scene and the test-triangle scene
    out = {}
    for name in ("default", "test_triangle"):
        P = oracle.Prepared(oracle.builtin_scene(name), bvh=False)
        rays = np.concatenate([camera_rays(oracle.camera(aspect=1.0), 48, 48), random_rays(4096, 3)])
        g, p, t, ng = P.intersect(rays)
        out[f"{name}_rays"], out[f"{name}_geom"], out[f"{name}_prim"] = rays, g, p
        out[f"{name}_t"], out[f"{name}_ng"] = t, ng
        occ_rays = random_rays(4096, 4)
        occ_rays[:, 6] = 1e-4
        out[f"{name}_occ_rays"], out[f"{name}_occ"] = occ_rays, P.occluded(occ_rays)
    np.savez_compressed(os.path.join(HERE, "hits.npz"), **out)

    # (iv) 1-spp radiance per max depth, 64x48, default + emitter scenes
    out = {}
    for name, wl in (("default", False), ("default_emitter", True)):
        P = oracle.Prepared(oracle.builtin_scene(name), bvh=False)
        for depth in range(1, 7):
            acc, rgb, cnt = P.render(cam, W, H, oracle.preset_materials(wl), oracle.default_lights(), frames=1,
                                     max_depth=depth, threads=8)
            out[f"{name}_d{depth}_accum"], out[f"{name}_d{depth}_rgb"] = acc, rgb
            out[f"{name}_d{depth}_rays"] = np.array([cnt["rays_closest"], cnt["rays_shadow"]], np.uint64)
    np.savez_compressed(os.path.join(HERE, "radiance.npz"), cam=cam, **out)

    # (v) config C1: default scene 256x256, 4 spp, depth 6
    W, H = 256, 256
    cam = oracle.camera(aspect=W / H)
    P = oracle.Prepared(oracle.builtin_scene("default"), bvh=False)
    acc, rgb, cnt = P.render(cam, W, H, oracle.preset_materials(False), oracle.default_lights(), frames=4,
                             max_depth=6, threads=8)
    np.savez_compressed(os.path.join(HERE, "c1_default_256_4spp.npz"), cam=cam, accum=acc, rgb=rgb,
                        rays=np.array([cnt["rays_closest"], cnt["rays_shadow"]], np.uint64))
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
