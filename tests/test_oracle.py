"""CPU: the oracle against the committed golden fixtures, its own internal consistency, and
analytic cases.  (Parity with the reference binary is unpinned — see oracle/wf_oracle.cpp.)"""
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _wang_hash_np(a):
    """wang_hash (include/wavefront/wf_math.h:35-43) in uint32 numpy arithmetic."""
    a = np.asarray(a, np.uint32).copy()
    with np.errstate(over="ignore"):
        a = (a ^ np.uint32(61)) ^ (a >> np.uint32(16))
        a = a * np.uint32(9)
        a = a ^ (a >> np.uint32(4))
        a = a * np.uint32(0x27D4EB2D)
        a = a ^ (a >> np.uint32(15))
    return a


def test_rng_golden_and_independent_restatement():
    g = _load("rng.npz")
    assert np.array_equal(np.array([oracle.wang_hash(int(s)) for s in g["seeds"]], np.uint32), g["hashes"])
    assert np.array_equal(_wang_hash_np(g["seeds"]), g["hashes"])
    for i, s in enumerate(g["seeds"]):
        vals, states = oracle.rand_stream(int(s), 16)
        assert np.array_equal(vals, g["streams"][i]) and np.array_equal(states, g["states"][i])
        # default_rand01 = (state & 0xFFFFFF) / 2^24 with state = wang_hash(previous)
        st = int(s)
        for k in range(16):
            st = int(_wang_hash_np(st))
            assert np.float32((st & 0xFFFFFF) / 16777216.0) == vals[k]


def test_primary_golden():
    g = _load("primary.npz")
    for acc, dk, rk in ((1, "dirs1", "rng1"), (5, "dirs5", "rng5")):
        d, r = oracle.primary(g["cam"], 64, 48, acc)
        assert np.array_equal(d.view(np.uint32), g[dk].view(np.uint32))
        assert np.array_equal(r, g[rk])
    # seeds follow GLRenderer.cpp:386-407: rng0 = wang_hash((y*W+x ^ acc) ^ 1)
    ps = np.arange(64 * 48, dtype=np.uint32).reshape(48, 64)
    assert np.array_equal(g["rng5"], _wang_hash_np((ps ^ np.uint32(5)) ^ np.uint32(1)))
    assert np.allclose(np.linalg.norm(g["dirs1"], axis=2), 1.0, atol=1e-6)


@pytest.mark.parametrize("name", ["default", "test_triangle"])
@pytest.mark.parametrize("bvh", [False, True])
def test_hits_golden(name, bvh):
    g = _load("hits.npz")
    P = oracle.Prepared(oracle.builtin_scene(name), bvh=bvh)
    geom, prim, t, ng = P.intersect(g[f"{name}_rays"])
    same = (geom == g[f"{name}_geom"]) & (prim == g[f"{name}_prim"])
    assert same.all()
    hit = geom != 0xFFFFFFFF
    assert np.array_equal(t[hit].view(np.uint32), g[f"{name}_t"][hit].view(np.uint32))
    assert np.array_equal(ng[hit].view(np.uint32), g[f"{name}_ng"][hit].view(np.uint32))
    assert np.array_equal(P.occluded(g[f"{name}_occ_rays"]), g[f"{name}_occ"])


@pytest.mark.parametrize("name", ["default", "default_emitter"])
def test_radiance_golden(name):
    g = _load("radiance.npz")
    P = oracle.Prepared(oracle.builtin_scene(name), bvh=True)
    mats = oracle.preset_materials(name == "default_emitter")
    for depth in range(1, 7):
        acc, rgb, cnt = P.render(g["cam"], 64, 48, mats, oracle.default_lights(), frames=1, max_depth=depth, threads=4)
        assert np.array_equal(acc.view(np.uint32), g[f"{name}_d{depth}_accum"].view(np.uint32)), depth
        assert np.array_equal(rgb, g[f"{name}_d{depth}_rgb"])
        assert [cnt["rays_closest"], cnt["rays_shadow"]] == list(g[f"{name}_d{depth}_rays"])


def test_c1_golden_and_thread_invariance():
    g = _load("c1_default_256_4spp.npz")
    P = oracle.Prepared(oracle.builtin_scene("default"), bvh=True)
    for threads in (1, 8):
        acc, rgb, cnt = P.render(g["cam"], 256, 256, oracle.preset_materials(False), oracle.default_lights(),
                                 frames=4, threads=threads)
        assert np.array_equal(rgb, g["rgb"])
        assert np.array_equal(acc.view(np.uint32), g["accum"].view(np.uint32))
        assert [cnt["rays_closest"], cnt["rays_shadow"]] == list(g["rays"])


def test_progressive_and_shards_in_oracle():
    P = oracle.Prepared(oracle.builtin_scene("default"), bvh=True)
    cam = oracle.camera(aspect=70 / 45)
    mats, lts = oracle.preset_materials(False), oracle.default_lights()
    full, frgb, _ = P.render(cam, 70, 45, mats, lts, frames=3)
    a, _, _ = P.render(cam, 70, 45, mats, lts, frames=1)
    a, rgb, _ = P.render(cam, 70, 45, mats, lts, frames=2, frame_begin=2, accum=a)
    assert np.array_equal(a, full) and np.array_equal(rgb, frgb)
    acc = np.zeros_like(full)
    for r in range(3):
        part, _, _ = P.render(cam, 70, 45, mats, lts, frames=3, shard_rank=r, shard_count=3)
        m = part.any(axis=2)
        acc[m] = part[m]
    assert np.array_equal(acc, full)


def test_bvh_matches_brute_force_on_mesh():
    sc = oracle.builtin_scene("sphere_mesh", 40, 80)
    Pb, Pf = oracle.Prepared(sc, bvh=True), oracle.Prepared(sc, bvh=False)
    g = np.random.default_rng(9)
    rays = np.zeros((20000, 8), np.float32)
    rays[:, 0:3] = g.uniform((-2, 0, 0), (2, 2, 5), size=(20000, 3))
    tgt = g.uniform((-0.8, 0.2, 1.2), (0.8, 1.8, 2.8), size=(20000, 3))
    d = tgt - rays[:, 0:3]
    rays[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = np.inf
    a, b = Pb.intersect(rays), Pf.intersect(rays)
    same = (a[0] == b[0]) & (a[1] == b[1])
    assert same.mean() >= 0.9999
    assert (a[0] != 0xFFFFFFFF).mean() > 0.5
    rays[:, 6] = 1e-4
    assert (Pb.occluded(rays) == Pf.occluded(rays)).all()


def test_analytic_sphere_and_triangle_hits():
    P = oracle.Prepared(oracle.builtin_scene("default"), bvh=False)
    rays = np.zeros((3, 8), np.float32)
    # toward the silver sphere (-1,1,0) r=1 from z=5: t = 4 exactly, Ng = (0,0,1); geomID 2
    rays[0] = [-1, 1, 5, 0, 0, -1, 0, np.inf]
    # straight down onto the glass cube top (y = 1.75) at x=z-center: geomID 0
    rays[1] = [0, 5, 2, 0, -1, 0, 0, np.inf]
    # straight up from below the scene: misses everything
    rays[2] = [10, -5, 10, 0, 1, 0, 0, np.inf]
    g, p, t, ng = P.intersect(rays)
    assert (g[0], p[0], t[0]) == (2, 0, np.float32(4.0))
    assert np.array_equal(ng[0], np.array([0, 0, 1], np.float32))
    assert g[1] == 0 and abs(t[1] - 3.25) < 1e-6 and ng[1][1] != 0 and ng[1][0] == 0 and ng[1][2] == 0
    assert g[2] == 0xFFFFFFFF


def test_sky_matches_float64_model():
    """EnvironmentManager::getSkyColor evaluated in float64 vs the oracle's float32 restatement."""
    dirs = np.array([[0, 1, 0], [0, -1, 0], [1, 0, 0], [0.3, 0.6, -0.8]], np.float64)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    out = oracle.env(dirs.astype(np.float32))
    for d, o in zip(dirs, out):
        t = 0.5 * (d[1] + 1.0)
        t = min(max(t, 0.0), 1.0)
        t = t * t * (3 - 2 * t)
        c = np.array([0.7, 0.8, 0.9]) * (1 - t) + np.array([0.2, 0.4, 0.8]) * t
        sd = np.array([0.3, 0.6, -0.8]) / np.linalg.norm([0.3, 0.6, -0.8])
        s = max(float(d @ sd), 0.0)
        c = (c + np.array([1.0, 0.9, 0.7]) * (s ** 64 + 0.3 * s ** 8)) * 0.8
        assert np.allclose(o, c, rtol=1e-5, atol=1e-6)


def test_resolve_matches_float64_model():
    acc = np.array([[[0.0, 0.5, 1.0], [2.0, 10.0, 0.01]]], np.float32) * 3
    rgb = oracle.resolve(acc, 3)
    x = acc.astype(np.float64) / 3
    c = np.clip((x * (2.51 * x + 0.03)) / (x * (2.43 * x + 0.59) + 0.14), 0, 1) ** (1 / 2.2)
    assert np.abs(rgb.astype(int) - np.floor(c * 255).astype(int)).max() <= 1
