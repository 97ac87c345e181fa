"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on identical inputs.

Tolerances (fp32 path tracing):
  * bit-exact: pixel/tile indexing, wang_hash seeds and RNG states, sample counts, shard mapping,
    accumulation order (progressive == one-shot, 1 shard == N shards);
  * primary directions and first-hit (geomID, primID, t): bit-exact expected (same IEEE op order,
    no contraction); asserted at >= 99.99 % identical;
  * images: >= 99.9 % of RGB8 pixels identical, and the linear radiance relative L1 <= 1e-3.
    Residual differences come from transcendental ulps (sin/cos/pow: glibc vs ocml) flipping a
    Russian-roulette or Fresnel decision on a handful of paths.
"""
import numpy as np
import pytest

import oracle
import sptr

pytestmark = pytest.mark.gpu


def _oracle_scene(name, p0=0, p1=0, bvh=False):
    return oracle.Prepared(oracle.builtin_scene(name, p0, p1), bvh=bvh)


def _image_close(rgb, orgb, acc, oacc, exact_frac=0.999, rel_l1=1e-3):
    diff = np.abs(rgb.astype(int) - orgb.astype(int))
    frac = float((diff == 0).all(axis=2).mean())
    # the reference's GGX term can overflow to inf on a perfect mirror alignment (dden == 0); such
    # samples must be non-finite on both sides, and the L1 is taken over the finite pixels
    fin, ofin = np.isfinite(acc), np.isfinite(oacc)
    assert (fin != ofin).sum() <= max(3, 1e-6 * fin.size), "non-finite pixels differ"
    m = fin & ofin
    rel = float(np.abs(acc[m] - oacc[m]).sum() / max(1e-12, np.abs(oacc[m]).sum()))
    assert frac >= exact_frac, f"exact-pixel fraction {frac}"
    assert rel <= rel_l1, f"relative L1 {rel}"
    return frac, rel


@pytest.mark.parametrize("acc", [1, 2, 77])
def test_primary_rays_bit_exact(renderer, acc):
    W, H = 96, 64
    cam = sptr.camera_lookat(aspect=W / H)
    dirs, rng = renderer.primary_rays(cam, W, H, acc)
    odirs, orng = oracle.primary(cam.as_array(), W, H, acc)
    assert np.array_equal(rng, orng)
    assert np.array_equal(dirs.view(np.uint32), odirs.view(np.uint32))


def _camera_rays(cam, W, H, acc=1):
    d, _ = oracle.primary(cam.as_array(), W, H, acc)
    o = np.broadcast_to(cam.as_array()[:3], d.shape)
    rays = np.zeros((W * H, 8), np.float32)
    rays[:, 0:3] = o.reshape(-1, 3)
    rays[:, 3:6] = d.reshape(-1, 3)
    rays[:, 6] = 0.0
    rays[:, 7] = np.inf
    return rays


def _random_rays(n, seed, lo=(-5, 0, -6), hi=(5, 3, 4)):
    g = np.random.default_rng(seed)
    o = g.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = g.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 3:6], rays[:, 6], rays[:, 7] = o, d.astype(np.float32), 0.0, np.inf
    return rays


@pytest.mark.parametrize("scene", ["default", "default_emitter", "test_triangle"])
def test_first_hits(renderer, scene):
    renderer.upload_scene(sptr.builtin_scene(scene))
    P = _oracle_scene(scene)
    cam = sptr.camera_lookat(aspect=1.0)
    rays = np.concatenate([_camera_rays(cam, 128, 128), _random_rays(50000, 7)])
    g, p, t, ng = renderer.intersect(rays)
    og, op, ot, ong = P.intersect(rays)
    same = (g == og) & (p == op)
    assert same.mean() >= 0.9999, same.mean()
    hit = same & (og != 0xFFFFFFFF)
    assert hit.sum() > (100 if scene == "test_triangle" else 1000)
    assert np.array_equal(t[hit].view(np.uint32), ot[hit].view(np.uint32))
    assert np.array_equal(ng[hit].view(np.uint32), ong[hit].view(np.uint32))


def test_occlusion(renderer):
    renderer.upload_scene(sptr.builtin_scene("default"))
    P = _oracle_scene("default")
    rays = _random_rays(50000, 11)
    rays[:, 6] = 1e-4
    rays[::2, 7] = np.float32(np.inf)
    rays[1::2, 7] = 2.5
    occ = renderer.occluded(rays)
    oocc = P.occluded(rays)
    assert (occ == oocc).mean() >= 0.9999
    assert 0.05 < occ.mean() < 0.95


def _render_pair(renderer, scene, W, H, spp, depth=6, env_faces=None, with_light=None, bvh=False, **kw):
    sptr.setup_default(renderer, scene, env_faces=env_faces)
    cam = sptr.camera_lookat(aspect=W / H)
    st = renderer.render(cam, W, H, spp=spp, max_depth=depth, **kw)
    rgb, acc = renderer.read_rgb8(), renderer.read_accum()
    wl = (scene == "default_emitter") if with_light is None else with_light
    P = _oracle_scene(scene, bvh=bvh)
    oacc, orgb, ocnt = P.render(cam.as_array(), W, H, oracle.preset_materials(wl), oracle.default_lights(),
                                frames=spp, max_depth=depth, env_faces=env_faces)
    return st, rgb, acc, orgb, oacc, ocnt


@pytest.mark.parametrize("depth", [1, 2, 6])
def test_render_default_depths(renderer, depth):
    st, rgb, acc, orgb, oacc, ocnt = _render_pair(renderer, "default", 96, 64, 2, depth=depth)
    _image_close(rgb, orgb, acc, oacc)
    assert st.samples == ocnt["samples"] == 96 * 64 * 2


def test_render_default_256_4spp(renderer):
    """BASELINE config C1 shape (default scene, 256x256, 4 spp, depth 6)."""
    st, rgb, acc, orgb, oacc, ocnt = _render_pair(renderer, "default", 256, 256, 4)
    _image_close(rgb, orgb, acc, oacc)
    # ray counts are per-query identical unless a path diverged
    assert abs(int(st.rays_closest) - ocnt["rays_closest"]) <= 0.001 * ocnt["rays_closest"]
    assert abs(int(st.rays_shadow) - ocnt["rays_shadow"]) <= 0.001 * ocnt["rays_shadow"] + 5


def test_render_emitter_scene(renderer):
    st, rgb, acc, orgb, oacc, ocnt = _render_pair(renderer, "default_emitter", 128, 96, 4)
    _image_close(rgb, orgb, acc, oacc)


def test_render_test_triangle_scene(renderer):
    st, rgb, acc, orgb, oacc, ocnt = _render_pair(renderer, "test_triangle", 64, 64, 2)
    _image_close(rgb, orgb, acc, oacc)


def test_render_ragged_size(renderer):
    """Image not a multiple of the 32x32 tile in either axis."""
    st, rgb, acc, orgb, oacc, ocnt = _render_pair(renderer, "default", 75, 41, 3)
    _image_close(rgb, orgb, acc, oacc)
    assert st.samples == 75 * 41 * 3


def test_progressive_equals_one_shot(renderer):
    sptr.setup_default(renderer, "default")
    W, H = 80, 48
    cam = sptr.camera_lookat(aspect=W / H)
    renderer.render(cam, W, H, spp=5)
    one = renderer.read_accum().copy(), renderer.read_rgb8().copy()
    renderer.render(cam, W, H, spp=2, frame_begin=1)
    renderer.render(cam, W, H, spp=1, frame_begin=3)
    renderer.render(cam, W, H, spp=2, frame_begin=4)
    prog = renderer.read_accum(), renderer.read_rgb8()
    assert np.array_equal(one[0].view(np.uint32), prog[0].view(np.uint32))
    assert np.array_equal(one[1], prog[1])


def test_wave_split_is_invisible(renderer):
    """Samples split over several wavefront batches accumulate in the same order."""
    sptr.setup_default(renderer, "default")
    W, H = 64, 64
    cam = sptr.camera_lookat(aspect=1.0)
    renderer.set_wave_paths(0)
    renderer.render(cam, W, H, spp=6)
    a = renderer.read_accum().copy()
    renderer.set_wave_paths(W * H)  # one sample per wave
    st = renderer.render(cam, W, H, spp=6)
    b = renderer.read_accum()
    renderer.set_wave_paths(0)
    assert st.waves == 6
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("G", [2, 3, 8])
def test_shards_union_equals_single(renderer, G):
    sptr.setup_default(renderer, "default")
    W, H = 150, 70
    cam = sptr.camera_lookat(aspect=W / H)
    renderer.render(cam, W, H, spp=2)
    full_rgb, full_acc = renderer.read_rgb8().copy(), renderer.read_accum().copy()
    rgb = np.zeros_like(full_rgb)
    acc = np.zeros_like(full_acc)
    total = 0
    for r in range(G):
        st = renderer.render(cam, W, H, spp=2, shard_rank=r, shard_count=G)
        total += st.samples
        part_rgb, part_acc = renderer.read_rgb8(), renderer.read_accum()
        m = part_acc.any(axis=2) | part_rgb.any(axis=2)
        rgb[m] = part_rgb[m]
        acc[m] = part_acc[m]
    assert total == W * H * 2
    assert np.array_equal(rgb, full_rgb)
    assert np.array_equal(acc.view(np.uint32), full_acc.view(np.uint32))


def test_sphere_mesh_scene(renderer):
    """C5 shape at reduced tessellation (40,000 triangles), oracle with its CPU BVH."""
    sptr.setup_default(renderer, "sphere_mesh", 100, 200)
    info = renderer.scene_info()
    assert info["prims"] == 2 * 100 * 200 + 8
    P = _oracle_scene("sphere_mesh", 100, 200, bvh=True)
    cam = sptr.camera_lookat(aspect=1.0)
    rays = np.concatenate([_camera_rays(cam, 96, 96), _random_rays(20000, 5)])
    g, p, t, ng = renderer.intersect(rays)
    og, op, ot, ong = P.intersect(rays)
    assert ((g == og) & (p == op)).mean() >= 0.9995
    W, H = 96, 72
    cam = sptr.camera_lookat(aspect=W / H)
    renderer.render(cam, W, H, spp=2)
    rgb, acc = renderer.read_rgb8(), renderer.read_accum()
    oacc, orgb, _ = P.render(cam.as_array(), W, H, oracle.preset_materials(False), oracle.default_lights(), frames=2)
    _image_close(rgb, orgb, acc, oacc, exact_frac=0.995, rel_l1=5e-3)


def _synthetic_equirect(w=256, h=128):
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.stack([0.5 + 0.5 * np.sin(x / w * 12.0), 0.3 + 0.7 * (y / h), 0.2 + 3.0 * ((x + y) % 17 == 0)], -1)
    return img.astype(np.float32)


def test_cubemap_environment(renderer):
    eq = _synthetic_equirect()
    faces = sptr.equirect_to_faces(eq, 64)
    assert np.array_equal(faces, oracle.equirect_to_faces(eq, 64))
    st, rgb, acc, orgb, oacc, _ = _render_pair(renderer, "default", 96, 64, 2, env_faces=faces)
    _image_close(rgb, orgb, acc, oacc)
    renderer.set_environment(None)


def test_debug_mode_hit_miss(renderer):
    sptr.setup_default(renderer, "default")
    W, H = 64, 48
    cam = sptr.camera_lookat(aspect=W / H)
    renderer.set_debug_mode(1)
    renderer.render(cam, W, H, spp=1)
    acc = renderer.read_accum()
    renderer.set_debug_mode(0)
    rays = _camera_rays(cam, W, H)
    g, _, _, _ = _oracle_scene("default").intersect(rays)
    hit = (g != 0xFFFFFFFF).reshape(H, W)
    assert ((acc[..., 0] == 1.0) == hit).mean() >= 0.999


@pytest.mark.parametrize("leaf", [1, 2, 8])
def test_leaf_size_invariance(renderer, leaf):
    """BVH leaf-range size only changes traversal work, never the image (default leaf size 4)."""
    W, H = 96, 64
    cam = sptr.camera_lookat(aspect=W / H)
    sptr.setup_default(renderer, "default_emitter")
    renderer.render(cam, W, H, spp=3)
    ref_acc = renderer.read_accum().copy()
    renderer.set_leaf_size(leaf)
    try:
        sptr.setup_default(renderer, "default_emitter")
        renderer.render(cam, W, H, spp=3)
        acc = renderer.read_accum()
    finally:
        renderer.set_leaf_size(0)
    assert np.array_equal(acc.view(np.uint32), ref_acc.view(np.uint32))


@pytest.mark.parametrize("scene,p0,p1", [("default_emitter", 0, 0), ("sphere_mesh", 60, 120)])
def test_bvh_width_invariance(renderer, scene, p0, p1):
    """BVH2 (the LBVH as built) and the collapsed BVH4 return the same hits and the same image."""
    W, H = 96, 64
    cam = sptr.camera_lookat(aspect=W / H)
    rays = _random_rays(20000, 11)
    out = {}
    try:
        for width in (2, 4):
            renderer.set_bvh_width(width)
            sptr.setup_default(renderer, scene, p0, p1)
            info = renderer.scene_layout()
            assert info["bvh_width"] == width
            renderer.render(cam, W, H, spp=3)
            out[width] = (renderer.read_accum().copy(), renderer.intersect(rays), info)
    finally:
        renderer.set_bvh_width(0)
    (a2, (g2, p2, t2, _), i2), (a4, (g4, p4, t4, _), i4) = out[2], out[4]
    assert i4["num_nodes"] < i2["num_nodes"]
    assert ((g2 == g4) & (p2 == p4)).mean() >= 0.9999
    assert np.array_equal(t2[g2 == g4].view(np.uint32), t4[g2 == g4].view(np.uint32))
    same = (a2 == a4).all(axis=2).mean()
    assert same >= 0.999


def test_async_renders_equal_sync(renderer):
    """SPTR_FRAME_ASYNC calls only defer the wait: same image, and collected stats = the sum."""
    sptr.setup_default(renderer, "default_emitter")
    W, H = 96, 64
    cam = sptr.camera_lookat(aspect=W / H)
    st1 = renderer.render(cam, W, H, spp=2)
    st2 = renderer.render(cam, W, H, spp=3, frame_begin=3)
    ref = renderer.read_accum().copy()
    for fb, spp in ((1, 2), (3, 3)):
        z = renderer.render(cam, W, H, spp=spp, frame_begin=fb, flags=sptr.SPTR_FRAME_ASYNC | sptr.SPTR_FRAME_TIMING)
        assert z.rays_closest == 0  # stats are deferred
    st = renderer.collect_stats()
    assert np.array_equal(renderer.read_accum().view(np.uint32), ref.view(np.uint32))
    assert st.rays_closest == st1.rays_closest + st2.rays_closest
    assert st.rays_shadow == st1.rays_shadow + st2.rays_shadow
    assert st.samples == W * H * 5 and st.ms_total > 0 and st.trace_launches > 0
    assert renderer.collect_stats().rays_closest == 0  # window restarted


@pytest.mark.parametrize("scene,p0,p1", [("default_emitter", 0, 0), ("sphere_mesh", 60, 120)])
def test_tail_depth_invariance(renderer, scene, p0, p1):
    """Where the wavefront stages hand over to the path-per-thread tail changes only the schedule:
    the image and the closest/any-hit query counts are identical for every split depth."""
    W, H = 96, 64
    cam = sptr.camera_lookat(aspect=W / H)
    sptr.setup_default(renderer, scene, p0, p1)
    out = {}
    try:
        for t in (1, 2, 3, 4, 5, 6, 0):
            renderer.set_tail_depth(t)
            st = renderer.render(cam, W, H, spp=4)
            out[t] = (renderer.read_accum().copy(), st.rays_closest, st.rays_shadow, st.rays_tail)
    finally:
        renderer.set_tail_depth(0)
    ref = out[6]
    assert ref[3] == 0  # tail at max_depth: all bounces are wavefront stages
    # automatic policy: an LDS-staged scene's small batch (96x64x4 paths) hands over to the tail at
    # bounce 4; a scene traversed from L2 (the BVH4 sphere mesh, < 4 MB) at bounce 2
    auto = 4 if renderer.scene_layout()["lds_bytes"] else 2
    assert out[0][3] == out[auto][3] > 0
    for t in (1, 2, 3, 4, 5, 0):
        acc, rc, rs, rt = out[t]
        assert np.array_equal(acc.view(np.uint32), ref[0].view(np.uint32)), t
        assert (rc, rs) == (ref[1], ref[2]), t
        assert 0 < rt < rc


def test_pixel_major_bounce0_accumulation(renderer):
    """At 1080p on one GPU the LDS-staged default scene runs bounce 0 pixel-major (leading misses
    folded into the accumulator, k_accum resuming at the first hit; kernels_wavefront.hip).  The
    folded sums must be bit-identical to the path-major kernel's (a 2-way shard runs path-major:
    too few pixels per resident thread), across progressive calls and across wave splits."""
    sptr.setup_default(renderer, "default_emitter")
    W, H, N = 1920, 1080, 4
    cam = sptr.camera_lookat(aspect=W / H)
    renderer.render(cam, W, H, spp=N)
    one_acc, one_rgb = renderer.read_accum().copy(), renderer.read_rgb8().copy()
    # progressive: the second call folds onto the first call's sums (no reset)
    renderer.render(cam, W, H, spp=1, frame_begin=1)
    renderer.render(cam, W, H, spp=N - 1, frame_begin=2)
    assert np.array_equal(one_acc.view(np.uint32), renderer.read_accum().view(np.uint32))
    # wave split: one sample per batch
    renderer.set_wave_paths(W * H)
    try:
        st = renderer.render(cam, W, H, spp=N)
    finally:
        renderer.set_wave_paths(0)
    assert st.waves == N
    assert np.array_equal(one_acc.view(np.uint32), renderer.read_accum().view(np.uint32))
    # path-major shards: their union is the same image, sample sums and all
    acc = np.zeros_like(one_acc)
    rgb = np.zeros_like(one_rgb)
    for r in range(2):
        renderer.render(cam, W, H, spp=N, shard_rank=r, shard_count=2)
        a_r, c_r = renderer.read_accum(), renderer.read_rgb8()
        m = a_r.any(axis=2) | c_r.any(axis=2)
        acc[m] = a_r[m]
        rgb[m] = c_r[m]
    assert np.array_equal(one_acc.view(np.uint32), acc.view(np.uint32))
    assert np.array_equal(one_rgb, rgb)


@pytest.mark.parametrize("scene,p0,p1,spp", [("default_emitter", 0, 0, 64), ("sphere_mesh", 60, 120, 40),
                                             ("default", 0, 0, 100)])
def test_wave_fold_bounce0_invariance(renderer, scene, p0, p1, spp):
    """Batches of >= 32 samples on small (or sharded, or L2/HBM-scene) frames run bounce 0 wave per
    pixel, folding each pixel's leading misses into the accumulator with a lane loop
    (k_trace_wp).  The sums must be bit-identical to path-major batches (8 samples per batch, every
    miss through rad[] and k_accum), including a partial last round of lanes (spp 40, 100)."""
    W, H = 96, 64
    cam = sptr.camera_lookat(aspect=W / H)
    sptr.setup_default(renderer, scene, p0, p1)
    try:
        st = renderer.render(cam, W, H, spp=spp)
        assert st.waves == 1
        acc, rgb = renderer.read_accum().copy(), renderer.read_rgb8().copy()
        P = 3 * 2 * 1024  # local pixels: 3 x 2 tiles
        renderer.set_wave_paths(P * 8)
        st8 = renderer.render(cam, W, H, spp=spp)
    finally:
        renderer.set_wave_paths(0)
    assert st8.waves == (spp + 7) // 8
    assert np.array_equal(acc.view(np.uint32), renderer.read_accum().view(np.uint32))
    assert np.array_equal(rgb, renderer.read_rgb8())
    assert (st.rays_closest, st.rays_shadow) == (st8.rays_closest, st8.rays_shadow)
    # progressive continuation from a folded batch
    renderer.render(cam, W, H, spp=spp, frame_begin=spp + 1)
    two = renderer.read_accum().copy()
    renderer.render(cam, W, H, spp=2 * spp)
    assert np.array_equal(two.view(np.uint32), renderer.read_accum().view(np.uint32))


def test_wave_fold_vs_oracle(renderer):
    st, rgb, acc, orgb, oacc, ocnt = _render_pair(renderer, "default_emitter", 64, 48, 48)
    _image_close(rgb, orgb, acc, oacc)
    assert st.samples == ocnt["samples"]


@pytest.mark.parametrize("integrator", [0, 1, 2])
def test_launch_graph_replay_equals_direct(renderer, integrator):
    """Repeated call shapes are captured into a hipGraph and replayed (sptr_set_launch_mode 3): the
    accumulation and the stats must match direct launches call for call — including progressive
    continuation (the per-call frame index is a graph-node argument), a camera change (new shape:
    direct launches again, then a second capture) and asynchronous calls.  The default mode 0 captures
    only shapes of at least 2^24 samples whose launches fork nothing to the side streams (small calls,
    forking or not, run direct; 1024x256x64 calls of the LDS scene fork nothing and are captured).  Calls with stage timing run as direct launches in every mode (no capture)."""
    W, H = 96, 64
    sptr.setup_default(renderer, "default_emitter")
    cams = [sptr.camera_lookat(aspect=W / H), sptr.camera_lookat(pos=(0.5, 3.0, 8.0), aspect=W / H)]
    out = {}
    try:
        for mode in (1, 3):
            renderer.set_launch_mode(mode)
            g0 = renderer.graph_info()
            seq = []
            for cam in (cams[0], cams[0], cams[0], cams[1], cams[1], cams[1]):
                fb = 1 if not seq or seq[-1][3] is not cam else seq[-1][4] + 2
                st = renderer.render(cam, W, H, spp=2, frame_begin=fb, integrator=integrator)
                seq.append((renderer.read_accum().copy(), st.rays_closest, st.rays_shadow, cam, fb, st.ms_total))
            for fb in (1, 3, 5):  # asynchronous replays, one collection
                renderer.render(cams[0], W, H, spp=2, frame_begin=fb, integrator=integrator,
                                flags=sptr.SPTR_FRAME_ASYNC)
            st = renderer.collect_stats()
            seq.append((renderer.read_accum().copy(), st.rays_closest, st.rays_shadow, None, 0, st.ms_total))
            out[mode] = seq
            g = renderer.graph_info()
            if mode == 3:  # one capture per camera, the asynchronous calls replay the first camera's again
                assert g["valid"] == 1 and g["captures"] == g0["captures"] + 3, (g0, g)
            else:
                assert g["captures"] == g0["captures"], (g0, g)
        # mode 0 (the default) on new shapes (other frame sizes): a small call runs direct; a large one
        # that forks nothing is captured on its second call (as one launch chain: two pixel lanes would
        # halve each chain's samples)
        renderer.set_pixel_lanes(1)
        for W0, H0, spp0, captured in ((80, H, 2, False), (1024, 256, 64, True)):
            cam0 = sptr.camera_lookat(aspect=W0 / H0)
            ref = []
            renderer.set_launch_mode(1)
            for fb in (1, 1 + spp0, 1 + 2 * spp0):
                renderer.render(cam0, W0, H0, spp=spp0, frame_begin=fb, integrator=integrator)
                ref.append(renderer.read_accum().copy())
            renderer.set_launch_mode(0)
            g0 = renderer.graph_info()
            for i, fb in enumerate((1, 1 + spp0, 1 + 2 * spp0)):
                renderer.render(cam0, W0, H0, spp=spp0, frame_begin=fb, integrator=integrator)
                assert np.array_equal(renderer.read_accum().view(np.uint32), ref[i].view(np.uint32))
            g = renderer.graph_info()
            assert g["captures"] == g0["captures"] + (1 if captured else 0), (W0, g0, g)
            if captured:
                assert g["valid"] == 1
        # stage timing: direct launches however often the shape repeats
        g0 = renderer.graph_info()
        for _ in range(3):
            st = renderer.render(cams[0], W, H, spp=2, integrator=integrator, flags=sptr.SPTR_FRAME_TIMING_TRACE)
            if integrator == 0:  # the trace launches' spans only: no call span, no cull span
                assert st.ms_total == 0.0 and st.ms_cull == 0.0
                assert st.trace_launches > 0 and st.ms_trace > 0.0
            else:  # path per thread: no trace stage; the call span
                assert st.ms_total > 0.0
        assert renderer.graph_info()["captures"] == g0["captures"]
    finally:
        renderer.set_launch_mode(0)
        renderer.set_pixel_lanes(0)
    for a, b in zip(out[1], out[3]):
        assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
        assert (a[1], a[2]) == (b[1], b[2])
        assert b[5] > 0.0  # the call span's events were re-pointed and recorded on replay
        # direct calls: the span of a wavefront call is its device wall-clock slot (k_frame_dyn's start, the last
        # k_accum's end), of a path-per-thread call two event records
        assert a[5] > 0.0


@pytest.mark.parametrize("scene", ["default", "default_emitter"])
def test_fused_shadow_equals_shadow_stage(renderer, scene):
    """LDS-staged one-light scenes trace the shadow ray inside k_shade; the visit-count pass keeps the
    separate k_shadow stage.  Both must accumulate the same bits and count the same any-hit queries
    (the in-shade query adds its contribution after the emission, as k_shadow's update does)."""
    W, H = 96, 64
    cam = sptr.camera_lookat(aspect=W / H)
    sptr.setup_default(renderer, scene)
    st = renderer.render(cam, W, H, spp=6)
    fused = renderer.read_accum().copy()
    st2 = renderer.render(cam, W, H, spp=6, flags=sptr.SPTR_FRAME_COUNT_VISITS)
    assert st2.shadow_node_visits > 0  # the separate stage ran
    assert np.array_equal(fused.view(np.uint32), renderer.read_accum().view(np.uint32))
    assert (st.rays_closest, st.rays_shadow) == (st2.rays_closest, st2.rays_shadow)


@pytest.mark.parametrize("scene,p0,p1,spp,W,H", [("default_emitter", 0, 0, 64, 256, 144), ("default", 0, 0, 3, 96, 64),
                                                 ("sphere_mesh", 60, 120, 4, 96, 64)])
def test_pixel_cull_invisible(renderer, scene, p0, p1, spp, W, H):
    """Bounce-0 pixel-frustum culling (k_cull) skips the traversal of camera rays that cannot hit the
    top BVH boxes: the accumulation and the ray counts equal a render without it (SPTR_FRAME_NO_CULL)
    bit for bit — in the thread-per-pixel, path-major and BVH4 bounce-0 kernels — while the
    instrumented pass shows fewer node visits."""
    cam = sptr.camera_lookat(aspect=W / H)
    sptr.setup_default(renderer, scene, p0, p1)
    st = renderer.render(cam, W, H, spp=spp)
    acc = renderer.read_accum().copy()
    st0 = renderer.render(cam, W, H, spp=spp, flags=sptr.SPTR_FRAME_NO_CULL)
    assert np.array_equal(acc.view(np.uint32), renderer.read_accum().view(np.uint32))
    assert (st.rays_closest, st.rays_shadow) == (st0.rays_closest, st0.rays_shadow)
    c1 = renderer.render(cam, W, H, spp=1, flags=sptr.SPTR_FRAME_COUNT_VISITS)
    c0 = renderer.render(cam, W, H, spp=1, flags=sptr.SPTR_FRAME_COUNT_VISITS | sptr.SPTR_FRAME_NO_CULL)
    assert c1.node_visits < c0.node_visits


@pytest.mark.parametrize("scene,p0,p1,spp", [("sphere_mesh", 60, 120, 16), ("sphere_mesh", 300, 600, 8)])
def test_overlapped_launches_equal_serial(renderer, scene, p0, p1, spp):
    """Scenes traversed from L2/HBM run k_shadow_dyn(d) on a second stream beside k_trace_dyn(d + 1)
    (bounce-trace misses deferred to k_shade) and k_sky beside the bounce-0 trace, in captured graphs
    (launch mode 3) and direct launches (modes 1 and 0, which runs forking calls directly); mode 2 keeps
    every launch on one stream.  The images and ray counts must be equal bit for bit, and repeated
    renders too."""
    W, H = 160, 96
    sptr.setup_default(renderer, scene, p0, p1)
    cam = sptr.camera_lookat(aspect=W / H)
    out = {}
    try:
        for mode in (2, 1, 0, 3):
            renderer.set_launch_mode(mode)
            runs = []
            for _ in range(3):  # mode 3: direct, then captured and replayed
                st = renderer.render(cam, W, H, spp=spp, frame_begin=1)
                runs.append((renderer.read_accum().copy(), st.rays_closest, st.rays_shadow))
            out[mode] = runs
    finally:
        renderer.set_launch_mode(0)
    ref = out[2][0]
    assert ref[2] > 0  # shadow rays traced
    for mode in (2, 1, 0, 3):
        for a in out[mode]:
            assert np.array_equal(a[0].view(np.uint32), ref[0].view(np.uint32)), mode
            assert a[1:] == ref[1:], mode


@pytest.mark.parametrize("nlights,depth", [(1, 6), (1, 32), (8, 32)])
def test_many_lights_deep_paths_overlapped_equal_serial(renderer, nlights, depth):
    """Scenes beyond an XCD's L2 with up to 8 lights (directional and point: 3-slot shadow tasks) and paths
    up to the maximum depth (32, so the tail carries 29 bounces): the overlapped launch sequence (shadow
    launches beside the next bounce trace, k_strag and k_sky beside the chain) in direct launches (modes 1
    and 0) and a replayed graph (mode 3) gives the one-stream sequence's (mode 2) image and query counts bit
    for bit.  (r06: this also covered a deferred tail, started beside the last shadow launch, measured
    no faster and not kept)"""
    W, H, S = 128, 96, 8
    sptr.setup_default(renderer, "sphere_mesh", 300, 600)
    lights = sptr.default_lights()
    extra = []
    for i in range(nlights - len(lights)):
        l = sptr.Light()
        l.type = 1 if i % 2 == 0 else 0
        l.v[0], l.v[1], l.v[2] = (1.5 - 0.4 * i, 2.0 + 0.1 * i, 1.0) if l.type == 1 else (0.3, 0.8 + 0.05 * i, 0.4)
        l.color[0], l.color[1], l.color[2] = 1.0, 0.9 - 0.05 * i, 0.8
        l.intensity = 2.0 if l.type == 1 else 0.5
        extra.append(l)
    cam = sptr.camera_lookat(aspect=W / H)
    out = {}
    try:
        renderer.set_lights((lights + extra)[:nlights])
        for mode in (2, 1, 0, 3):
            renderer.set_launch_mode(mode)
            runs = []
            for _ in range(2 if mode != 3 else 3):
                st = renderer.render(cam, W, H, spp=S, max_depth=depth)
                runs.append((renderer.read_accum().copy(), st.rays_closest, st.rays_shadow))
            out[mode] = runs
    finally:
        renderer.set_launch_mode(0)
        renderer.set_lights(lights)
    ref = out[2][0]
    assert ref[2] > 0
    for mode in (2, 1, 0, 3):
        for a in out[mode]:
            assert np.array_equal(a[0].view(np.uint32), ref[0].view(np.uint32)), mode
            assert a[1:] == ref[1:], mode


@pytest.mark.parametrize("mode", [1, 3])
def test_many_calls_without_collect(renderer, mode):
    """1500 asynchronous calls of an L2-scene frame with no collection in between, each forking k_sky
    and the shadow launches to the side streams and joining them back: direct launches (mode 1, as the
    default mode 0 runs a forking call), and one captured graph replayed (mode 3).  No state may
    accumulate in the runtime (r03 saw a host stack
    overflow inside libamdhip64 in this suite — the recursion of hipStreamEndCapture over a cyclic
    capture-stream list, DESIGN.md §6 "Launch graphs"), and every call must give the same image."""
    W, H = 96, 64
    sptr.setup_default(renderer, "sphere_mesh", 60, 120)
    cam = sptr.camera_lookat(aspect=W / H)
    try:
        renderer.set_launch_mode(mode)
        g0 = renderer.graph_info()
        renderer.render(cam, W, H, spp=4, frame_begin=1)
        ref = renderer.read_accum().copy()
        for _ in range(1500):
            renderer.render(cam, W, H, spp=4, frame_begin=1, flags=sptr.SPTR_FRAME_ASYNC)
        renderer.collect_stats()
        assert np.array_equal(ref.view(np.uint32), renderer.read_accum().view(np.uint32))
        g = renderer.graph_info()
        if mode == 3:
            assert g["valid"] == 1 and g["captures"] == g0["captures"] + 1, (g0, g)
        else:
            assert g["captures"] == g0["captures"], (g0, g)
    finally:
        renderer.set_launch_mode(0)


@pytest.mark.parametrize("lanes", [64, 12])
def test_straggler_handoff_changes_no_result(renderer, lanes):
    """Straggler hand-off (sptr_set_stragglers, scenes beyond an XCD's L2): bounce traces hand the rays
    still running in their drained waves to k_strag, which finishes those paths beside the chain.  With
    every drained wave's rays handed off (64 lanes) and with the default (12), the accumulation is
    bit-identical to no hand-off, the query counts are equal, and paths were handed off — in direct
    launches (mode 1), a captured graph (mode 3) and one stream (mode 2)."""
    W, H, S = 128, 96, 8
    sptr.setup_default(renderer, "sphere_mesh", 300, 600)  # 360 K triangles, 17 MB: beyond one L2
    cam = sptr.camera_lookat(aspect=W / H)
    try:
        renderer.set_stragglers(0)
        st0 = renderer.render(cam, W, H, spp=S)
        ref = renderer.read_accum().copy()
        assert st0.paths_handed_off == 0
        renderer.set_stragglers(lanes)
        for mode in (1, 3, 2):
            renderer.set_launch_mode(mode)
            for _ in range(3):
                st = renderer.render(cam, W, H, spp=S)
                assert np.array_equal(ref.view(np.uint32), renderer.read_accum().view(np.uint32)), (mode, lanes)
                assert (st.rays_closest, st.rays_shadow) == (st0.rays_closest, st0.rays_shadow), (mode, lanes)
                if lanes == 64:
                    assert st.paths_handed_off > 0, mode
            print("stragglers", lanes, "mode", mode, "handed off", st.paths_handed_off)
    finally:
        renderer.set_launch_mode(0)
        renderer.set_stragglers(12)


def test_straggler_handoff_multibatch(renderer):
    """Hand-off in a call of several sample batches (set_wave_paths: 4 samples per batch): each batch's
    k_strag is joined before that batch's k_accum, which zeroes the counts for the next batch; the
    accumulation equals the one-batch call without hand-off, bit for bit, direct and captured."""
    W, H, S = 96, 64, 16
    sptr.setup_default(renderer, "sphere_mesh", 300, 600)
    cam = sptr.camera_lookat(aspect=W / H)
    P = 3 * 2 * 1024  # local pixels: 3 x 2 tiles
    try:
        renderer.set_stragglers(0)
        st0 = renderer.render(cam, W, H, spp=S)
        ref = renderer.read_accum().copy()
        renderer.set_stragglers(64)
        renderer.set_wave_paths(P * 4)
        for mode in (1, 3):
            renderer.set_launch_mode(mode)
            for _ in range(3):
                st = renderer.render(cam, W, H, spp=S)
                assert st.waves == S // 4
                assert np.array_equal(ref.view(np.uint32), renderer.read_accum().view(np.uint32)), mode
                assert (st.rays_closest, st.rays_shadow) == (st0.rays_closest, st0.rays_shadow), mode
                assert st.paths_handed_off > 0, mode
    finally:
        renderer.set_wave_paths(0)
        renderer.set_launch_mode(0)
        renderer.set_stragglers(12)


def test_large_forked_call_launches_direct(renderer):
    """Launch mode 0 leaves a large call whose launches fork to the side streams (here 8.4 M samples,
    the shadow launches beside the traces of the L2-resident sphere mesh) to direct launches — the
    graph executor runs a graph's branches one after another, r04h — and mode 3 captures it; both give
    the same image."""
    W, H, S = 1024, 1024, 8
    sptr.setup_default(renderer, "sphere_mesh", 60, 120)
    cam = sptr.camera_lookat(aspect=W / H)
    out = {}
    try:
        for mode in (0, 3):
            renderer.set_launch_mode(mode)
            g0 = renderer.graph_info()
            for _ in range(3):
                renderer.render(cam, W, H, spp=S, flags=sptr.SPTR_FRAME_RECULL)
            g = renderer.graph_info()
            assert g["captures"] == g0["captures"] + (1 if mode == 3 else 0), (mode, g0, g)
            out[mode] = renderer.read_accum().copy()
    finally:
        renderer.set_launch_mode(0)
    assert np.array_equal(out[0].view(np.uint32), out[3].view(np.uint32))


@pytest.mark.parametrize("scene,p0,p1,spp", [("sphere_mesh", 60, 120, 24), ("default_emitter", 0, 0, 24)])
def test_multibatch_overlapped_graph_replay(renderer, scene, p0, p1, spp):
    """A call of several sample batches (set_wave_paths: 8 samples per batch -> 3 batches) with the
    overlapped side-stream launches (k_sky beside each bounce-0 trace, k_shadow_dyn(d) beside the next
    bounce's trace, on the L2/HBM scene) captured into one graph (launch mode 3, call 2; mode 0 would run
    a forking call directly) and replayed (calls 3-4): the graph passes the DAG check, and every call is
    bit-identical to the serial one-stream direct launches (mode 2)."""
    W, H = 96, 64
    sptr.setup_default(renderer, scene, p0, p1)
    cam = sptr.camera_lookat(aspect=W / H)
    P = 3 * 2 * 1024  # local pixels: 3 x 2 tiles
    out = {}
    try:
        renderer.set_wave_paths(P * 8)
        for mode in (2, 3):
            renderer.set_launch_mode(mode)
            g0 = renderer.graph_info()
            runs = []
            for _ in range(4):
                st = renderer.render(cam, W, H, spp=spp, frame_begin=1)
                assert st.waves == spp // 8
                runs.append((renderer.read_accum().copy(), st.rays_closest, st.rays_shadow))
            out[mode] = runs
            if mode == 3:
                g = renderer.graph_info()
                assert g["valid"] == 1 and g["captures"] == g0["captures"] + 1, (g0, g)
                # a DAG whose longest path runs through every batch's sequence
                assert 3 * spp // 8 < g["depth"] <= g["nodes"] <= 4096, g
                assert g["edges"] >= g["nodes"] - 1, g
    finally:
        renderer.set_wave_paths(0)
        renderer.set_launch_mode(0)
    ref = out[2][0]
    for mode in (2, 3):
        for a in out[mode]:
            assert np.array_equal(a[0].view(np.uint32), ref[0].view(np.uint32)), mode
            assert a[1:] == ref[1:], mode


def test_overlap_probe(renderer):
    """sptr_overlap_probe runs and reports plausible spin times (the bench line records them)."""
    p = renderer.overlap_probe()
    print("overlap_probe", p)
    assert 0.3 < p["serial_ms"] < 5.0, p
    assert 0.15 < p["side_ms"] <= p["serial_ms"] * 1.2, p
    assert 0.15 < p["sky_side_ms"] <= p["serial_ms"] * 1.2, p


@pytest.mark.parametrize("scene,p0,p1", [("default_emitter", 0, 0), ("sphere_mesh", 60, 120)])
def test_graph_replay_after_camera_switch(renderer, scene, p0, p1):
    """A launch graph captured for camera A must run against A's pixel-cull mask when it is replayed
    after a call with camera B recomputed the mask (calls A, A [captured], B, A [replayed], A): each
    call's image equals the direct-launch image of its camera, in the thread-per-pixel (LDS scene) and
    the path-major cull-list (BVH4 scene) bounce-0 kernels."""
    W, H = 96, 64
    sptr.setup_default(renderer, scene, p0, p1)
    cams = {"A": sptr.camera_lookat(aspect=W / H),
            "B": sptr.camera_lookat(pos=(4.0, 2.0, 6.0), target=(-1.0, 1.0, 0.0), aspect=W / H)}
    out = {}
    try:
        for mode in (1, 3):
            renderer.set_launch_mode(mode)
            out[mode] = []
            for name in "AABAA":
                st = renderer.render(cams[name], W, H, spp=16, frame_begin=1)
                out[mode].append((renderer.read_accum().copy(), st.rays_closest, st.rays_shadow, st.traced_primary))
    finally:
        renderer.set_launch_mode(0)
    assert not np.array_equal(out[1][0][0], out[1][2][0])  # the two cameras see different images
    for a, b in zip(out[1], out[3]):
        assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
        assert a[1:] == b[1:]


def test_traced_ray_counts(renderer):
    """traced_primary counts the camera rays bounce 0 actually traverses (culled pixels' samples are
    answered without a traversal), traced_bounce the queued rays of the later trace launches; with the
    path-per-thread tail off and no fused bounce (BVH4 scene), every closest-hit query is one of them
    or a culled camera ray."""
    W, H, spp = 96, 64, 4
    cam = sptr.camera_lookat(aspect=W / H)
    sptr.setup_default(renderer, "sphere_mesh", 60, 120)
    try:
        renderer.set_tail_depth(32)
        st0 = renderer.render(cam, W, H, spp=spp, flags=sptr.SPTR_FRAME_NO_CULL)
        st = renderer.render(cam, W, H, spp=spp, flags=sptr.SPTR_FRAME_RECULL)
    finally:
        renderer.set_tail_depth(0)
    assert st0.traced_primary == st0.samples == W * H * spp
    assert 0 < st.traced_primary < st.samples and st.traced_primary % spp == 0
    assert st.cull_launches == 1 and st0.cull_launches == 0
    assert st.traced_bounce == st0.traced_bounce > 0
    assert st0.rays_closest == st0.traced_primary + st0.traced_bounce
    assert st.rays_closest == st0.rays_closest
    # per bounce: bounce 0 = the traversed camera rays; the bounces add up to the trace kernels' rays
    assert st.traced_by_depth[0] == st.traced_primary
    assert sum(st.traced_by_depth) == st.traced_primary + st.traced_bounce
    # instrumented pass: every traversed ray lands in one visit-histogram bin, every any-hit query too
    try:
        renderer.set_tail_depth(32)
        sc = renderer.render(cam, W, H, spp=spp, flags=sptr.SPTR_FRAME_COUNT_VISITS)
    finally:
        renderer.set_tail_depth(0)
    assert sum(sc.trace_visit_hist) == sc.traced_primary + sc.traced_bounce
    assert sum(sc.shadow_visit_hist) == sc.rays_shadow
    assert sum(sc.nodes_by_depth) == sc.node_visits


def test_split_references_change_no_result(renderer):
    """Split references (early split clipping of sliver triangles, sptr_set_split_refs): the sphere
    mesh's polar rows are slivers, so with splits on the BVH holds more references than triangles.  First
    hits (geomID, primID, t bits) on camera and random rays, occlusion, and a render with shadow rays
    are the same with and without splits (a closest hit can differ only on an exact t tie between two
    triangles, which the two trees may test in a different order)."""
    W, H = 96, 64
    cam = sptr.camera_lookat(aspect=W / H)
    g = np.random.default_rng(5)
    d = g.normal(size=(40000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((40000, 8), np.float32)
    rays[:, 0:3] = g.uniform((-1.2, 0.2, -1.2), (1.2, 2.4, 1.2), size=(40000, 3))  # around the mesh's poles
    rays[:, 3:6] = d
    rays[:, 7] = np.inf
    out = {}
    try:
        for pieces in (1, 16):
            renderer.set_split_refs(pieces)
            sptr.setup_default(renderer, "sphere_mesh", 60, 120)
            lay = renderer.scene_layout()
            st = renderer.render(cam, W, H, spp=8)
            out[pieces] = (lay, renderer.intersect(rays), renderer.occluded(rays), renderer.read_rgb8().copy(), st)
    finally:
        renderer.set_split_refs(0)
    (l1, h1, o1, rgb1, st1), (l16, h16, o16, rgb16, st16) = out[1], out[16]
    assert l1["num_prim_refs"] == l1["num_tris"] + l1["num_spheres"]
    assert l16["num_prim_refs"] > l16["num_tris"] + l16["num_spheres"]
    same = (h1[0] == h16[0]) & (h1[1] == h16[1])
    tie = (h1[2].view(np.uint32) == h16[2].view(np.uint32))
    assert (same | tie).all()
    assert same.mean() >= 0.9999
    assert np.array_equal(h1[2][same].view(np.uint32), h16[2][same].view(np.uint32))
    assert np.array_equal(o1, o16)
    assert (rgb1 == rgb16).all(axis=2).mean() >= 0.9999
    assert abs(int(st1.rays_closest) - int(st16.rays_closest)) <= 1e-4 * st1.rays_closest


def test_setter_argument_checks(renderer):
    """The r04 setters refuse out-of-range values with a message and leave the context usable."""
    with pytest.raises(sptr.SptrError, match="straggler lanes"):
        renderer.set_stragglers(65)
    with pytest.raises(sptr.SptrError, match="launch mode"):
        renderer.set_launch_mode(4)
    with pytest.raises(sptr.SptrError, match="split references"):
        renderer.set_split_refs(3)
    renderer.set_stragglers(12)
    renderer.set_launch_mode(0)
    W, H = 64, 48
    sptr.setup_default(renderer, "default")
    st = renderer.render(sptr.camera_lookat(aspect=W / H), W, H, spp=1)
    assert st.samples == W * H


class _DevWords:
    """A device buffer of 32-bit words seen by torch (__cuda_array_interface__)."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes // 4,), "typestr": "<i4", "data": (ptr, False),
                                         "version": 3}


@pytest.mark.parametrize("shard", [(0, 1), (1, 3)])
def test_pixel_lanes_equal_one_chain(renderer, shard):
    """Pixel lanes (sptr_set_pixel_lanes 2): the shard's even and odd tiles rendered as two concurrent
    launch chains by the context and its internal lane context.  The accumulation (read_accum), the
    resolved image, the shard's tile buffer (sptr_tiles_device, the multi-GPU gather's send buffer) and
    the query counts must equal the one-chain render bit for bit — also across a progressive
    continuation, asynchronous calls collected once, and a return to one chain."""
    import torch

    W, H = 320, 200
    R, G = shard
    sptr.setup_default(renderer, "default_emitter")
    cam = sptr.camera_lookat(aspect=W / H)

    def run(lanes):
        renderer.set_pixel_lanes(lanes)
        st1 = renderer.render(cam, W, H, spp=6, shard_rank=R, shard_count=G)
        st2 = renderer.render(cam, W, H, spp=5, frame_begin=7, shard_rank=R, shard_count=G)
        acc = renderer.read_accum().copy()
        rgb = renderer.read_rgb8().copy()
        ptr, nbytes = renderer.tiles_device()
        tiles = torch.as_tensor(_DevWords(ptr, nbytes), device="cuda").cpu().numpy().copy()
        for fb in (1, 4, 7):  # asynchronous calls, one collection
            renderer.render(cam, W, H, spp=3, frame_begin=fb, shard_rank=R, shard_count=G, flags=sptr.SPTR_FRAME_ASYNC)
        st3 = renderer.collect_stats()
        acc3 = renderer.read_accum().copy()
        counts = [(s.rays_closest, s.rays_shadow, s.samples) for s in (st1, st2, st3)]
        return acc, rgb, tiles, acc3, counts

    try:
        one = run(1)
        two = run(2)
        back = run(1)
    finally:
        renderer.set_pixel_lanes(0)
    for a, b in ((one, two), (one, back)):
        assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
        assert np.array_equal(a[1], b[1])
        assert np.array_equal(a[3].view(np.uint32), b[3].view(np.uint32))
        assert a[4] == b[4]
        assert np.array_equal(a[2], b[2])
    assert one[4][0][2] > 0


@pytest.mark.gpu
def test_trace_busy_time(renderer):
    """sptr_stats::ms_trace_busy, the union of the trace launches' intervals: equal to the summed launch
    durations (ms_trace) for one launch chain, and between half of them and all of them for two pixel
    lanes, whose trace launches overlap."""
    W, H = 320, 200
    sptr.setup_default(renderer, "default_emitter")
    cam = sptr.camera_lookat(aspect=W / H)
    try:
        for lanes in (1, 2):
            renderer.set_pixel_lanes(lanes)
            st = renderer.render(cam, W, H, spp=8, flags=sptr.SPTR_FRAME_TIMING_TRACE)
            assert renderer.pixel_lanes_info()["active"] == (lanes == 2)
            assert st.ms_trace > 0 and st.ms_trace_busy > 0
            assert st.ms_trace_busy <= st.ms_trace * 1.001 + 1e-3
            if lanes == 1:
                assert st.ms_trace_busy >= st.ms_trace * 0.999 - 1e-3
            else:
                assert st.ms_trace_busy >= st.ms_trace * 0.5 - 1e-3
    finally:
        renderer.set_pixel_lanes(0)


@pytest.mark.gpu
def test_pixel_lanes_graph_replay(renderer):
    """Pixel lanes in launch mode 3: each lane context captures its repeated call shape into a graph of
    its own (on its own capture stream) and replays it on its lane stream between the fork and the join;
    the accumulation equals one chain's direct launches bit for bit."""
    W, H = 320, 200
    sptr.setup_default(renderer, "default_emitter")
    cam = sptr.camera_lookat(aspect=W / H)

    def run(lanes, mode):
        renderer.set_launch_mode(mode)
        renderer.set_pixel_lanes(lanes)
        g0 = renderer.graph_info()
        for fb in (1, 5, 9, 13):
            renderer.render(cam, W, H, spp=4, frame_begin=fb)
        g = renderer.graph_info()
        return renderer.read_accum().copy(), renderer.read_rgb8().copy(), g["captures"] - g0["captures"], g["valid"]

    try:
        one = run(1, 1)
        two = run(2, 3)
    finally:
        renderer.set_pixel_lanes(0)
        renderer.set_launch_mode(0)
    assert one[2] == 0
    assert two[2] >= 1 and two[3] == 1, "the lane call shape was not captured"
    assert np.array_equal(one[0].view(np.uint32), two[0].view(np.uint32))
    assert np.array_equal(one[1], two[1])


def test_pixel_lanes_follow_shading_changes(renderer):
    """The lane context reads its parent's shading state (materials, lights, environment, debug mode)
    instead of holding copies: after each change — with the lane's launch graph captured before it
    (launch mode 3) — the two-lane image must equal the one-chain image, and must have changed."""
    W, H = 160, 96
    cam = sptr.camera_lookat(aspect=W / H)
    faces = np.random.default_rng(5).random((6, 16, 16, 3), dtype=np.float32) * 2.0

    def run(lanes):
        out = []
        sptr.setup_default(renderer, "default_emitter")
        renderer.set_launch_mode(3)
        renderer.set_pixel_lanes(lanes)
        for step in range(5):
            if step == 1:
                lights = sptr.default_lights()
                lights[0].intensity = 0.5
                renderer.set_lights(lights)
            elif step == 2:
                mats = sptr.preset_materials(True)
                mats[0].albedo[0], mats[0].albedo[1], mats[0].albedo[2] = 0.9, 0.1, 0.1
                renderer.set_materials(mats)
            elif step == 3:
                renderer.set_environment(faces)
            elif step == 4:
                renderer.set_debug_mode(1)
            for _ in range(3):  # (the shape is captured on its second call and replayed on its third)
                renderer.render(cam, W, H, spp=4)
            out.append(renderer.read_rgb8().copy())
        renderer.set_debug_mode(0)
        renderer.set_environment(None)
        return out

    try:
        one = run(1)
        two = run(2)
    finally:
        renderer.set_pixel_lanes(0)
        renderer.set_launch_mode(0)
        renderer.set_debug_mode(0)
    for i, (a, b) in enumerate(zip(one, two)):
        assert np.array_equal(a, b), f"step {i}: two lanes differ from one chain"
        if i:
            assert not np.array_equal(two[i], two[i - 1]), f"step {i}: the change had no effect"


@pytest.mark.gpu
def test_ray_accounting_fused_bounces(renderer):
    """Every closest-hit query is a camera ray (one per sample, culled or not), a bounce ray of a trace
    launch (traced_bounce), of a fused bounce launch (traced_fused: k_bounce) or of the path-per-thread
    tail (rays_tail); the per-bounce counts cover the traversed ones."""
    W, H = 320, 200
    sptr.setup_default(renderer, "default_emitter")
    cam = sptr.camera_lookat(aspect=W / H)
    st = renderer.render(cam, W, H, spp=8, flags=sptr.SPTR_FRAME_TIMING_TRACE)
    assert st.traced_fused > 0, "the small LDS-scene call is expected to fuse its bounces"
    assert st.rays_closest == st.samples + st.traced_bounce + st.traced_fused + st.rays_tail
    assert sum(st.traced_by_depth) == st.traced_primary + st.traced_bounce + st.traced_fused
    assert st.trace_launches > 1 and st.ms_trace > 0


@pytest.mark.gpu
def test_pixel_lanes_scene_changes(renderer):
    """Two lanes apply to scenes staged into LDS only (a 40 000-triangle mesh renders as one chain even
    when two lanes are asked for), and a scene upload in the middle of a two-lane accumulation starts
    the next one afresh: the default scene rendered again after the mesh equals its first render."""
    W, H = 320, 200
    cam = sptr.camera_lookat(aspect=W / H)
    try:
        renderer.set_pixel_lanes(2)
        sptr.setup_default(renderer, "default_emitter")
        renderer.render(cam, W, H, spp=4)
        assert renderer.pixel_lanes_info()["active"]
        first = renderer.read_accum().copy()
        sptr.setup_default(renderer, "sphere_mesh", 100, 200)
        assert renderer.scene_layout()["lds_bytes"] == 0
        renderer.render(cam, W, H, spp=4)
        assert not renderer.pixel_lanes_info()["active"]
        sptr.setup_default(renderer, "default_emitter")
        renderer.render(cam, W, H, spp=4)
        assert renderer.pixel_lanes_info()["active"]
        assert np.array_equal(first.view(np.uint32), renderer.read_accum().view(np.uint32))
    finally:
        renderer.set_pixel_lanes(0)
