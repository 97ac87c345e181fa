"""CPU: the product library's host side — C ABI exports, host scene layer vs the oracle (bit
equality), index math, tile packing, HDR and glTF readers.  No GPU calls."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
import sptr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    text = open(os.path.join(ROOT, "include", "sptr_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sptr_\w+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = sptr.lib()
    names = _header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(sptr.EXPORTS)
    assert L.sptr_abi_version() == 9


def test_no_device_means_loud_failure():
    """Without a GPU the renderer refuses to start (there is no CPU fallback)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(sptr.SptrError):
        sptr.Renderer(0)


@pytest.mark.parametrize("name,p0,p1", [("default", 0, 0), ("default_emitter", 0, 0), ("test_triangle", 0, 0),
                                        ("sphere_mesh", 30, 70)])
def test_builtin_scenes_bit_equal_to_oracle(name, p0, p1):
    a, b = sptr.builtin_scene(name, p0, p1), oracle.builtin_scene(name, p0, p1)
    for k in ("positions", "indices", "tri_geom_first", "spheres", "geom_material"):
        x, y = getattr(a, k), b[k]
        assert x.shape == y.shape, k
        assert np.array_equal(x.view(np.uint32) if x.dtype == np.float32 else x,
                              y.view(np.uint32) if y.dtype == np.float32 else y), k


def test_default_scene_layout():
    s = sptr.builtin_scene("default")
    assert s.indices.shape == (12, 3) and s.spheres.shape == (8, 4)
    assert list(s.geom_material) == [4, 0, 1, 2, 3, 5, 6, 7, 8]  # glass cube instance, then spheres
    assert np.allclose(s.positions.min(0), [-0.75, 0.25, 1.25]) and np.allclose(s.positions.max(0), [0.75, 1.75, 2.75])


@pytest.mark.parametrize("aspect", [800 / 600, 1920 / 1080, 1.0, 75 / 41])
def test_camera_bit_equal_to_oracle(aspect):
    a = sptr.camera_lookat(aspect=aspect).as_array()
    b = oracle.camera(aspect=aspect)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_presets_and_lights_equal_oracle():
    for wl in (False, True):
        assert np.array_equal(sptr.materials_as_array(sptr.preset_materials(wl)), oracle.preset_materials(wl))
    assert np.array_equal(sptr.lights_as_array(sptr.default_lights()), oracle.default_lights())
    glass = sptr.preset_materials(False)[4]
    assert glass.roughness == np.float32(0.01)  # Material ctor clamp (Material.h:36-38)
    light = sptr.preset_materials(True)[9]
    assert list(light.emission) == [5.0, 5.0, 5.0] and light.ior == np.float32(1.5)


def test_equirect_faces_equal_oracle():
    g = np.random.default_rng(1)
    eq = g.uniform(0, 4, size=(64, 128, 3)).astype(np.float32)
    assert np.array_equal(sptr.equirect_to_faces(eq, 32), oracle.equirect_to_faces(eq, 32))


def test_index_math_cpp(tmp_path):
    exe = tmp_path / "tim"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "simple-path-tracer_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "test_index_math.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout


@pytest.mark.parametrize("W,H,G", [(64, 64, 1), (75, 41, 2), (150, 70, 3), (1920, 1080, 8), (33, 31, 5)])
def test_tile_pack_unpack_roundtrip(W, H, G):
    g = np.random.default_rng(W * H + G)
    img = g.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    tpr = sptr.tiles_per_rank(W, H, G)
    gathered = np.concatenate([sptr.pack_tiles(img, G, r) for r in range(G)])
    assert gathered.size == G * tpr * 1024
    assert np.array_equal(sptr.unpack_tiles(gathered, G, W, H), img)


def _write_hdr(path, rgbe, rle):
    h, w = rgbe.shape[:2]
    with open(path, "wb") as f:
        f.write(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n")
        f.write(f"-Y {h} +X {w}\n".encode())
        for y in range(h):
            row = rgbe[y]
            if not rle:
                f.write(row.tobytes())
                continue
            f.write(bytes([2, 2, w >> 8, w & 0xFF]))
            for c in range(4):
                ch = row[:, c]
                x = 0
                while x < w:  # alternate a run and a literal block to exercise both codes
                    run = 1
                    while x + run < w and run < 127 and ch[x + run] == ch[x]:
                        run += 1
                    if run >= 3:
                        f.write(bytes([128 + run, ch[x]]))
                        x += run
                    else:
                        n = min(128, w - x)
                        f.write(bytes([n]) + ch[x:x + n].tobytes())
                        x += n


@pytest.mark.parametrize("rle", [False, True])
def test_hdr_reader(tmp_path, rle):
    g = np.random.default_rng(3)
    h, w = 12, 40
    rgbe = g.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    rgbe[:, :10, :] = rgbe[:, :1, :]  # runs
    rgbe[3, 5, 3] = 0
    p = tmp_path / "t.hdr"
    _write_hdr(p, rgbe, rle)
    img = sptr.load_hdr(str(p))
    scale = np.ldexp(1.0, rgbe[..., 3].astype(np.int32) - 136).astype(np.float32)
    expect = np.where(rgbe[..., 3:4] == 0, 0, rgbe[..., :3].astype(np.float32) * scale[..., None])
    assert np.array_equal(img, expect.astype(np.float32))


def test_gltf_chair_scene():
    path = os.path.join(ROOT, "assets", "rattan_dining_chair", "scene.gltf")
    s = sptr.builtin_scene("gltf:" + path, 7)
    # 1 mesh, 1 triangle primitive: 18348 indices = 6116 triangles, 3617 vertices
    assert s.indices.shape == (6116, 3) and s.positions.shape == (3617, 3)
    assert list(s.geom_material) == [7] and s.spheres.shape == (0, 4)
    lo, hi = s.positions.min(0), s.positions.max(0)
    # node matrices turn the Z-up model into Y-up at 0.01 scale: roughly chair-sized, standing on y
    assert 0.3 < hi[1] - lo[1] < 1.5 and abs(lo[1]) < 0.05
