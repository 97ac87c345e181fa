"""The BASELINE.json configurations as renderer setups (SURVEY.md §8(d) "Configs -> synthetic inputs").

  c1  default scene, 256x256, 4 spp                       (the reference's CPU plumbing case)
  c2  default scene + emissive sphere, 1920x1080, 64 spp   (bench.py's headline workload)
  c3  rattan chair glTF (6116 tris, Wood) + synthetic HDR sky, 1920x1080, 256 spp
  c4  default scene, 3840x2160, 1024 spp                   (the 8-GPU tile-sharded case)
  c5  default scene with the glass cube replaced by a 1250x4000 sphere mesh = 10M triangles,
      1920x1080, 64 spp                                     (the HBM roofline run)

All inputs are synthetic and deterministic: the reference's procedural scenes, and for c3 an
analytic equirect sky (the reference's HDRs are missing blobs) encoded as a
Radiance .hdr and read back through the product's reader (Cubemap::loadFromFile path).
"""
from __future__ import annotations

import os
import tempfile
from dataclasses import dataclass

import numpy as np

import sptr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHAIR = os.path.join(ROOT, "assets", "rattan_dining_chair", "scene.gltf")


@dataclass(frozen=True)
class Workload:
    name: str
    scene: str
    p0: int
    p1: int
    width: int
    height: int
    spp: int
    max_depth: int = 6
    hdr_env: bool = False
    description: str = ""


WORKLOADS = {
    "c1": Workload("c1", "default", 0, 0, 256, 256, 4, description="C1: default scene, 256x256, 4 spp, depth 6"),
    "c2": Workload("c2", "default_emitter", 0, 0, 1920, 1080, 64,
                   description="C2: default scene + emitter, 1920x1080, 64 spp, depth 6"),
    "c3": Workload("c3", "gltf:" + CHAIR, 7, 0, 1920, 1080, 256, hdr_env=True,
                   description="C3: rattan chair glTF (6116 tris) + synthetic HDR env, 1920x1080, 256 spp, depth 6"),
    "c4": Workload("c4", "default", 0, 0, 3840, 2160, 1024,
                   description="C4: default scene, 3840x2160, 1024 spp, depth 6"),
    "c5": Workload("c5", "sphere_mesh", 1250, 4000, 1920, 1080, 64,
                   description="C5: default scene with a 10M-triangle sphere mesh, 1920x1080, 64 spp, depth 6"),
}


def synthetic_sky_equirect(width: int = 2048, height: int = 1024) -> np.ndarray:
    """Analytic HDR sky as float RGB (height, width, 3): zenith/horizon gradient, a bright sun disc
    (radiance ~40, above the reference's clamp of 5) and a dim ground.  Row 0 is the zenith, as
    Cubemap::loadEquirectangular expects (v = acos(y)/pi)."""
    v = (np.arange(height, dtype=np.float64) + 0.5) / height
    u = (np.arange(width, dtype=np.float64) + 0.5) / width
    theta = v[:, None] * np.pi
    phi = u[None, :] * 2.0 * np.pi - np.pi
    y = np.cos(theta) * np.ones_like(phi)
    x = np.sin(theta) * np.cos(phi)
    z = np.sin(theta) * np.sin(phi)
    up = np.clip(y, 0.0, 1.0)[..., None]
    sky = (1 - up) * np.array([1.1, 1.05, 1.0]) + up * np.array([0.25, 0.45, 1.2])
    ground = np.array([0.18, 0.15, 0.12]) * np.ones_like(sky)
    img = np.where((y >= 0)[..., None], sky, ground)
    sun = np.array([0.4, 0.55, -0.73])
    sun /= np.linalg.norm(sun)
    cosang = x * sun[0] + y * sun[1] + z * sun[2]
    img = img + (cosang > np.cos(np.radians(2.5)))[..., None] * np.array([40.0, 36.0, 30.0])
    return img.astype(np.float32)


def write_hdr(path: str, rgb: np.ndarray) -> None:
    """Flat (non-RLE) Radiance RGBE writer, -Y H +X W."""
    rgb = np.asarray(rgb, np.float32)
    h, w = rgb.shape[:2]
    m = rgb.max(axis=2)
    e = np.zeros(m.shape, np.int32)
    mant, ex = np.frexp(m)
    ok = m >= 1e-32
    e[ok] = ex[ok]
    scale = np.where(ok, np.ldexp(1.0, 8 - e), 0.0)
    rgbe = np.zeros((h, w, 4), np.uint8)
    rgbe[..., :3] = np.clip(np.floor(rgb * scale[..., None]), 0, 255).astype(np.uint8)
    rgbe[..., 3] = np.where(ok, e + 128, 0).astype(np.uint8)
    with open(path, "wb") as f:
        f.write(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n")
        f.write(f"-Y {h} +X {w}\n".encode())
        f.write(rgbe.tobytes())


_ENV_CACHE: dict = {}


def hdr_env_faces(face_size: int = 512) -> np.ndarray:
    """Synthetic sky -> .hdr file -> product HDR reader -> equirect-to-cubemap faces."""
    if face_size not in _ENV_CACHE:
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "sky.hdr")
            write_hdr(p, synthetic_sky_equirect())
            eq = sptr.load_hdr(p)
        _ENV_CACHE[face_size] = sptr.equirect_to_faces(eq, face_size)
    return _ENV_CACHE[face_size]


def setup(r: "sptr.Renderer", wl: Workload) -> "sptr.FlatScene":
    """Upload the workload's scene and the reference's default state; returns the flat scene."""
    return sptr.setup_default(r, wl.scene, wl.p0, wl.p1, env_faces=hdr_env_faces() if wl.hdr_env else None)


def camera(wl: Workload) -> "sptr.Camera":
    return sptr.camera_lookat(aspect=wl.width / wl.height)
