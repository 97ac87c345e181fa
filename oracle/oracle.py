"""TEST INFRASTRUCTURE ONLY — ctypes access to oracle/liboracle.so, the CPU restatement of the
reference's Embree-backend wavefront path tracer (see wf_oracle.cpp's header for the reference
file:line list).  Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg; the product (simple-path-tracer_amd/) never loads it.

PARITY UNPINNED: the reference ships no tests or golden vectors and cannot be built here, so the
oracle is a restatement checked for internal consistency and against committed fixtures it produced.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


class SceneIn(C.Structure):
    _fields_ = [
        ("positions", C.POINTER(C.c_float)), ("num_verts", C.c_uint32),
        ("indices", C.POINTER(C.c_uint32)), ("num_tris", C.c_uint32),
        ("tri_geom_first", C.POINTER(C.c_uint32)), ("num_tri_geoms", C.c_uint32),
        ("spheres", C.POINTER(C.c_float)), ("num_spheres", C.c_uint32),
        ("geom_material", C.POINTER(C.c_uint32)),
    ]


class Job(C.Structure):
    _fields_ = [
        ("materials", C.POINTER(C.c_float)), ("num_materials", C.c_uint32),
        ("lights", C.POINTER(C.c_float)), ("num_lights", C.c_uint32),
        ("env_faces", C.POINTER(C.c_float)), ("env_size", C.c_int32),
        ("env_intensity", C.c_float), ("env_clamp", C.c_float),
        ("cam", C.c_float * 14), ("width", C.c_int32), ("height", C.c_int32),
        ("frame_begin", C.c_uint32), ("num_frames", C.c_uint32), ("max_depth", C.c_uint32),
        ("shard_rank", C.c_int32), ("shard_count", C.c_int32), ("threads", C.c_int32), ("use_bvh", C.c_int32),
        ("accum", C.POINTER(C.c_float)), ("rgb", C.POINTER(C.c_uint8)), ("counters", C.c_uint64 * 4),
        ("pixels", C.POINTER(C.c_uint32)), ("num_pixels", C.c_uint32),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, fp, up, bp = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)
        sig = {
            "oracle_version": (C.c_int, []),
            "oracle_wang_hash": (C.c_uint32, [C.c_uint32]),
            "oracle_rand_stream": (None, [C.c_uint32, C.c_uint32, fp, up]),
            "oracle_prepare": (vp, [C.POINTER(SceneIn), C.c_int]),
            "oracle_release": (None, [vp]),
            "oracle_builtin_scene": (vp, [C.c_int, C.c_uint32, C.c_uint32]),
            "oracle_flat_view": (None, [vp, C.POINTER(SceneIn)]),
            "oracle_flat_free": (None, [vp]),
            "oracle_preset_materials": (C.c_int, [C.c_int, fp, C.c_int]),
            "oracle_camera": (None, [fp, fp, C.c_float, C.c_float, fp]),
            "oracle_primary": (None, [fp, C.c_int, C.c_int, C.c_uint32, fp, up]),
            "oracle_intersect": (None, [vp, fp, C.c_uint32, C.c_int, up, up, fp, fp]),
            "oracle_occluded": (None, [vp, fp, C.c_uint32, C.c_int, bp]),
            "oracle_env": (None, [fp, C.c_int, C.c_float, C.c_float, fp, C.c_uint32, fp]),
            "oracle_equirect_to_faces": (None, [fp, C.c_int, C.c_int, C.c_int, fp]),
            "oracle_render": (C.c_int, [vp, C.POINTER(Job)]),
            "oracle_render_pt": (C.c_int, [vp, C.POINTER(Job), C.c_uint32]),
            "oracle_render_optix": (C.c_int, [vp, C.POINTER(Job), fp]),
            "oracle_resolve": (None, [fp, C.c_uint32, C.c_uint32, bp]),
            "oracle_set_device_math": (None, [fp, C.c_int]),
            "oracle_path_rays": (C.c_int, [vp, C.POINTER(Job), C.c_int, C.c_int, C.c_uint32, fp, C.c_int]),
        }
        for n, (r, a) in sig.items():
            f = getattr(L, n)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _u(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def _b(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


BUILTIN = {"default": 0, "default_emitter": 1, "sphere_mesh": 2, "test_triangle": 3}


def builtin_scene(name: str, stacks: int = 0, slices: int = 0) -> dict:
    """The oracle's own restatement of the builtin scenes, flattened (numpy copies)."""
    L = lib()
    h = L.oracle_builtin_scene(BUILTIN[name], stacks, slices)
    try:
        v = SceneIn()
        L.oracle_flat_view(h, C.byref(v))

        def arr(p, n, dt):
            return np.ctypeslib.as_array(p, shape=(n,)).copy().astype(dt) if n else np.zeros(0, dt)
        return {
            "positions": arr(v.positions, v.num_verts * 3, np.float32).reshape(-1, 3),
            "indices": arr(v.indices, v.num_tris * 3, np.uint32).reshape(-1, 3),
            "tri_geom_first": arr(v.tri_geom_first, v.num_tri_geoms + 1, np.uint32),
            "spheres": arr(v.spheres, v.num_spheres * 4, np.float32).reshape(-1, 4),
            "geom_material": arr(v.geom_material, v.num_tri_geoms + v.num_spheres, np.uint32),
        }
    finally:
        L.oracle_flat_free(h)


def preset_materials(with_light: bool = False) -> np.ndarray:
    out = np.zeros((16, 12), np.float32)
    n = lib().oracle_preset_materials(1 if with_light else 0, _f(out), 16)
    return out[:n].copy()


def camera(pos=(0.0, 3.0, 8.0), target=(0.0, 1.0, 0.0), fov=60.0, aspect=800 / 600) -> np.ndarray:
    out = np.zeros(14, np.float32)
    p = np.array(pos, np.float32)
    t = np.array(target, np.float32)
    lib().oracle_camera(_f(p), _f(t), C.c_float(fov), C.c_float(aspect), _f(out))
    return out


def default_lights() -> np.ndarray:
    # setupLights (src/main.cpp:85-94): type, direction, color, intensity
    return np.array([[0, -0.5, -1.0, 0.3, 1.0, 0.95, 0.8, 2.0]], np.float32)


class Prepared:
    """A flattened scene prepared for intersection (optionally with the CPU BVH)."""

    def __init__(self, scene: dict, bvh: bool = True):
        self._keep = [np.ascontiguousarray(scene["positions"], np.float32),
                      np.ascontiguousarray(scene["indices"], np.uint32),
                      np.ascontiguousarray(scene["tri_geom_first"], np.uint32),
                      np.ascontiguousarray(scene["spheres"], np.float32),
                      np.ascontiguousarray(scene["geom_material"], np.uint32)]
        p, i, g, s, m = self._keep
        sin = SceneIn(_f(p), len(p), _u(i), len(i), _u(g), len(g) - 1, _f(s), len(s), _u(m))
        self.bvh = bvh
        self.h = lib().oracle_prepare(C.byref(sin), 1 if bvh else 0)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_release(self.h)
            self.h = None

    def intersect(self, rays: np.ndarray, use_bvh: bool | None = None):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        n = len(rays)
        geom, prim = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        t, ng = np.zeros(n, np.float32), np.zeros((n, 3), np.float32)
        ub = self.bvh if use_bvh is None else use_bvh
        lib().oracle_intersect(self.h, _f(rays), n, 1 if ub else 0, _u(geom), _u(prim), _f(t), _f(ng))
        return geom, prim, t, ng

    def occluded(self, rays: np.ndarray, use_bvh: bool | None = None) -> np.ndarray:
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        out = np.zeros(len(rays), np.uint8)
        ub = self.bvh if use_bvh is None else use_bvh
        lib().oracle_occluded(self.h, _f(rays), len(rays), 1 if ub else 0, _b(out))
        return out

    def path_rays(self, cam: np.ndarray, width: int, height: int, materials: np.ndarray, lights: np.ndarray,
                  x: int, y: int, frame: int, max_depth: int = 6, env_faces: np.ndarray | None = None,
                  env_intensity: float = 0.8, env_clamp: float = 5.0):
        """The rays of pixel (x, y)'s wavefront path at accumulation index `frame`, in trace order:
        (kinds (n,) 0 closest hit / 1 shadow, rays (n, 8) float32 o3 d3 tnear tfar) — residue diagnosis."""
        mats = np.ascontiguousarray(materials, np.float32)
        lts = np.ascontiguousarray(lights, np.float32)
        j = Job()
        j.materials, j.num_materials = _f(mats), len(mats)
        j.lights, j.num_lights = _f(lts), len(lts)
        if env_faces is not None:
            ef = np.ascontiguousarray(env_faces, np.float32)
            j.env_faces, j.env_size = _f(ef), ef.shape[1]
        j.env_intensity, j.env_clamp = env_intensity, env_clamp
        j.cam[:] = [float(v) for v in cam]
        j.width, j.height, j.max_depth = width, height, max_depth
        j.use_bvh = 1 if self.bvh else 0
        out = np.zeros((64, 9), np.float32)
        n = lib().oracle_path_rays(self.h, C.byref(j), x, y, frame, _f(out), 64)
        if n < 0:
            raise RuntimeError("oracle_path_rays")
        out = out[:min(n, 64)]
        return out[:, 0].astype(np.int32), np.ascontiguousarray(out[:, 1:9])

    def render(self, cam: np.ndarray, width: int, height: int, materials: np.ndarray, lights: np.ndarray,
               frames: int = 1, frame_begin: int = 1, max_depth: int = 6, shard_rank: int = 0,
               shard_count: int = 1, threads: int = 0, env_faces: np.ndarray | None = None,
               env_intensity: float = 0.8, env_clamp: float = 5.0, accum: np.ndarray | None = None,
               pathtracer_spf: int = 0, optix: bool = False, accum_w: np.ndarray | None = None,
               pixels: np.ndarray | None = None):
        """Returns (accum (H,W,3) float32 sums, rgb8 (H,W,3), counters dict).  pathtracer_spf > 0 selects
        the PathTracer integrator (the reference's default CPU path) with that many samples per frame;
        optix=True the OptiX device-program shading (accum_w: the per-pixel sample counts, (H,W) float32,
        returned as the 4th counters key "accum_w").  pixels (wavefront only): render just these pixel
        indices y * width + x; the other accum / rgb entries stay as given."""
        mats = np.ascontiguousarray(materials, np.float32)
        lts = np.ascontiguousarray(lights, np.float32)
        acc = np.zeros((height, width, 3), np.float32) if accum is None else np.ascontiguousarray(accum, np.float32)
        rgb = np.zeros((height, width, 3), np.uint8)
        j = Job()
        j.materials, j.num_materials = _f(mats), len(mats)
        j.lights, j.num_lights = _f(lts), len(lts)
        if env_faces is not None:
            ef = np.ascontiguousarray(env_faces, np.float32)
            j.env_faces, j.env_size = _f(ef), ef.shape[1]
        j.env_intensity, j.env_clamp = env_intensity, env_clamp
        j.cam[:] = [float(x) for x in cam]
        j.width, j.height = width, height
        j.frame_begin, j.num_frames, j.max_depth = frame_begin, frames, max_depth
        j.shard_rank, j.shard_count = shard_rank, shard_count
        j.threads, j.use_bvh = threads, 1 if self.bvh else 0
        j.accum, j.rgb = _f(acc), _b(rgb)
        if pixels is not None:
            pix = np.ascontiguousarray(pixels, np.uint32)
            j.pixels, j.num_pixels = _u(pix), len(pix)
        aw = None
        if optix:
            aw = np.zeros((height, width), np.float32) if accum_w is None else np.ascontiguousarray(accum_w, np.float32)
            rc = lib().oracle_render_optix(self.h, C.byref(j), _f(aw))
        elif pathtracer_spf:
            rc = lib().oracle_render_pt(self.h, C.byref(j), pathtracer_spf)
        else:
            rc = lib().oracle_render(self.h, C.byref(j))
        if rc != 0:
            raise RuntimeError(f"oracle_render rc={rc}")
        c = list(j.counters)
        out = {"rays_closest": c[0], "rays_shadow": c[1], "samples": c[2]}
        if aw is not None:
            out["accum_w"] = aw
        return acc, rgb, out


class device_math:
    """Context manager for the residue diagnosis: the oracle's wavefront path takes the GPU's values
    for the cosine sample's sin/cos (sin_cos: (2^24, 2) float32 from sptr.Renderer.cosine_sincos_table,
    or None) and the GPU's double squaring chains for pow(x, 5/8/64) (pow_chains)."""

    def __init__(self, sin_cos: np.ndarray | None = None, pow_chains: bool = False):
        self.tab = None if sin_cos is None else np.ascontiguousarray(sin_cos, np.float32)
        assert self.tab is None or self.tab.shape == (1 << 24, 2)
        self.pow_chains = pow_chains

    def __enter__(self):
        lib().oracle_set_device_math(None if self.tab is None else _f(self.tab), 1 if self.pow_chains else 0)
        return self

    def __exit__(self, *exc):
        lib().oracle_set_device_math(None, 0)
        return False


def primary(cam: np.ndarray, width: int, height: int, acc: int):
    dirs = np.zeros((height, width, 3), np.float32)
    rng = np.zeros((height, width), np.uint32)
    c = np.ascontiguousarray(cam, np.float32)
    lib().oracle_primary(_f(c), width, height, acc, _f(dirs), _u(rng))
    return dirs, rng


def rand_stream(seed: int, n: int):
    out = np.zeros(n, np.float32)
    st = np.zeros(n, np.uint32)
    lib().oracle_rand_stream(seed, n, _f(out), _u(st))
    return out, st


def wang_hash(a: int) -> int:
    return lib().oracle_wang_hash(a)


def env(dirs: np.ndarray, faces: np.ndarray | None = None, intensity=0.8, clamp=5.0) -> np.ndarray:
    d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
    out = np.zeros_like(d)
    if faces is None:
        lib().oracle_env(None, 0, intensity, clamp, _f(d), len(d), _f(out))
    else:
        f = np.ascontiguousarray(faces, np.float32)
        lib().oracle_env(_f(f), f.shape[1], intensity, clamp, _f(d), len(d), _f(out))
    return out


def equirect_to_faces(rgb: np.ndarray, size: int) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, np.float32)
    h, w = rgb.shape[:2]
    faces = np.zeros((6, size, size, 3), np.float32)
    lib().oracle_equirect_to_faces(_f(rgb), w, h, size, _f(faces))
    return faces


def resolve(accum: np.ndarray, n: int) -> np.ndarray:
    a = np.ascontiguousarray(accum, np.float32)
    out = np.zeros(a.shape[:-1] + (3,), np.uint8)
    lib().oracle_resolve(_f(a), a.size // 3, n, _b(out))
    return out
