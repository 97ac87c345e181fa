"""sptr — Python (ctypes) binding of libsptr_hip.so, the MI355X wavefront path-tracing backend.

This is the ctypes form of the binding a reference-side maintainer would add:
every call goes straight to the C ABI in include/sptr_hip.h.  There is no CPU fallback: if the
library is missing or no GPU is present, constructing a Renderer raises.

Reference mapping: Renderer mirrors backends::OptixBackend (include/backends/OptixBackend.h:39-71)
with the CPU wavefront integrator's semantics (src/wavefront/wf_pt_cpu.cpp:61-255).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPTR_LIB") or os.path.join(HERE, "libsptr_hip.so")  # SPTR_LIB: A/B builds

SPTR_ABI_VERSION = 9  # include/sptr_hip.h
SPTR_FRAME_TIMING = 1
SPTR_FRAME_NO_RESOLVE = 2
SPTR_FRAME_COUNT_VISITS = 4
SPTR_FRAME_ASYNC = 8
SPTR_FRAME_TIMING_TRACE = 16
SPTR_FRAME_NO_CULL = 32
SPTR_FRAME_RECULL = 64

SPTR_INTEGRATOR_WAVEFRONT = 0   # WavefrontPathTracerCPU semantics (default)
SPTR_INTEGRATOR_PATHTRACER = 1  # PathTracer (the reference's default CPU integrator) semantics
SPTR_INTEGRATOR_OPTIX = 2       # the reference's OptiX device-program shading (GPU 'G' path)


class SptrError(RuntimeError):
    pass


class Scene(C.Structure):
    _fields_ = [
        ("positions", C.POINTER(C.c_float)), ("num_verts", C.c_uint32),
        ("indices", C.POINTER(C.c_uint32)), ("num_tris", C.c_uint32),
        ("tri_geom_first", C.POINTER(C.c_uint32)), ("num_tri_geoms", C.c_uint32),
        ("spheres", C.POINTER(C.c_float)), ("num_spheres", C.c_uint32),
        ("geom_material", C.POINTER(C.c_uint32)),
    ]


class Material(C.Structure):
    _fields_ = [("albedo", C.c_float * 3), ("metallic", C.c_float), ("roughness", C.c_float),
                ("emission", C.c_float * 3), ("ior", C.c_float), ("type", C.c_int32), ("pad", C.c_float * 2)]


class Light(C.Structure):
    _fields_ = [("type", C.c_int32), ("v", C.c_float * 3), ("color", C.c_float * 3), ("intensity", C.c_float)]


class Environment(C.Structure):
    _fields_ = [("faces", C.POINTER(C.c_float)), ("size", C.c_int32), ("intensity", C.c_float),
                ("max_clamp", C.c_float)]


class Camera(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("forward", C.c_float * 3), ("right", C.c_float * 3),
                ("up", C.c_float * 3), ("half_width", C.c_float), ("half_height", C.c_float)]

    def as_array(self) -> np.ndarray:
        return np.array(list(self.pos) + list(self.forward) + list(self.right) + list(self.up)
                        + [self.half_width, self.half_height], dtype=np.float32)


class Frame(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("camera", Camera), ("frame_begin", C.c_uint32),
                ("spp", C.c_uint32), ("max_depth", C.c_uint32), ("shard_rank", C.c_int32),
                ("shard_count", C.c_int32), ("flags", C.c_uint32), ("integrator", C.c_uint32),
                ("samples_per_frame", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("rays_closest", C.c_uint64), ("rays_shadow", C.c_uint64), ("samples", C.c_uint64),
                ("waves", C.c_uint64), ("ms_total", C.c_double), ("ms_raygen", C.c_double),
                ("ms_trace", C.c_double), ("ms_shade", C.c_double), ("ms_shadow", C.c_double),
                ("ms_accum", C.c_double), ("trace_launches", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("sphere_tests", C.c_uint64), ("shadow_node_visits", C.c_uint64),
                ("shadow_prim_tests", C.c_uint64), ("ms_trace0", C.c_double), ("ms_shade0", C.c_double),
                ("rays_tail", C.c_uint64), ("ms_tail", C.c_double), ("traced_primary", C.c_uint64),
                ("traced_bounce", C.c_uint64), ("node_visits_primary", C.c_uint64),
                ("tri_tests_primary", C.c_uint64), ("sphere_tests_primary", C.c_uint64), ("ms_cull", C.c_double),
                ("cull_launches", C.c_uint64), ("shadow_launches", C.c_uint64),
                ("traced_by_depth", C.c_uint64 * 8), ("nodes_by_depth", C.c_uint64 * 8),
                ("trace_visit_hist", C.c_uint64 * 16), ("shadow_visit_hist", C.c_uint64 * 16),
                ("hits_primary", C.c_uint64), ("hits_bounce", C.c_uint64), ("paths_handed_off", C.c_uint64), ("strag_visits", C.c_uint64 * 3),
                ("ms_trace_busy", C.c_double), ("traced_fused", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: (list(v) if isinstance(v, C.Array) else v) for k, v in ((k, getattr(self, k)) for k, _ in self._fields_)}


class SceneLayout(C.Structure):
    _fields_ = [("num_tris", C.c_uint32), ("num_spheres", C.c_uint32), ("num_nodes", C.c_uint32),
                ("leaf_size", C.c_uint32), ("bvh_depth", C.c_uint32), ("lds_bytes", C.c_uint32),
                ("node_bytes", C.c_uint64), ("tri_bytes", C.c_uint64), ("sphere_bytes", C.c_uint64),
                ("prim_ref_bytes", C.c_uint64), ("bvh_width", C.c_uint32), ("num_prim_refs", C.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None

# every symbol include/sptr_hip.h declares
EXPORTS = [
    "sptr_abi_version", "sptr_create", "sptr_destroy", "sptr_last_error", "sptr_set_debug_mode",
    "sptr_set_wave_paths", "sptr_set_launch_mode", "sptr_set_pixel_lanes", "sptr_pixel_lanes_info", "sptr_graph_info", "sptr_capture_error", "sptr_overlap_probe", "sptr_set_tail_depth", "sptr_set_leaf_size", "sptr_set_split_refs", "sptr_set_stragglers", "sptr_set_bvh_width", "sptr_upload_scene", "sptr_set_materials", "sptr_set_lights",
    "sptr_set_environment", "sptr_scene_info", "sptr_scene_layout_info", "sptr_render", "sptr_collect_stats",
    "sptr_read_rgb8", "sptr_read_rgb8_lagged",
    "sptr_read_accum",
    "sptr_tiles_device", "sptr_unpack_tiles", "sptr_intersect", "sptr_occluded", "sptr_primary_rays",
    "sptr_sort_pairs_u64", "sptr_scan_u32", "sptr_eval_math",
    "sptr_host_builtin_scene", "sptr_host_scene_view", "sptr_host_scene_free", "sptr_host_camera_lookat",
    "sptr_host_preset_materials", "sptr_host_default_lights", "sptr_host_equirect_to_faces",
    "sptr_host_pack_tiles", "sptr_host_unpack_tiles", "sptr_host_load_hdr", "sptr_host_free",
]


def lib() -> C.CDLL:
    """Load libsptr_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SptrError(f"{LIB_PATH} not built (run make in simple-path-tracer_amd/)")
    L = C.CDLL(LIB_PATH)
    vp, i32, u32, u64 = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64
    fp, up, bp = C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)
    sig = {
        "sptr_abi_version": (C.c_int, []),
        "sptr_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "sptr_destroy": (C.c_int, [vp]),
        "sptr_last_error": (C.c_char_p, [vp]),
        "sptr_set_debug_mode": (C.c_int, [vp, C.c_int]),
        "sptr_set_wave_paths": (C.c_int, [vp, u64]),
        "sptr_set_launch_mode": (C.c_int, [vp, u32]),
        "sptr_set_pixel_lanes": (C.c_int, [vp, u32]),
        "sptr_pixel_lanes_info": (C.c_int, [vp, C.POINTER(u32), C.POINTER(u32)]),
        "sptr_graph_info": (C.c_int, [vp, up, up, up, up, up, C.POINTER(C.c_int32)]),
        "sptr_capture_error": (C.c_char_p, [vp]),
        "sptr_overlap_probe": (C.c_int, [vp, C.POINTER(C.c_double)]),
        "sptr_set_tail_depth": (C.c_int, [vp, u32]),
        "sptr_set_leaf_size": (C.c_int, [vp, u32]),
        "sptr_set_split_refs": (C.c_int, [vp, u32]),
        "sptr_set_stragglers": (C.c_int, [vp, u32]),
        "sptr_set_bvh_width": (C.c_int, [vp, u32]),
        "sptr_upload_scene": (C.c_int, [vp, C.POINTER(Scene)]),
        "sptr_set_materials": (C.c_int, [vp, C.POINTER(Material), u32]),
        "sptr_set_lights": (C.c_int, [vp, C.POINTER(Light), u32]),
        "sptr_set_environment": (C.c_int, [vp, C.POINTER(Environment)]),
        "sptr_scene_info": (C.c_int, [vp, up, up, up, C.POINTER(C.c_double)]),
        "sptr_scene_layout_info": (C.c_int, [vp, C.POINTER(SceneLayout)]),
        "sptr_render": (C.c_int, [vp, C.POINTER(Frame), vp, C.POINTER(Stats)]),
        "sptr_collect_stats": (C.c_int, [vp, C.POINTER(Stats)]),
        "sptr_read_rgb8": (C.c_int, [vp, bp]),
        "sptr_read_rgb8_lagged": (C.c_int, [vp, bp, C.POINTER(u32)]),
        "sptr_read_accum": (C.c_int, [vp, fp]),
        "sptr_tiles_device": (C.c_int, [vp, C.POINTER(vp), C.POINTER(C.c_size_t)]),
        "sptr_unpack_tiles": (C.c_int, [vp, vp, i32, u32, i32, i32, vp, vp]),
        "sptr_intersect": (C.c_int, [vp, fp, u32, up, up, fp, fp]),
        "sptr_occluded": (C.c_int, [vp, fp, u32, bp]),
        "sptr_primary_rays": (C.c_int, [vp, C.POINTER(Camera), i32, i32, u32, fp, up]),
        "sptr_sort_pairs_u64": (C.c_int, [vp, C.POINTER(C.c_uint64), up, u32, C.POINTER(C.c_uint64), up]),
        "sptr_scan_u32": (C.c_int, [vp, up, u32, up]),
        "sptr_eval_math": (C.c_int, [vp, C.c_int, fp, u32, fp]),
        "sptr_host_builtin_scene": (C.c_int, [C.c_char_p, u32, u32, C.POINTER(vp)]),
        "sptr_host_scene_view": (C.c_int, [vp, C.POINTER(Scene)]),
        "sptr_host_scene_free": (None, [vp]),
        "sptr_host_camera_lookat": (C.c_int, [fp, fp, C.c_float, C.c_float, C.POINTER(Camera)]),
        "sptr_host_preset_materials": (C.c_int, [C.c_int, C.POINTER(Material), C.c_int]),
        "sptr_host_default_lights": (C.c_int, [C.POINTER(Light), C.c_int]),
        "sptr_host_equirect_to_faces": (C.c_int, [fp, i32, i32, i32, fp]),
        "sptr_host_pack_tiles": (C.c_int, [bp, i32, i32, i32, i32, up]),
        "sptr_host_unpack_tiles": (C.c_int, [up, i32, u32, i32, i32, bp]),
        "sptr_host_load_hdr": (C.c_int, [C.c_char_p, C.POINTER(fp), C.POINTER(i32), C.POINTER(i32)]),
        "sptr_host_free": (None, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.sptr_abi_version() != SPTR_ABI_VERSION:  # a stale build would misread the structs below
        raise SptrError(f"{LIB_PATH}: ABI {L.sptr_abi_version()}, this binding expects {SPTR_ABI_VERSION} (rebuild)")
    _lib = L
    return L


def _f(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _u(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def _b(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


# --------------------------------------------------------------------------------- host scene layer
@dataclass
class FlatScene:
    """World-space flattened scene in EmbreeBackend::build geomID order (numpy-owned copies)."""
    positions: np.ndarray       # (V,3) float32
    indices: np.ndarray         # (T,3) uint32
    tri_geom_first: np.ndarray  # (G+1,) uint32
    spheres: np.ndarray         # (S,4) float32
    geom_material: np.ndarray   # (G+S,) uint32

    def to_c(self) -> Scene:
        self._keep = [np.ascontiguousarray(self.positions, np.float32), np.ascontiguousarray(self.indices, np.uint32),
                      np.ascontiguousarray(self.tri_geom_first, np.uint32),
                      np.ascontiguousarray(self.spheres, np.float32),
                      np.ascontiguousarray(self.geom_material, np.uint32)]
        p, i, g, s, m = self._keep
        return Scene(_f(p), len(p), _u(i), len(i), _u(g), len(g) - 1, _f(s), len(s), _u(m))


def builtin_scene(name: str, p0: int = 0, p1: int = 0) -> FlatScene:
    """Scenes built by the C++ host layer: default, default_emitter, test_triangle,
    sphere_mesh (p0 stacks, p1 slices), gltf:<path> (p0 = material)."""
    L = lib()
    h = C.c_void_p()
    rc = L.sptr_host_builtin_scene(name.encode(), p0, p1, C.byref(h))
    if rc != 0:
        raise SptrError(f"builtin scene {name!r} failed ({rc})")
    try:
        v = Scene()
        L.sptr_host_scene_view(h, C.byref(v))

        def arr(ptr, n, dt, cols):
            if n == 0:
                return np.zeros((0, cols) if cols > 1 else (0,), dt)
            a = np.ctypeslib.as_array(ptr, shape=(n * cols,)).copy().astype(dt)
            return a.reshape(n, cols) if cols > 1 else a

        return FlatScene(
            positions=arr(v.positions, v.num_verts, np.float32, 3),
            indices=arr(v.indices, v.num_tris, np.uint32, 3),
            tri_geom_first=arr(v.tri_geom_first, v.num_tri_geoms + 1, np.uint32, 1),
            spheres=arr(v.spheres, v.num_spheres, np.float32, 4),
            geom_material=arr(v.geom_material, v.num_tri_geoms + v.num_spheres, np.uint32, 1),
        )
    finally:
        L.sptr_host_scene_free(h)


def camera_lookat(pos=(0.0, 3.0, 8.0), target=(0.0, 1.0, 0.0), fov=60.0, aspect=800 / 600) -> Camera:
    """Camera(pos, target, +Y, fov, aspect) as src/main.cpp:97-103 sets it up."""
    L = lib()
    c = Camera()
    p = np.array(pos, np.float32)
    t = np.array(target, np.float32)
    rc = L.sptr_host_camera_lookat(_f(p), _f(t), C.c_float(fov), C.c_float(aspect), C.byref(c))
    if rc != 0:
        raise SptrError("camera_lookat failed")
    return c


def preset_materials(with_light: bool = False) -> list:
    L = lib()
    arr = (Material * 16)()
    n = L.sptr_host_preset_materials(1 if with_light else 0, arr, 16)
    return [arr[i] for i in range(n)]


def materials_as_array(mats) -> np.ndarray:
    """(n,12) float32: albedo3 metallic roughness emission3 ior type pad pad (oracle layout)."""
    out = np.zeros((len(mats), 12), np.float32)
    for i, m in enumerate(mats):
        out[i, 0:3] = list(m.albedo)
        out[i, 3] = m.metallic
        out[i, 4] = m.roughness
        out[i, 5:8] = list(m.emission)
        out[i, 8] = m.ior
        out[i, 9] = m.type
    return out


def default_lights() -> list:
    L = lib()
    arr = (Light * 8)()
    n = L.sptr_host_default_lights(arr, 8)
    return [arr[i] for i in range(n)]


def lights_as_array(lights) -> np.ndarray:
    out = np.zeros((len(lights), 8), np.float32)
    for i, l in enumerate(lights):
        out[i, 0] = l.type
        out[i, 1:4] = list(l.v)
        out[i, 4:7] = list(l.color)
        out[i, 7] = l.intensity
    return out


def equirect_to_faces(rgb: np.ndarray, size: int = 512) -> np.ndarray:
    L = lib()
    rgb = np.ascontiguousarray(rgb, np.float32)
    h, w = rgb.shape[:2]
    faces = np.zeros((6, size, size, 3), np.float32)
    if L.sptr_host_equirect_to_faces(_f(rgb), w, h, size, _f(faces)) != 0:
        raise SptrError("equirect_to_faces failed")
    return faces


def tiles_per_rank(width: int, height: int, shard_count: int) -> int:
    ntiles = ((width + 31) // 32) * ((height + 31) // 32)
    return (ntiles + shard_count - 1) // shard_count


def pack_tiles(rgb: np.ndarray, shard_count: int, shard_rank: int) -> np.ndarray:
    """Host twin of the device tile packing: this shard's pixels as RGBA8 words, tile-packed and
    padded to tiles_per_rank tiles (the send buffer of the gather to rank 0)."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w = rgb.shape[:2]
    out = np.zeros(tiles_per_rank(w, h, shard_count) * 1024, np.uint32)
    if lib().sptr_host_pack_tiles(_b(rgb), w, h, shard_count, shard_rank, _u(out)) != 0:
        raise SptrError("pack_tiles failed")
    return out


def unpack_tiles(gathered: np.ndarray, shard_count: int, width: int, height: int) -> np.ndarray:
    g = np.ascontiguousarray(gathered, np.uint32)
    out = np.zeros((height, width, 3), np.uint8)
    if lib().sptr_host_unpack_tiles(_u(g), shard_count, tiles_per_rank(width, height, shard_count), width, height,
                                    _b(out)) != 0:
        raise SptrError("unpack_tiles failed")
    return out


def load_hdr(path: str) -> np.ndarray:
    L = lib()
    p = C.POINTER(C.c_float)()
    w, h = C.c_int32(), C.c_int32()
    if L.sptr_host_load_hdr(path.encode(), C.byref(p), C.byref(w), C.byref(h)) != 0:
        raise SptrError(f"cannot read {path}")
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        L.sptr_host_free(p)


# --------------------------------------------------------------------------------- device renderer
class Renderer:
    """One sptr context (one GPU).  Raises SptrError on any failure; never falls back to the CPU."""

    def __init__(self, device: int = 0):
        L = lib()
        self._L = L
        h = C.c_void_p()
        rc = L.sptr_create(device, C.byref(h))
        if rc != 0:
            raise SptrError(f"sptr_create(device={device}) failed ({rc}); a HIP GPU is required")
        self._h = h
        self.width = self.height = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.sptr_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self._L.sptr_last_error(self._h)
            raise SptrError(f"{what}: rc={rc}: {msg.decode() if msg else ''}")

    def upload_scene(self, s: FlatScene):
        cs = s.to_c()
        self._check(self._L.sptr_upload_scene(self._h, C.byref(cs)), "upload_scene")

    def scene_info(self) -> dict:
        n, nn, dep = C.c_uint32(), C.c_uint32(), C.c_uint32()
        ms = C.c_double()
        self._check(self._L.sptr_scene_info(self._h, C.byref(n), C.byref(nn), C.byref(dep), C.byref(ms)), "info")
        return {"prims": n.value, "nodes": nn.value, "depth": dep.value, "build_ms": ms.value}

    def scene_layout(self) -> dict:
        lay = SceneLayout()
        self._check(self._L.sptr_scene_layout_info(self._h, C.byref(lay)), "scene_layout")
        return lay.as_dict()

    def set_materials(self, mats):
        arr = (Material * len(mats))(*mats)
        self._check(self._L.sptr_set_materials(self._h, arr, len(mats)), "set_materials")

    def set_lights(self, lights):
        arr = (Light * max(1, len(lights)))(*lights)
        self._check(self._L.sptr_set_lights(self._h, arr, len(lights)), "set_lights")

    def set_environment(self, faces: np.ndarray | None = None, intensity: float = 0.8, max_clamp: float = 5.0):
        e = Environment()
        if faces is not None:
            self._env_keep = np.ascontiguousarray(faces, np.float32)
            e.faces = _f(self._env_keep)
            e.size = self._env_keep.shape[1]
        e.intensity = intensity
        e.max_clamp = max_clamp
        self._check(self._L.sptr_set_environment(self._h, C.byref(e)), "set_environment")

    def set_wave_paths(self, n: int):
        self._check(self._L.sptr_set_wave_paths(self._h, n), "set_wave_paths")

    def graph_info(self) -> dict:
        """sptr_graph_info: the held launch graph (valid, nodes, edges, longest-path depth)."""
        v = [C.c_uint32() for _ in range(5)] + [C.c_int32()]
        self._check(self._L.sptr_graph_info(self._h, *[C.byref(x) for x in v]), "graph_info")
        d = dict(zip(("valid", "nodes", "edges", "depth", "captures", "capture_status"), (int(x.value) for x in v)))
        d["capture_error"] = self._L.sptr_capture_error(self._h).decode()
        return d

    def overlap_probe(self) -> dict:
        """sptr_overlap_probe: ms of two 200-us spins serial, and beside each side stream."""
        ms = (C.c_double * 3)()
        self._check(self._L.sptr_overlap_probe(self._h, ms), "overlap_probe")
        return {"serial_ms": round(ms[0], 4), "side_ms": round(ms[1], 4), "sky_side_ms": round(ms[2], 4),
                "side_has_own_queue": bool(ms[1] < 0.75 * ms[0]), "sky_side_has_own_queue": bool(ms[2] < 0.75 * ms[0])}

    def set_launch_mode(self, mode: int):
        """0: replay captured launch graphs for large repeated call shapes that fork nothing (default);
        1: direct launches; 2: direct launches, all on the render stream (no overlap); 3: launch graphs
        for every repeated shape."""
        self._check(self._L.sptr_set_launch_mode(self._h, mode), "set_launch_mode")

    def set_pixel_lanes(self, lanes: int):
        """0: automatic (two lanes for large calls on LDS-staged scenes); 1: one launch chain; 2: the
        shard's even and odd tiles as two concurrent launch chains (include/sptr_hip.h)."""
        self._check(self._L.sptr_set_pixel_lanes(self._h, lanes), "set_pixel_lanes")

    def pixel_lanes_info(self) -> dict:
        """{"requested": 0/1/2, "active": whether the current accumulation runs in two lanes}."""
        r, a = C.c_uint32(), C.c_uint32()
        self._check(self._L.sptr_pixel_lanes_info(self._h, C.byref(r), C.byref(a)), "pixel_lanes_info")
        return {"requested": r.value, "active": bool(a.value)}

    def set_tail_depth(self, n: int):
        self._check(self._L.sptr_set_tail_depth(self._h, n), "set_tail_depth")

    def set_leaf_size(self, n: int):
        self._check(self._L.sptr_set_leaf_size(self._h, n), "set_leaf_size")

    def set_split_refs(self, max_pieces: int):
        """sptr_set_split_refs: most references per split triangle (0 = default 1: none); next upload."""
        self._check(self._L.sptr_set_split_refs(self._h, max_pieces), "set_split_refs")

    def set_stragglers(self, lanes: int):
        """sptr_set_stragglers: hand a drained wave's rays off once at most `lanes` lanes still trace
        (0 = off, default 12); HBM-resident scenes only."""
        self._check(self._L.sptr_set_stragglers(self._h, lanes), "set_stragglers")

    def set_bvh_width(self, n: int):
        self._check(self._L.sptr_set_bvh_width(self._h, n), "set_bvh_width")

    def set_debug_mode(self, m: int):
        self._check(self._L.sptr_set_debug_mode(self._h, m), "set_debug_mode")

    def render(self, cam: Camera, width: int, height: int, spp: int = 1, frame_begin: int = 1,
               max_depth: int = 6, shard_rank: int = 0, shard_count: int = 1, flags: int = 0,
               stream: int | None = None, integrator: int = SPTR_INTEGRATOR_WAVEFRONT,
               samples_per_frame: int = 0) -> Stats:
        """spp = progressive frames; integrator / samples_per_frame as in include/sptr_hip.h."""
        f = Frame(width, height, cam, frame_begin, spp, max_depth, shard_rank, shard_count, flags, integrator,
                  samples_per_frame)
        st = Stats()
        self._check(self._L.sptr_render(self._h, C.byref(f), C.c_void_p(stream) if stream else None, C.byref(st)),
                    "render")
        self.width, self.height = width, height
        return st

    def collect_stats(self) -> Stats:
        """Wait for the SPTR_FRAME_ASYNC renders and return their summed stats."""
        st = Stats()
        self._check(self._L.sptr_collect_stats(self._h, C.byref(st)), "collect_stats")
        return st

    def read_rgb8(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 3), np.uint8)
        self._check(self._L.sptr_read_rgb8(self._h, _b(out)), "read_rgb8")
        return out

    def read_rgb8_lagged(self, out: np.ndarray) -> bool:
        """After an asynchronous render: out <- the image of the previous such call (True), or False
        (out untouched) when there is none of this size yet.  out stays page-locked while in use."""
        assert out.dtype == np.uint8 and out.flags.c_contiguous and out.size == self.width * self.height * 3
        got = C.c_uint32()
        self._check(self._L.sptr_read_rgb8_lagged(self._h, _b(out), C.byref(got)), "read_rgb8_lagged")
        return bool(got.value)

    def read_accum(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 3), np.float32)
        self._check(self._L.sptr_read_accum(self._h, _f(out)), "read_accum")
        return out

    def tiles_device(self) -> tuple[int, int]:
        p = C.c_void_p()
        n = C.c_size_t()
        self._check(self._L.sptr_tiles_device(self._h, C.byref(p), C.byref(n)), "tiles_device")
        return p.value, n.value

    def unpack_tiles(self, gathered_ptr: int, shard_count: int, tiles_per_rank: int, width: int, height: int,
                     out_ptr: int, stream: int | None = None):
        self._check(self._L.sptr_unpack_tiles(self._h, C.c_void_p(gathered_ptr), shard_count, tiles_per_rank, width,
                                              height, C.c_void_p(out_ptr),
                                              C.c_void_p(stream) if stream else None), "unpack_tiles")

    def intersect(self, rays: np.ndarray):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        n = len(rays)
        geom = np.zeros(n, np.uint32)
        prim = np.zeros(n, np.uint32)
        t = np.zeros(n, np.float32)
        ng = np.zeros((n, 3), np.float32)
        self._check(self._L.sptr_intersect(self._h, _f(rays), n, _u(geom), _u(prim), _f(t), _f(ng)), "intersect")
        return geom, prim, t, ng

    def occluded(self, rays: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        out = np.zeros(len(rays), np.uint8)
        self._check(self._L.sptr_occluded(self._h, _f(rays), len(rays), _b(out)), "occluded")
        return out

    def primary_rays(self, cam: Camera, width: int, height: int, acc: int):
        dirs = np.zeros((height, width, 3), np.float32)
        rng = np.zeros((height, width), np.uint32)
        self._check(self._L.sptr_primary_rays(self._h, C.byref(cam), width, height, acc, _f(dirs), _u(rng)),
                    "primary_rays")
        return dirs, rng

    def sort_pairs_u64(self, keys: np.ndarray, vals: np.ndarray):
        """The LBVH build's stable device radix sort (kernels_sort.hip): (keys, vals) sorted by key."""
        k = np.ascontiguousarray(keys, np.uint64)
        v = np.ascontiguousarray(vals, np.uint32)
        assert k.shape == v.shape and k.ndim == 1
        ko, vo = np.empty_like(k), np.empty_like(v)
        u64p = C.POINTER(C.c_uint64)
        self._check(self._L.sptr_sort_pairs_u64(self._h, k.ctypes.data_as(u64p), _u(v), len(k),
                                                ko.ctypes.data_as(u64p), _u(vo)), "sort_pairs_u64")
        return ko, vo

    def cosine_sincos_table(self) -> np.ndarray:
        """(sin, cos) of the cosine sample's phi for every r1 = k / 2^24, as the device computes them:
        (2^24, 2) float32 (sptr_eval_math, fn 0)."""
        out = np.empty((1 << 24, 2), np.float32)
        self._check(self._L.sptr_eval_math(self._h, 0, None, 0, _f(out)), "eval_math")
        return out

    def gamma_pow(self, x: np.ndarray) -> np.ndarray:
        """powf(x, 1/2.2) as the device's resolve computes it (sptr_eval_math, fn 1)."""
        a = np.ascontiguousarray(x, np.float32).ravel()
        out = np.empty_like(a)
        self._check(self._L.sptr_eval_math(self._h, 1, _f(a), len(a), _f(out)), "eval_math")
        return out.reshape(np.shape(x))

    def scan_u32(self, counts: np.ndarray) -> np.ndarray:
        """The LBVH build's device exclusive prefix sum of u32 counts (mod 2^32)."""
        a = np.ascontiguousarray(counts, np.uint32)
        out = np.empty_like(a)
        self._check(self._L.sptr_scan_u32(self._h, _u(a), len(a), _u(out)), "scan_u32")
        return out


def setup_default(r: Renderer, scene: str = "default", p0: int = 0, p1: int = 0, env_faces=None) -> FlatScene:
    """Upload a builtin scene with the reference's default state (presets, one sun, sky)."""
    s = builtin_scene(scene, p0, p1)
    r.upload_scene(s)
    r.set_materials(preset_materials(with_light=(scene == "default_emitter")))
    r.set_lights(default_lights())
    r.set_environment(env_faces)
    return s
