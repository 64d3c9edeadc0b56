"""oracle.py — ctypes binding of the CPU ORACLE (oracle/libpm_oracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker; never by the product path.
PARITY UNPINNED against reference outputs (see pm_oracle.h). Struct layouts
mirror include/pm.h (duplicated here so the oracle stays independent of the
product library).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpm_oracle.so")


class Float3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Int3(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("z", C.c_int32)]


class Material(C.Structure):
    _fields_ = [("albedo", Float3), ("diffuse", C.c_float), ("specular", C.c_float),
                ("transmission", C.c_float), ("refraction_idx", C.c_float)]


class Mesh(C.Structure):
    _fields_ = [("vertices", C.POINTER(Float3)), ("num_vertices", C.c_int32),
                ("indices", C.POINTER(Int3)), ("num_triangles", C.c_int32), ("material", Material)]


class Light(C.Structure):
    _fields_ = [("source_type", C.c_int32), ("pos", Float3), ("power", C.c_double), ("rgb", Float3),
                ("normal", Float3), ("side_length", C.c_double), ("num_photons", C.c_int32)]


class Camera(C.Structure):
    _fields_ = [("pos", Float3), ("dir_00", Float3), ("dir_du", Float3), ("dir_dv", Float3)]


class ViewerParams(C.Structure):
    _fields_ = [("look_from", Float3), ("look_at", Float3), ("look_up", Float3), ("fovy", C.c_float),
                ("width", C.c_int32), ("height", C.c_int32)]


class TraceParams(C.Structure):
    _fields_ = [("casted_photons", C.c_int64), ("max_depth", C.c_int32), ("caustics_mode", C.c_int32),
                ("shard_rank", C.c_int32), ("shard_count", C.c_int32)]


class RenderParams(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("samples_per_pixel", C.c_int32),
                ("max_depth", C.c_int32), ("camera", Camera), ("sky_colour", Float3),
                ("tile_rank", C.c_int32), ("tile_count", C.c_int32), ("caustic_k", C.c_int32)]


class RenderStats(C.Structure):
    _fields_ = [("pixels", C.c_int64), ("path_vertices", C.c_int64), ("caustic_queries", C.c_int64),
                ("global_queries", C.c_int64), ("rays", C.c_int64)]


_P = C.c_void_p


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"oracle not built: make -C {_HERE}")
    lib = C.CDLL(LIB_PATH)
    sig = {
        "orc_lcg_init": (C.c_uint32, [C.c_uint32, C.c_uint32]),
        "orc_lcg_next": (C.c_float, [C.POINTER(C.c_uint32)]),
        "orc_acosf": (C.c_float, [C.c_float]),
        "orc_sinf": (C.c_float, [C.c_float]),
        "orc_cosf": (C.c_float, [C.c_float]),
        "orc_random_point_in_unit_sphere": (None, [C.POINTER(C.c_uint32), C.POINTER(C.c_float)]),
        "orc_quantize6": (None, [_P, _P, C.c_int64]),
        "orc_viewer_matrix": (None, [C.POINTER(ViewerParams), C.POINTER(C.c_float)]),
        "orc_photon_view": (C.c_int, [_P, _P, C.c_int64, C.POINTER(ViewerParams), _P]),
        "orc_emit_photon": (None, [C.POINTER(Light), C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
        "orc_refract": (None, [C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_float, C.POINTER(C.c_float)]),
        "orc_scene_create": (C.c_int, [C.POINTER(Mesh), C.c_int32, C.c_int32, C.POINTER(_P)]),
        "orc_scene_destroy": (None, [_P]),
        "orc_scene_num_triangles": (C.c_int64, [_P]),
        "orc_intersect": (C.c_int, [_P, _P, C.c_int64, _P]),
        "orc_occluded": (C.c_int, [_P, _P, C.c_int64, _P]),
        "orc_photons_per_light": (C.c_int, [C.POINTER(Light), C.c_int32, C.c_int64, C.POINTER(C.c_int64)]),
        "orc_trace_photons": (C.c_int, [_P, C.POINTER(Light), C.c_int32, C.POINTER(TraceParams), C.c_int32, _P,
                                        C.c_int64, C.POINTER(C.c_int64)]),
        "orc_trace_photon_range": (C.c_int, [_P, C.POINTER(Light), C.c_int32, C.POINTER(TraceParams), C.c_int64,
                                             C.c_int64, C.c_int32, _P, C.c_int64, C.POINTER(C.c_int64)]),
        "orc_map_create": (C.c_int, [_P, C.c_int64, C.c_float, _P, C.c_int64, C.c_float, C.POINTER(_P)]),
        "orc_map_set_spec": (C.c_int, [_P, C.c_int32, C.c_int32]),
        "orc_map_destroy": (None, [_P]),
        "orc_set_build_threads": (None, [C.c_int32]),
        "orc_kd_left_balanced": (C.c_int, [_P, C.c_int64, C.c_int64, C.c_int32, _P]),
        "orc_left_size": (C.c_int64, [C.c_int64]),
        "orc_knn": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_float, C.c_int32, _P, _P, _P]),
        "orc_gather": (C.c_int, [_P, _P, _P, C.c_int64, C.c_int32, _P]),
        "orc_gather_k": (C.c_int, [_P, _P, _P, C.c_int64, C.c_int32, C.c_int32, _P]),
        "orc_camera_setup": (C.c_int, [Float3, Float3, Float3, C.c_float, C.c_int32, C.c_int32,
                                       C.POINTER(Camera)]),
        "orc_render": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(Light), C.c_int32, _P, _P, C.c_int32,
                                 C.c_int32, C.c_int32, _P, _P, C.POINTER(RenderStats)]),
    }
    for n, (r, a) in sig.items():
        f = getattr(lib, n)
        f.restype = r
        f.argtypes = a
    return lib


lib = _load()


def _chk(st, what):
    if st != 0:
        raise RuntimeError(f"oracle {what} failed with status {st}")


def _f3(v):
    return Float3(float(v[0]), float(v[1]), float(v[2]))


def lights_array(lights):
    arr = (Light * max(1, len(lights)))()
    for i, l in enumerate(lights):
        arr[i].pos = _f3(l["pos"])
        arr[i].rgb = _f3(l["rgb"])
        arr[i].power = float(l["power"])
        if "side" in l:   # SQUARE_LIGHT
            arr[i].source_type = 1
            arr[i].normal = _f3(l["normal"])
            arr[i].side_length = float(l["side"])
    return arr


def _mesh_array(meshes):
    arr = (Mesh * max(1, len(meshes)))()
    keep = []
    for i, m in enumerate(meshes):
        v = np.ascontiguousarray(m.vertices, np.float32)
        ix = np.ascontiguousarray(m.indices, np.int32)
        keep += [v, ix]
        arr[i].vertices = v.ctypes.data_as(C.POINTER(Float3))
        arr[i].num_vertices = len(v)
        arr[i].indices = ix.ctypes.data_as(C.POINTER(Int3))
        arr[i].num_triangles = len(ix)
        mt = np.asarray(m.material, np.float32)
        arr[i].material = Material(Float3(*map(float, mt[:3])), *map(float, mt[3:7]))
    return arr, keep


class Scene:
    def __init__(self, meshes, use_bvh=True):
        arr, keep = _mesh_array(meshes)
        h = _P()
        _chk(lib.orc_scene_create(arr, len(meshes), int(use_bvh), C.byref(h)), "scene_create")
        self.h = h

    def intersect(self, rays: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays, np.float32)
        hits = np.zeros((len(rays), 4), np.int32)
        _chk(lib.orc_intersect(self.h, rays.ctypes.data, len(rays), hits.ctypes.data), "intersect")
        return hits

    def occluded(self, rays: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays, np.float32)
        occ = np.zeros((len(rays),), np.int32)
        _chk(lib.orc_occluded(self.h, rays.ctypes.data, len(rays), occ.ctypes.data), "occluded")
        return occ

    def __del__(self):
        if getattr(self, "h", None):
            lib.orc_scene_destroy(self.h)
            self.h = None


def emit_photon(light: dict, pid: int):
    """(origin, direction) of photon `pid` of one light (RNG seeded (pid, 0))."""
    arr = lights_array([light])
    o, d = (C.c_float * 3)(), (C.c_float * 3)()
    lib.orc_emit_photon(arr, pid, o, d)
    return np.array(o[:], np.float32), np.array(d[:], np.float32)


def photons_per_light(lights, casted):
    out = (C.c_int64 * max(1, len(lights)))()
    _chk(lib.orc_photons_per_light(lights_array(lights), len(lights), int(casted), out), "photons_per_light")
    return [out[i] for i in range(len(lights))]


def trace(scene: Scene, lights, casted, max_depth, caustics, shard_rank=0, shard_count=1, nthreads=8,
          g_range=None) -> np.ndarray:
    p = TraceParams(int(casted), int(max_depth), int(bool(caustics)), int(shard_rank), int(shard_count))
    la = lights_array(lights)
    cnt = C.c_int64()
    # first pass with zero capacity to learn the count
    if g_range is None:
        st = lib.orc_trace_photons(scene.h, la, len(lights), C.byref(p), nthreads, None, 0, C.byref(cnt))
    else:
        st = lib.orc_trace_photon_range(scene.h, la, len(lights), C.byref(p), g_range[0], g_range[1], nthreads,
                                        None, 0, C.byref(cnt))
    if st not in (0, 6):
        _chk(st, "trace")
    out = np.zeros((max(1, cnt.value), 10), np.float32)
    if g_range is None:
        st = lib.orc_trace_photons(scene.h, la, len(lights), C.byref(p), nthreads, out.ctypes.data, len(out),
                                   C.byref(cnt))
    else:
        st = lib.orc_trace_photon_range(scene.h, la, len(lights), C.byref(p), g_range[0], g_range[1], nthreads,
                                        out.ctypes.data, len(out), C.byref(cnt))
    _chk(st, "trace")
    return out[: cnt.value]


class PhotonMap:
    def __init__(self, a: np.ndarray, pa: float, b: np.ndarray = None, pb: float = 0.0, nthreads: int = 1):
        a = np.ascontiguousarray(a if a is not None else np.zeros((0, 10), np.float32), np.float32)
        b = np.ascontiguousarray(b if b is not None else np.zeros((0, 10), np.float32), np.float32)
        self._keep = (a, b)
        h = _P()
        lib.orc_set_build_threads(int(nthreads))
        _chk(lib.orc_map_create(a.ctypes.data if len(a) else None, len(a), float(pa),
                                b.ctypes.data if len(b) else None, len(b), float(pb), C.byref(h)), "map_create")
        self.h = h
        self.n = len(a) + len(b)

    # alternative specifications of the gather (orc_map_set_spec; a measured
    # bound on the unpinned choices, not the parity spec): HEAP is required
    SPEC_DOMAIN_DIM, SPEC_HEAP, SPEC_FMA = 1, 2, 4

    def set_spec(self, flags: int, nthreads: int = 8):
        """Later gathers / renders through this map follow specification
        `flags` (0: production, sorted (d^2, original index) lists)."""
        _chk(lib.orc_map_set_spec(self.h, int(flags), int(nthreads)), "map_set_spec")

    def knn(self, q: np.ndarray, k=50, radius=100.0, nthreads=8):
        q = np.ascontiguousarray(q, np.float32)
        ids = np.zeros((len(q), k), np.int32)
        d2 = np.zeros((len(q), k), np.float32)
        md = np.zeros((len(q),), np.float32)
        _chk(lib.orc_knn(self.h, q.ctypes.data, len(q), k, float(radius), nthreads, ids.ctypes.data,
                         d2.ctypes.data, md.ctypes.data), "knn")
        return ids, d2, md

    def gather(self, pts: np.ndarray, brdf: np.ndarray, nthreads=8, k=50):
        pts = np.ascontiguousarray(pts, np.float32)
        brdf = np.ascontiguousarray(brdf, np.float32)
        out = np.zeros((len(pts), 3), np.float32)
        _chk(lib.orc_gather_k(self.h, pts.ctypes.data, brdf.ctypes.data, len(pts), int(k), nthreads,
                              out.ctypes.data), "gather")
        return out

    def __del__(self):
        if getattr(self, "h", None):
            lib.orc_map_destroy(self.h)
            self.h = None


def kd_left_balanced(pos: np.ndarray, nthreads: int = 8) -> np.ndarray:
    """cukd::buildTree's left-balanced layout (ray-tracer/src/hostCode.cu:94-95):
    int32 tag per node, original index << 2 | split dimension. `pos` is (n, >=3)
    float32; columns 0..2 are the point."""
    pos = np.ascontiguousarray(pos, np.float32)
    n = len(pos)
    tags = np.zeros((max(1, n),), np.int32)
    stride = pos.shape[1] if pos.ndim == 2 else 3
    _chk(lib.orc_kd_left_balanced(pos.ctypes.data if n else None, stride, n, int(nthreads),
                                  tags.ctypes.data), "kd_left_balanced")
    return tags[:n]


def left_size(s: int) -> int:
    return int(lib.orc_left_size(int(s)))


def camera_setup(look_from, look_at, look_up, fovy, w, h) -> Camera:
    cam = Camera()
    _chk(lib.orc_camera_setup(_f3(look_from), _f3(look_at), _f3(look_up), float(fovy), int(w), int(h),
                              C.byref(cam)), "camera_setup")
    return cam


def render(scene: Scene, camera: Camera, w, h, spp, depth, sky, lights, gmap: PhotonMap, cmap: PhotonMap,
           rows=None, tile_rank=0, tile_count=1, nthreads=8, caustic_k=0):
    p = RenderParams(int(w), int(h), int(spp), int(depth), camera, _f3(sky), int(tile_rank), int(tile_count),
                     int(caustic_k))
    rgba = np.zeros((h, w), np.uint32)
    rgb = np.zeros((h, w, 3), np.float32)
    st = RenderStats()
    lo, hi = (0, 0) if rows is None else rows
    _chk(lib.orc_render(scene.h, C.byref(p), lights_array(lights), len(lights), gmap.h, cmap.h, lo, hi, nthreads,
                        rgba.ctypes.data, rgb.ctypes.data, C.byref(st)), "render")
    return rgba, rgb, st


def viewer_params(look_from, look_at, look_up, fovy, w, h) -> ViewerParams:
    return ViewerParams(_f3(look_from), _f3(look_at), _f3(look_up), float(fovy), int(w), int(h))


def viewer_matrix(params: ViewerParams) -> np.ndarray:
    """glm perspective * lookAt as the oracle builds it, column-major [4][4]."""
    m = (C.c_float * 16)()
    lib.orc_viewer_matrix(C.byref(params), m)
    return np.array(m[:], np.float32).reshape(4, 4)


def view_photons(scene: Scene, photons: np.ndarray, params: ViewerParams) -> np.ndarray:
    ph = np.ascontiguousarray(photons, np.float32)
    rgba = np.zeros((params.height, params.width), np.uint32)
    _chk(lib.orc_photon_view(scene.h, ph.ctypes.data, len(ph), C.byref(params), rgba.ctypes.data), "photon_view")
    return rgba


def quantize6(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    lib.orc_quantize6(x.ctypes.data, out.ctypes.data, x.size)
    return out
