"""pm_amd — Python host mirror of the photon-mapping hot path over libpm_hip.so.

Thin ctypes layer over the C-ABI in include/pm.h. Device buffers are torch
tensors on ``cuda`` (PyTorch is plumbing here: memory, streams and
torch.distributed); every compute call runs the gfx950 HIP kernels of
libpm_hip.so. There is NO CPU fallback: importing works anywhere (so host-side
I/O and symbol checks run on CPU), but compute entry points raise
``PMError(PM_ERR_NO_DEVICE)`` without a GPU, and a missing library raises at
import time.

Function names follow the reference's host code:
  compute_photons_per_watt / run_point_light_ray_gen / run_normal / run_caustics
      <- photon-mapping/src/hostCode.cu:72-138
  write_alive_photons / read_photons_from_file
      <- photon-mapping/src/hostCode.cu:31-49, ray-tracer/src/hostCode.cu:26-52
  load_photons (+ build_tree) <- ray-tracer/src/hostCode.cu:54-99
  setup_camera <- ray-tracer/src/hostCode.cu:100-108
  knn / gather_photons <- ray-tracer/cuda/shading.h:11-18, 93-121
  render (simpleRayGen launch) <- ray-tracer/src/hostCode.cu:231-240
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PM_HIP_LIB", os.path.join(_HERE, "..", "lib", "libpm_hip.so"))

(PM_OK, PM_ERR_INVALID, PM_ERR_HIP, PM_ERR_OOM, PM_ERR_NO_DEVICE, PM_ERR_IO, PM_ERR_CAPACITY, PM_ERR_OVERFLOW,
 PM_ERR_DEVICE) = range(9)
PHASES = {"trace": 0, "compact": 1, "kdbuild": 2, "paths": 3, "gather": 4, "resolve": 5, "bvh": 6,
          "gather_global": 7}


class PMError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {_lib.pm_status_string(status).decode() if _lib else status} (status {status})")


# ----------------------------------------------------------------- structs
class Float3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Int3(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("z", C.c_int32)]


class Material(C.Structure):  # common/src/mesh.h:6-12
    _fields_ = [("albedo", Float3), ("diffuse", C.c_float), ("specular", C.c_float),
                ("transmission", C.c_float), ("refraction_idx", C.c_float)]


class Mesh(C.Structure):  # common/src/mesh.h:22-27
    _fields_ = [("vertices", C.POINTER(Float3)), ("num_vertices", C.c_int32),
                ("indices", C.POINTER(Int3)), ("num_triangles", C.c_int32), ("material", Material)]


class Light(C.Structure):  # common/src/world.h:16-27
    _fields_ = [("source_type", C.c_int32), ("pos", Float3), ("power", C.c_double), ("rgb", Float3),
                ("normal", Float3), ("side_length", C.c_double), ("num_photons", C.c_int32)]


class Photon(C.Structure):  # photon-mapping/include/photon.h:5-11
    _fields_ = [("pos", Float3), ("dir", Float3), ("power", C.c_int32), ("color", Float3)]


class KdPhoton(C.Structure):  # ray-tracer/include/photon.h:11-21
    _fields_ = [("pos", Float3), ("dir", Float3), ("color", Float3), ("power", C.c_float),
                ("quantized_normal", C.c_uint8 * 3), ("split_dim", C.c_uint8)]


class Box(C.Structure):
    _fields_ = [("lower", Float3), ("upper", Float3)]


class Camera(C.Structure):  # common/src/camera.h:5-10
    _fields_ = [("pos", Float3), ("dir_00", Float3), ("dir_du", Float3), ("dir_dv", Float3)]


class Ray(C.Structure):
    _fields_ = [("origin", Float3), ("tmin", C.c_float), ("direction", Float3), ("tmax", C.c_float)]


class Hit(C.Structure):
    _fields_ = [("t", C.c_float), ("mesh", C.c_int32), ("prim", C.c_int32), ("tri", C.c_int32)]


class SceneStats(C.Structure):
    _fields_ = [("num_triangles", C.c_int64), ("num_nodes", C.c_int64), ("num_meshes", C.c_int32),
                ("max_depth", C.c_int32), ("bounds", Box)]


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


class ViewerParams(C.Structure):  # pm_viewer_params (photon-viewer camera + fb_size)
    _fields_ = [("look_from", Float3), ("look_at", Float3), ("look_up", Float3), ("fovy", C.c_float),
                ("width", C.c_int32), ("height", C.c_int32)]


class Config(C.Structure):
    _fields_ = [("look_from", Float3), ("look_at", Float3), ("look_up", Float3), ("fovy", C.c_float),
                ("photons_file", C.c_char * 512), ("caustics_photons_file", C.c_char * 512),
                ("model_path", C.c_char * 512), ("sky_colour", Float3), ("output_filename", C.c_char * 512),
                ("fb_width", C.c_int32), ("fb_height", C.c_int32), ("samples_per_pixel", C.c_int32),
                ("depth", C.c_int32), ("viewer_output_filename", C.c_char * 512),
                ("viewer_caustics_output_filename", C.c_char * 512), ("viewer_fb_width", C.c_int32),
                ("viewer_fb_height", C.c_int32), ("casted_diffuse_photons", C.c_int64),
                ("casted_caustics_photons", C.c_int64), ("max_depth", C.c_int32), ("present_mask", C.c_uint32),
                ("error", C.c_char * 512)]


ROWS_MAX_SEGS = 32   # PM_ROWS_MAX_SEGS


class PhotonRowsStruct(C.Structure):   # pm_photon_rows
    _fields_ = [("d_rows", C.c_void_p), ("row_floats", C.c_int32), ("color_offset", C.c_int32),
                ("nseg", C.c_int32), ("reserved", C.c_int32), ("seg_row0", C.c_int64 * ROWS_MAX_SEGS),
                ("seg_count", C.c_int64 * ROWS_MAX_SEGS)]


assert C.sizeof(Material) == 28 and C.sizeof(Photon) == 40 and C.sizeof(KdPhoton) == 44
assert C.sizeof(PhotonRowsStruct) == 24 + 16 * ROWS_MAX_SEGS
assert C.sizeof(Light) == 64

# ----------------------------------------------------------------- library
_P = C.c_void_p
_SIGNATURES = {
    "pm_abi_version": (C.c_int, []),
    "pm_status_string": (C.c_char_p, [C.c_int]),
    "pm_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
    "pm_last_phase_us": (C.c_int, [C.c_int32, C.POINTER(C.c_double)]),
    "pm_device_alloc": (C.c_int, [C.c_size_t, C.POINTER(_P)]),
    "pm_device_free": (C.c_int, [_P]),
    "pm_copy_to_device": (C.c_int, [_P, _P, C.c_size_t]),
    "pm_copy_to_host": (C.c_int, [_P, _P, C.c_size_t]),
    "pm_device_pool_stats": (C.c_int, [C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "pm_scene_create": (C.c_int, [C.POINTER(Mesh), C.c_int32, C.POINTER(_P)]),
    "pm_scene_stats_get": (C.c_int, [_P, C.POINTER(SceneStats)]),
    "pm_scene_destroy": (C.c_int, [_P]),
    "pm_scene_intersect": (C.c_int, [_P, _P, C.c_int64, _P, _P]),
    "pm_scene_occluded": (C.c_int, [_P, _P, C.c_int64, _P, _P]),
    "pm_photons_per_light": (C.c_int, [C.POINTER(Light), C.c_int32, C.c_int64, C.POINTER(C.c_int64)]),
    "pm_trace_capacity": (C.c_int, [C.POINTER(Light), C.c_int32, C.POINTER(TraceParams), C.POINTER(C.c_int64)]),
    "pm_trace_photons": (C.c_int, [_P, C.POINTER(Light), C.c_int32, C.POINTER(TraceParams), _P, C.c_int64,
                                   C.POINTER(C.c_int64), _P]),
    "pm_trace_photon_sets": (C.c_int, [_P, C.POINTER(Light), C.c_int32, C.POINTER(TraceParams), C.POINTER(_P),
                                       C.POINTER(C.c_int64), C.POINTER(C.c_int64), _P]),
    "pm_kdtree_build": (C.c_int, [_P, C.c_int64, _P, _P]),
    "pm_photon_map_create": (C.c_int, [_P, C.c_int64, C.c_float, _P, C.c_int64, C.c_float, C.POINTER(_P), _P]),
    "pm_photon_map_create_rows": (C.c_int, [_P, C.c_float, _P, C.c_float, C.POINTER(_P), _P]),
    "pm_photon_map_size": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "pm_photon_map_export": (C.c_int, [_P, _P, _P]),
    "pm_photon_map_destroy": (C.c_int, [_P]),
    "pm_kd_shard_plan_create": (C.c_int, [_P, C.c_int64, C.c_float, _P, C.c_int64, C.c_float, C.c_int32,
                                          C.POINTER(_P), _P]),
    "pm_kd_shard_subtrees": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    "pm_kd_shard_build": (C.c_int, [_P, C.c_int32, _P, _P]),
    "pm_photon_map_create_sharded": (C.c_int, [_P, _P, C.POINTER(_P), _P]),
    "pm_kd_shard_plan_create_rows": (C.c_int, [_P, C.c_float, _P, C.c_float, C.c_int32, C.POINTER(_P), _P]),
    "pm_kd_shard_plan_destroy": (C.c_int, [_P]),
    "pm_kd_top_sel_create": (C.c_int, [_P, C.c_int64, C.c_int64, _P, C.c_int64, C.c_int64, C.c_int64, C.c_int32,
                                       C.POINTER(_P), _P]),
    "pm_kd_top_sel_step": (C.c_int, [_P, _P, C.POINTER(C.c_int64), C.POINTER(C.c_int32), _P]),
    "pm_kd_shard_plan_create_from_sel": (C.c_int, [_P, _P, C.c_int64, C.c_float, _P, C.c_int64, C.c_float,
                                                   C.POINTER(_P), _P]),
    "pm_kd_shard_plan_create_from_sel_rows": (C.c_int, [_P, _P, C.c_float, _P, C.c_float, C.POINTER(_P), _P]),
    "pm_kd_top_sel_destroy": (C.c_int, [_P]),
    "pm_knn": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_float, _P, _P, _P, _P]),
    "pm_gather": (C.c_int, [_P, _P, _P, C.c_int64, _P, _P]),
    "pm_gather_k": (C.c_int, [_P, _P, _P, C.c_int64, C.c_int32, _P, _P]),
    "pm_camera_setup": (C.c_int, [Float3, Float3, Float3, C.c_float, C.c_int32, C.c_int32, C.POINTER(Camera)]),
    "pm_render": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(Light), C.c_int32, _P, _P, _P, _P, _P]),
    "pm_render_stats_get": (C.c_int, [C.POINTER(RenderStats)]),
    "pm_render_begin": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(Light), C.c_int32, C.POINTER(_P), _P]),
    "pm_render_finish": (C.c_int, [_P, _P, _P, _P, _P, _P]),
    "pm_render_job_destroy": (C.c_int, [_P]),
    "pm_render_job_queries": (C.c_int, [_P, C.c_int32, _P, _P, C.c_int64, C.POINTER(C.c_int64), _P]),
    "pm_render_gather_caustic": (C.c_int, [_P, _P, _P]),
    "pm_photon_view": (C.c_int, [_P, _P, C.c_int64, C.POINTER(ViewerParams), _P, _P]),
    "pm_config_load": (C.c_int, [C.c_char_p, C.POINTER(Config)]),
    "pm_config_key_name": (C.c_char_p, [C.c_int32]),
    "pm_scene_data_load": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "pm_scene_data_counts": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                       C.POINTER(C.c_int64)]),
    "pm_scene_data_meshes": (C.c_int, [_P, C.POINTER(C.POINTER(Mesh))]),
    "pm_scene_data_lights": (C.c_int, [_P, C.POINTER(C.POINTER(Light))]),
    "pm_scene_data_mesh_name": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_char_p)]),
    "pm_scene_data_free": (C.c_int, [_P]),
    "pm_photons_write_txt": (C.c_int, [C.c_char_p, _P, C.c_int64]),
    "pm_photons_read_txt": (C.c_int, [C.c_char_p, C.POINTER(_P), C.POINTER(C.c_int64)]),
    "pm_write_png_rgba": (C.c_int, [C.c_char_p, _P, C.c_int32, C.c_int32]),
    "pm_photons_quantize": (C.c_int, [_P, C.c_int64, _P]),
    "pm_photons_write_bin": (C.c_int, [C.c_char_p, _P, C.c_int64]),
    "pm_photons_read_bin": (C.c_int, [C.c_char_p, C.POINTER(_P), C.POINTER(C.c_int64)]),
    "pm_free": (None, [_P]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libpm_hip.so not built at {LIB_PATH}: run `make -C photon-mapping_amd` "
                          "(or __graft_entry__.build()); the product has no CPU fallback")
    # libpm_hip.so and torch both need libamdhip64.so.7 (one soname, two builds:
    # /opt/rocm and torch's bundled copy); the first one loaded serves the whole
    # process, and torch only finds the GPU with its own. Load torch first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = _load()
lib = _lib


def exported_symbols() -> List[str]:
    return list(_SIGNATURES)


def _check(st: int, what: str):
    if st != PM_OK:
        raise PMError(st, what)


def device_count() -> int:
    n = C.c_int32(0)
    _lib.pm_device_count(C.byref(n))
    return n.value


def pool_stats(device: int = -1):
    """(live, cached) bytes of the library's caching allocator on `device` (-1: all)."""
    live, cached = C.c_int64(0), C.c_int64(0)
    _check(_lib.pm_device_pool_stats(int(device), C.byref(live), C.byref(cached)), "pm_device_pool_stats")
    return live.value, cached.value


def phase_us(name: str) -> float:
    v = C.c_double(0)
    _check(_lib.pm_last_phase_us(PHASES[name], C.byref(v)), "pm_last_phase_us")
    return v.value


def _ptr(t) -> int:
    if t is None:
        return None
    return t.data_ptr()


def _stream(stream) -> Optional[int]:
    if stream is None:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.current_stream().cuda_stream or None
        return None
    return stream


def _f3(v) -> Float3:
    return Float3(float(v[0]), float(v[1]), float(v[2]))


# ----------------------------------------------------------------- host data
@dataclass
class MeshData:
    vertices: np.ndarray   # (V,3) float32
    indices: np.ndarray    # (T,3) int32
    material: np.ndarray   # (7,) float32: albedo rgb, diffuse, specular, transmission, ior
    name: str = ""


def lights_array(lights: Sequence[dict]) -> C.Array:
    """LightSource (world.h:13-24) array. A dict with "normal" and "side" is a
    SQUARE_LIGHT (this build's emission definition, include/pm.h)."""
    arr = (Light * max(1, len(lights)))()
    for i, l in enumerate(lights):
        square = "side" in l
        arr[i].source_type = 1 if square else 0
        arr[i].pos = _f3(l["pos"])
        arr[i].rgb = _f3(l["rgb"])
        arr[i].power = float(l["power"])
        if square:
            arr[i].normal = _f3(l["normal"])
            arr[i].side_length = float(l["side"])
    return arr


def light_dicts(arr, n: int) -> List[dict]:
    out = []
    for i in range(n):
        d = {"pos": (arr[i].pos.x, arr[i].pos.y, arr[i].pos.z), "rgb": (arr[i].rgb.x, arr[i].rgb.y, arr[i].rgb.z),
             "power": arr[i].power}
        if arr[i].source_type == 1:
            d["normal"] = (arr[i].normal.x, arr[i].normal.y, arr[i].normal.z)
            d["side"] = arr[i].side_length
        out.append(d)
    return out


def load_scene_file(path: str):
    """assets::import_scene (common/src/assetImporter.cxx:16-31): returns (meshes, lights)."""
    h = _P()
    _check(_lib.pm_scene_data_load(path.encode(), C.byref(h)), f"import_scene({path})")
    try:
        nm, nl, nv, nt = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
        _lib.pm_scene_data_counts(h, C.byref(nm), C.byref(nl), C.byref(nv), C.byref(nt))
        mp = C.POINTER(Mesh)()
        lp = C.POINTER(Light)()
        _lib.pm_scene_data_meshes(h, C.byref(mp))
        _lib.pm_scene_data_lights(h, C.byref(lp))
        meshes = []
        for i in range(nm.value):
            m = mp[i]
            v = np.ctypeslib.as_array(C.cast(m.vertices, C.POINTER(C.c_float)), (m.num_vertices * 3,)).reshape(-1, 3).copy() \
                if m.num_vertices else np.zeros((0, 3), np.float32)
            ix = np.ctypeslib.as_array(C.cast(m.indices, C.POINTER(C.c_int32)), (m.num_triangles * 3,)).reshape(-1, 3).copy() \
                if m.num_triangles else np.zeros((0, 3), np.int32)
            mt = m.material
            mat = np.array([mt.albedo.x, mt.albedo.y, mt.albedo.z, mt.diffuse, mt.specular, mt.transmission,
                            mt.refraction_idx], np.float32)
            name = C.c_char_p()
            _lib.pm_scene_data_mesh_name(h, i, C.byref(name))
            meshes.append(MeshData(v, ix, mat, name.value.decode()))
        lights = light_dicts(lp, nl.value)
        return meshes, lights
    finally:
        _lib.pm_scene_data_free(h)


def mesh_array(meshes: Sequence[MeshData]):
    """Build a ctypes pm_mesh array (keeps numpy buffers alive via the returned tuple)."""
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
        arr[i].material = Material(Float3(*map(float, mt[:3])), float(mt[3]), float(mt[4]), float(mt[5]), float(mt[6]))
    return arr, keep


def load_config(path: str) -> Config:
    """parse_config (common/src/configLoader.h:8-19) for an explicit path."""
    c = Config()
    st = _lib.pm_config_load(path.encode(), C.byref(c))
    if st != PM_OK:
        raise PMError(st, f"config {path}: {c.error.decode()}")
    return c


def config_key_present(c: Config, key: str) -> bool:
    i = 0
    while True:
        k = _lib.pm_config_key_name(i)
        if k is None:
            return False
        if k.decode() == key:
            return bool(c.present_mask & (1 << i))
        i += 1


# ----------------------------------------------------------------- device objects
class Scene:
    """Device scene + LBVH (loadGeometry, common/src/world.cpp:3-58)."""

    def __init__(self, meshes: Sequence[MeshData]):
        arr, keep = mesh_array(meshes)
        h = _P()
        _check(_lib.pm_scene_create(arr, len(meshes), C.byref(h)), "pm_scene_create")
        self._h = h
        self.meshes = list(meshes)

    @property
    def handle(self):
        return self._h

    def stats(self) -> SceneStats:
        s = SceneStats()
        _check(_lib.pm_scene_stats_get(self._h, C.byref(s)), "pm_scene_stats_get")
        return s

    def intersect(self, rays, stream=None):
        import torch
        n = rays.shape[0]
        hits = torch.empty((n, 4), dtype=torch.int32, device=rays.device)
        _check(_lib.pm_scene_intersect(self._h, _ptr(rays), n, _ptr(hits), _stream(stream)), "pm_scene_intersect")
        return hits

    def occluded(self, rays, stream=None):
        import torch
        n = rays.shape[0]
        occ = torch.empty((n,), dtype=torch.int32, device=rays.device)
        _check(_lib.pm_scene_occluded(self._h, _ptr(rays), n, _ptr(occ), _stream(stream)), "pm_scene_occluded")
        return occ

    def close(self):
        if getattr(self, "_h", None):
            _lib.pm_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def compute_photons_per_watt(lights: Sequence[dict], casted: int) -> List[int]:
    """computePhotonsPerWatt + initialPhotons per light (hostCode.cu:86, 102-110)."""
    la = lights_array(lights)
    out = (C.c_int64 * max(1, len(lights)))()
    _check(_lib.pm_photons_per_light(la, len(lights), int(casted), out), "pm_photons_per_light")
    return [out[i] for i in range(len(lights))]


def trace_capacity(lights, casted, max_depth, caustics, shard_rank=0, shard_count=1) -> int:
    la = lights_array(lights)
    p = TraceParams(int(casted), int(max_depth), int(bool(caustics)), int(shard_rank), int(shard_count))
    cap = C.c_int64()
    _check(_lib.pm_trace_capacity(la, len(lights), C.byref(p), C.byref(cap)), "pm_trace_capacity")
    return cap.value


def run_point_light_ray_gen(scene: Scene, lights, casted: int, max_depth: int, caustics: bool,
                            shard_rank: int = 0, shard_count: int = 1, out=None, stream=None):
    """Traces every light's photons (one fused launch); returns a cuda float32 tensor
    (n, 10) = pm_photon records (pos, dir, power bits, color) in (g, bounce) order."""
    import torch
    la = lights_array(lights)
    p = TraceParams(int(casted), int(max_depth), int(bool(caustics)), int(shard_rank), int(shard_count))
    cap = C.c_int64()
    _check(_lib.pm_trace_capacity(la, len(lights), C.byref(p), C.byref(cap)), "pm_trace_capacity")
    buf = out if out is not None else torch.empty((max(1, cap.value), 10), dtype=torch.float32, device="cuda")
    cnt = C.c_int64()
    _check(_lib.pm_trace_photons(scene.handle, la, len(lights), C.byref(p), _ptr(buf), buf.shape[0], C.byref(cnt),
                                 _stream(stream)), "pm_trace_photons")
    return buf[: cnt.value]


def run_photon_sets(scene: Scene, lights, casted: int, caustic: int, max_depth: int, shard_rank: int = 0,
                    shard_count: int = 1, out=(None, None), stream=None):
    """runNormal + runCaustics (photon-mapping/src/hostCode.cu:112-138) in ONE
    launch (pm_trace_photon_sets): returns (diffuse, caustic) tensors, each
    exactly run_point_light_ray_gen's output for its set. phase_us("trace") is
    the trace window (launch through the last compaction), "compact" the
    compactions."""
    import torch
    la = lights_array(lights)
    ps = (TraceParams * 2)(TraceParams(int(casted), int(max_depth), 0, int(shard_rank), int(shard_count)),
                           TraceParams(int(caustic), int(max_depth), 1, int(shard_rank), int(shard_count)))
    bufs = []
    for k in range(2):
        cap = C.c_int64()
        _check(_lib.pm_trace_capacity(la, len(lights), C.byref(ps[k]), C.byref(cap)), "pm_trace_capacity")
        bufs.append(out[k] if out[k] is not None else
                    torch.empty((max(1, cap.value), 10), dtype=torch.float32, device="cuda"))
    ptrs = (_P * 2)(_ptr(bufs[0]), _ptr(bufs[1]))
    caps = (C.c_int64 * 2)(bufs[0].shape[0], bufs[1].shape[0])
    cnt = (C.c_int64 * 2)()
    _check(_lib.pm_trace_photon_sets(scene.handle, la, len(lights), ps, ptrs, caps, cnt, _stream(stream)),
           "pm_trace_photon_sets")
    return bufs[0][: cnt[0]], bufs[1][: cnt[1]]


def run_normal(scene, lights, casted, max_depth, **kw):
    """runNormal (photon-mapping/src/hostCode.cu:112-124) without the file write."""
    return run_point_light_ray_gen(scene, lights, casted, max_depth, False, **kw)


def run_caustics(scene, lights, casted, max_depth, **kw):
    """runCaustics (photon-mapping/src/hostCode.cu:126-138) without the file write."""
    return run_point_light_ray_gen(scene, lights, casted, max_depth, True, **kw)


PHOTON_POWER = 1.0                       # ray-tracer/src/hostCode.cu:21
CAUSTICS_PHOTON_POWER = PHOTON_POWER * 0.5   # hostCode.cu:22


class PhotonRows:
    """One photon set as row segments of one device buffer (pm_photon_rows):
    what the N > 1 exchange delivers -- (position, colour) rows padded per rank
    in one all-gather buffer -- handed to the maps without a compaction or a
    re-expansion copy. `buf` is a 2-D float32 cuda tensor (rows of
    buf.shape[1] floats, position at 0..2, colour at color_offset..+2);
    `segments` = [(first row, rows), ...] in map order."""

    def __init__(self, buf, segments, color_offset: int):
        import torch
        # the C side reads d_rows as float32 device rows (pm_photon_rows)
        assert buf.dim() == 2 and buf.dtype == torch.float32 and buf.is_cuda and buf.is_contiguous()
        assert len(segments) <= ROWS_MAX_SEGS and 3 <= color_offset <= buf.shape[1] - 3
        assert all(0 <= r0 and 0 <= c and r0 + c <= buf.shape[0] for r0, c in segments)
        self.buf, self.segments, self.color_offset = buf, [(int(r0), int(c)) for r0, c in segments], int(color_offset)
        self.n = sum(c for _, c in self.segments)

    @classmethod
    def of_photons(cls, t):
        """A pm_photon tensor (n, 10): one segment, colour at float 7."""
        return cls(t, [(0, t.shape[0])], 7)

    @classmethod
    def of_padded(cls, buf, counts, m: int, color_offset: int = 3):
        """The all-gather's padded buffer: rank r's counts[r] rows start at row r * m."""
        return cls(buf, [(r * m, c) for r, c in enumerate(counts)], color_offset)

    def struct(self):
        st = PhotonRowsStruct()
        st.d_rows = self.buf.data_ptr() if self.n else None
        st.row_floats, st.color_offset, st.nseg = self.buf.shape[1], self.color_offset, len(self.segments)
        for k, (r0, c) in enumerate(self.segments):
            st.seg_row0[k], st.seg_count[k] = r0, c
        return st

    def rows(self):
        """(n, 6) position + colour, concatenated (a copy; tests and tools)."""
        import torch
        parts = [self.buf[r0: r0 + c] for r0, c in self.segments]
        cat = torch.cat(parts) if parts else self.buf[:0]
        co = self.color_offset
        return torch.cat([cat[:, 0:3], cat[:, co: co + 3]], dim=1).contiguous()

    def photons(self):
        """pm_photon rows (n, 10), direction and power zero (a copy; tests and tools)."""
        import torch
        r = self.rows()
        t = torch.zeros((r.shape[0], 10), dtype=r.dtype, device=r.device)
        t[:, 0:3], t[:, 7:10] = r[:, 0:3], r[:, 3:6]
        return t


def _rows_arg(x):
    """None / pm_photon tensor / PhotonRows -> (pm_photon_rows struct or None, n)"""
    if x is None:
        return None, 0
    r = x if isinstance(x, PhotonRows) else PhotonRows.of_photons(x)
    return (C.byref(r.struct()) if r.n else None), r.n


class PhotonMap:
    """Photon kd-tree + gather payload (loadPhotons + cukd::buildTree). The sets
    are pm_photon tensors (n, 10) or PhotonRows (pm_photon_map_create_rows)."""

    def __init__(self, a, power_a: float, b=None, power_b: float = 0.0, stream=None):
        h = _P()
        if isinstance(a, PhotonRows) or isinstance(b, PhotonRows):
            ra, na = _rows_arg(a)
            rb, nb = _rows_arg(b)
            _check(_lib.pm_photon_map_create_rows(ra, float(power_a), rb, float(power_b), C.byref(h),
                                                  _stream(stream)), "pm_photon_map_create_rows")
        else:
            na = 0 if a is None else a.shape[0]
            nb = 0 if b is None else b.shape[0]
            _check(_lib.pm_photon_map_create(_ptr(a) if na else None, na, float(power_a), _ptr(b) if nb else None,
                                             nb, float(power_b), C.byref(h), _stream(stream)), "pm_photon_map_create")
        self._h = h
        self.n = na + nb

    @property
    def handle(self):
        return self._h

    def export(self, stream=None):
        import torch
        out = torch.empty((max(1, self.n), 11), dtype=torch.float32, device="cuda")
        _check(_lib.pm_photon_map_export(self._h, _ptr(out), _stream(stream)), "pm_photon_map_export")
        return out[: self.n]

    def close(self):
        if getattr(self, "_h", None):
            _lib.pm_photon_map_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class KdShardPlan:
    """The global map's tree split across `world` ranks (pm_kd_shard_plan_*,
    SURVEY §8e): top levels selected here; the subtrees are dealt to ranks by
    `pm_amd.dist.shard_owners(plan.sizes, world)` (size-balanced, deterministic),
    each rank builds its own (`build`), the caller all-gathers them and
    `map(all_subtrees)` places them (subtree order)."""

    def __init__(self, a, power_a: float, b=None, power_b: float = 0.0, world: int = 1, stream=None,
                 sel: "KdTopSel" = None):
        """sel: a finished KdTopSel (the distributed top selection) instead of
        selecting the top levels here from the gathered photons. The sets are
        pm_photon tensors or PhotonRows (the exchange's buffer as it is)."""
        h = _P()
        if isinstance(a, PhotonRows) or isinstance(b, PhotonRows):
            ra, na = _rows_arg(a)
            rb, nb = _rows_arg(b)
            if sel is None:
                _check(_lib.pm_kd_shard_plan_create_rows(ra, float(power_a), rb, float(power_b), int(world),
                                                         C.byref(h), _stream(stream)), "pm_kd_shard_plan_create_rows")
            else:
                _check(_lib.pm_kd_shard_plan_create_from_sel_rows(sel._h, ra, float(power_a), rb, float(power_b),
                                                                  C.byref(h), _stream(stream)),
                       "pm_kd_shard_plan_create_from_sel_rows")
        else:
            na = 0 if a is None else a.shape[0]
            nb = 0 if b is None else b.shape[0]
            if sel is None:
                _check(_lib.pm_kd_shard_plan_create(_ptr(a) if na else None, na, float(power_a),
                                                    _ptr(b) if nb else None, nb, float(power_b), int(world),
                                                    C.byref(h), _stream(stream)), "pm_kd_shard_plan_create")
            else:
                _check(_lib.pm_kd_shard_plan_create_from_sel(sel._h, _ptr(a) if na else None, na, float(power_a),
                                                             _ptr(b) if nb else None, nb, float(power_b), C.byref(h),
                                                             _stream(stream)), "pm_kd_shard_plan_create_from_sel")
        self._h = h
        self.n = na + nb
        cnt = C.c_int32(0)
        _check(_lib.pm_kd_shard_subtrees(h, C.byref(cnt), None), "pm_kd_shard_subtrees")
        sizes = (C.c_int64 * max(1, cnt.value))()
        _check(_lib.pm_kd_shard_subtrees(h, C.byref(cnt), sizes), "pm_kd_shard_subtrees")
        self.sizes = [int(sizes[j]) for j in range(cnt.value)]   # [] : not split

    def build(self, j: int, out=None, stream=None):
        """Subtree j as (size,) int32 node tags, original index << 2 | split dim
        (its own implicit layout)."""
        import torch
        if out is None:
            out = torch.empty((max(1, self.sizes[j]),), dtype=torch.int32, device="cuda")
        _check(_lib.pm_kd_shard_build(self._h, int(j), _ptr(out), _stream(stream)), "pm_kd_shard_build")
        return out[: self.sizes[j]]

    def map(self, subtrees=None, stream=None) -> "PhotonMap":
        """The photon map from all subtrees' tags concatenated in subtree order (None when not split)."""
        h = _P()
        _check(_lib.pm_photon_map_create_sharded(self._h, _ptr(subtrees) if self.sizes else None, C.byref(h),
                                                 _stream(stream)), "pm_photon_map_create_sharded")
        m = PhotonMap.__new__(PhotonMap)
        m._h = h
        m.n = self.n
        return m

    def close(self):
        if getattr(self, "_h", None):
            _lib.pm_kd_shard_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class KdTopSel:
    """Distributed top selection (pm_kd_top_sel_*): this rank's own photons
    (`a` / `b`, global indices a_first.. / b_first.. in the gathered map of
    n_total photons) select the same top levels as KdShardPlan over the gathered
    map, with `reduce(buf, op)` reducing each pass's small int64 output across
    the ranks in place (op "sum" / "min"). Then KdShardPlan(..., sel=self)."""

    def __init__(self, a, a_first: int, b, b_first: int, n_total: int, world: int, stream=None):
        import torch
        h = _P()
        na = 0 if a is None else a.shape[0]
        nb = 0 if b is None else b.shape[0]
        _check(_lib.pm_kd_top_sel_create(_ptr(a) if na else None, na, int(a_first), _ptr(b) if nb else None, nb,
                                         int(b_first), int(n_total), int(world), C.byref(h), _stream(stream)),
               "pm_kd_top_sel_create")
        self._h = h
        self.buf = torch.empty((4096,), dtype=torch.int64, device="cuda")   # PM_KD_TOP_SEL_BUF
        self.steps = 0

    def step(self, stream=None):
        """Consume the reduced previous pass, issue the next: (count, op) with op
        None when finished, else "sum" / "min" over self.buf[:count]."""
        cnt, op = C.c_int64(0), C.c_int32(0)
        _check(_lib.pm_kd_top_sel_step(self._h, _ptr(self.buf), C.byref(cnt), C.byref(op), _stream(stream)),
               "pm_kd_top_sel_step")
        self.steps += 1
        return cnt.value, {0: None, 1: "sum", 2: "min"}[op.value]

    def run(self, reduce, stream=None):
        """Drive every pass: reduce(view, op) reduces self.buf[:count] across ranks in place."""
        while True:
            cnt, op = self.step(stream)
            if op is None:
                return self
            reduce(self.buf[:cnt], op)

    def close(self):
        if getattr(self, "_h", None):
            _lib.pm_kd_top_sel_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_photons(diffuse, caustic, stream=None):
    """loadPhotons (ray-tracer/src/hostCode.cu:54-99): global = diffuse(1.0) ++ caustic(0.5),
    caustic = caustic(0.5); both kd-trees built on the GPU."""
    g = PhotonMap(diffuse, PHOTON_POWER, caustic, CAUSTICS_PHOTON_POWER, stream=stream)
    c = PhotonMap(caustic, CAUSTICS_PHOTON_POWER, stream=stream)
    return g, c


def build_tree(kd_photons, bounds: bool = True, stream=None):
    """cukd::buildTree<Photon, Photon_traits> in place on a (n, 11) float32 cuda tensor of
    pm_kd_photon records; returns the bounds tensor (2,3) if requested."""
    import torch
    b = torch.empty((2, 3), dtype=torch.float32, device="cuda") if bounds else None
    _check(_lib.pm_kdtree_build(_ptr(kd_photons), kd_photons.shape[0], _ptr(b), _stream(stream)), "pm_kdtree_build")
    return b


def knn(pmap: PhotonMap, queries, k: int = 50, max_radius: float = 100.0, stream=None):
    """KNearestPhotons (shading.h:11-18): (ids[nq,k] original indices / -1, d2[nq,k], maxd2[nq])."""
    import torch
    nq = queries.shape[0]
    ids = torch.empty((nq, k), dtype=torch.int32, device="cuda")
    d2 = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    md = torch.empty((nq,), dtype=torch.float32, device="cuda")
    _check(_lib.pm_knn(pmap.handle, _ptr(queries), nq, k, float(max_radius), _ptr(ids), _ptr(d2), _ptr(md),
                       _stream(stream)), "pm_knn")
    return ids, d2, md


def gather_photons(pmap: PhotonMap, points, brdf, stream=None, k: int = 50):
    """gatherPhotons (shading.h:93-121) for a batch of hit points; k != 50
    (up to 256) is pm_gather_k (config 5's k = 200 caustic gather)."""
    import torch
    nq = points.shape[0]
    out = torch.empty((nq, 3), dtype=torch.float32, device="cuda")
    if k == 50:
        _check(_lib.pm_gather(pmap.handle, _ptr(points), _ptr(brdf), nq, _ptr(out), _stream(stream)), "pm_gather")
    else:
        _check(_lib.pm_gather_k(pmap.handle, _ptr(points), _ptr(brdf), nq, int(k), _ptr(out), _stream(stream)),
               "pm_gather_k")
    return out


def setup_camera(look_from, look_at, look_up, fovy, width, height) -> Camera:
    """setupCamera (ray-tracer/src/hostCode.cu:100-108)."""
    cam = Camera()
    _check(_lib.pm_camera_setup(_f3(look_from), _f3(look_at), _f3(look_up), float(fovy), int(width), int(height),
                                C.byref(cam)), "pm_camera_setup")
    return cam


def render(scene: Scene, camera: Camera, width: int, height: int, spp: int, depth: int, sky, lights,
           global_map: PhotonMap, caustic_map: PhotonMap, tile_rank: int = 0, tile_count: int = 1,
           want_rgb: bool = True, rgba=None, stream=None, caustic_k: int = 0):
    """owlRayGenLaunch2D(simpleRayGen, W, H) (ray-tracer/src/hostCode.cu:231-237).
    caustic_k: neighbours of the caustic gather (0 = the reference's 50; config 5: 200).
    Returns (rgba int32 [H,W], rgb float32 [H,W,3] or None)."""
    import torch
    p = RenderParams(int(width), int(height), int(spp), int(depth), camera, _f3(sky), int(tile_rank),
                     int(tile_count), int(caustic_k))
    la = lights_array(lights)
    if rgba is None:
        rgba = torch.zeros((height, width), dtype=torch.int32, device="cuda")
    rgb = torch.zeros((height, width, 3), dtype=torch.float32, device="cuda") if want_rgb else None
    _check(_lib.pm_render(scene.handle, C.byref(p), la, len(lights), global_map.handle, caustic_map.handle,
                          _ptr(rgba), _ptr(rgb), _stream(stream)), "pm_render")
    return rgba, rgb


class RenderJob:
    """pm_render_begin's map-independent half of a render (camera paths, shadow
    and final-gather rays, direct light, sorted gather queries). It reads only
    the scene, so it may run on another stream and host thread (ctypes releases
    the GIL) while the photons are traced and the kd-trees built; finish() runs
    the gathers and resolve. begin + finish == render()."""

    def __init__(self, scene: Scene, camera: Camera, width: int, height: int, spp: int, depth: int, sky, lights,
                 tile_rank: int = 0, tile_count: int = 1, stream=None, caustic_k: int = 0):
        self.width, self.height = int(width), int(height)
        self._scene = scene   # keeps the scene alive while the job refers to it
        p = RenderParams(self.width, self.height, int(spp), int(depth), camera, _f3(sky), int(tile_rank),
                         int(tile_count), int(caustic_k))
        la = lights_array(lights)
        h = _P()
        _check(_lib.pm_render_begin(scene.handle, C.byref(p), la, len(lights), C.byref(h), _stream(stream)),
               "pm_render_begin")
        self._h = h.value

    def gather_caustic(self, caustic_map: PhotonMap, stream=None):
        """pm_render_gather_caustic: the caustic gather now, ahead of finish()
        (which then takes caustic_map=None or this same map)."""
        _check(_lib.pm_render_gather_caustic(self._h, caustic_map.handle, _stream(stream)),
               "pm_render_gather_caustic")

    def finish(self, global_map: PhotonMap, caustic_map: Optional[PhotonMap], want_rgb: bool = True, rgba=None,
               stream=None):
        import torch
        if rgba is None:
            rgba = torch.zeros((self.height, self.width), dtype=torch.int32, device="cuda")
        rgb = torch.zeros((self.height, self.width, 3), dtype=torch.float32, device="cuda") if want_rgb else None
        _check(_lib.pm_render_finish(self._h, global_map.handle, caustic_map.handle if caustic_map else None,
                                     _ptr(rgba), _ptr(rgb), _stream(stream)), "pm_render_finish")
        return rgba, rgb

    def queries(self, which: str = "global", results: bool = True, stream=None):
        """pm_render_job_queries: (queries (n, 4) = hit point + brdf, results
        (n, 4) = radiance + 0 or None) of the "global" or "caustic" gather,
        in the job's dense order; results only after finish()."""
        import torch
        w = {"global": 0, "caustic": 1}[which]
        n = C.c_int64(0)
        _check(_lib.pm_render_job_queries(self._h, w, None, None, 0, C.byref(n), None), "pm_render_job_queries")
        q = torch.empty((max(1, n.value), 4), dtype=torch.float32, device="cuda")
        r = torch.empty((max(1, n.value), 4), dtype=torch.float32, device="cuda") if results else None
        _check(_lib.pm_render_job_queries(self._h, w, _ptr(q), _ptr(r), q.shape[0], C.byref(n), _stream(stream)),
               "pm_render_job_queries")
        return q[: n.value], (r[: n.value] if r is not None else None)

    def close(self):
        if getattr(self, "_h", None):
            _lib.pm_render_job_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def render_begin(scene: Scene, camera: Camera, width: int, height: int, spp: int, depth: int, sky, lights,
                 tile_rank: int = 0, tile_count: int = 1, stream=None, caustic_k: int = 0) -> RenderJob:
    return RenderJob(scene, camera, width, height, spp, depth, sky, lights, tile_rank, tile_count, stream,
                     caustic_k=caustic_k)


def view_photons(scene: Scene, photons, look_from, look_at, look_up, fovy: float, width: int, height: int,
                 stream=None):
    """photonViewer run() (photon-viewer/src/hostCode.cu:109-154): splat a photon
    array (N x 10 float32, device) onto a width x height RGBA8 image (int32 [H][W])."""
    import torch
    p = ViewerParams(_f3(look_from), _f3(look_at), _f3(look_up), float(fovy), int(width), int(height))
    rgba = torch.empty((height, width), dtype=torch.int32, device="cuda")
    _check(_lib.pm_photon_view(scene.handle, _ptr(photons), photons.shape[0], C.byref(p), _ptr(rgba),
                               _stream(stream)), "pm_photon_view")
    return rgba


def render_stats() -> RenderStats:
    s = RenderStats()
    _lib.pm_render_stats_get(C.byref(s))
    return s


# ----------------------------------------------------------------- files
def write_alive_photons(photons: np.ndarray, filename: str):
    """writeAlivePhotons (photon-mapping/src/hostCode.cu:31-49); photons (n,10) float32."""
    a = np.ascontiguousarray(photons, np.float32)
    _check(_lib.pm_photons_write_txt(filename.encode(), a.ctypes.data if len(a) else None, len(a)),
           "writeAlivePhotons")


def read_photons_from_file(filename: str) -> np.ndarray:
    """readPhotonsFromFile (ray-tracer/src/hostCode.cu:26-52): (n,10) float32, n = 0 if missing."""
    p = _P()
    n = C.c_int64()
    _check(_lib.pm_photons_read_txt(filename.encode(), C.byref(p), C.byref(n)), "readPhotonsFromFile")
    if n.value == 0:
        return np.zeros((0, 10), np.float32)
    arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), (n.value * 10,)).reshape(-1, 10).copy()
    _lib.pm_free(p)
    return arr


def quantize_photons(photons, stream=None):
    """In place: the %.6f text round trip (write_alive_photons ->
    read_photons_from_file) applied on the device."""
    _check(_lib.pm_photons_quantize(_ptr(photons), photons.shape[0], _stream(stream)), "pm_photons_quantize")
    return photons


def write_photons_bin(photons: np.ndarray, filename: str):
    ph = np.ascontiguousarray(photons, np.float32)
    _check(_lib.pm_photons_write_bin(filename.encode(), ph.ctypes.data, len(ph)), "pm_photons_write_bin")


def read_photons_bin(filename: str) -> np.ndarray:
    h = _P()
    n = C.c_int64()
    _check(_lib.pm_photons_read_bin(filename.encode(), C.byref(h), C.byref(n)), "pm_photons_read_bin")
    try:
        if n.value == 0:
            return np.zeros((0, 10), np.float32)
        return np.ctypeslib.as_array(C.cast(h, C.POINTER(C.c_float)), (n.value * 10,)).reshape(-1, 10).copy()
    finally:
        _lib.pm_free(h)


def write_png(filename: str, rgba: np.ndarray):
    """stbi_write_png(filename, W, H, 4, fb, W*4) (ray-tracer/src/hostCode.cu:240)."""
    a = np.ascontiguousarray(rgba).view(np.uint32)
    h, w = a.shape
    _check(_lib.pm_write_png_rgba(filename.encode(), a.ctypes.data, w, h), "stbi_write_png")
