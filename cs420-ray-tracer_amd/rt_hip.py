"""ctypes binding of include/rt_hip.h (librt_hip.so) -- the Python host mirror.

This is the binding a reference-side maintainer would add to drive the HIP
render loop from Python; the C++ host (csrc/ray_hip.cpp) uses the same ABI.
Nothing here falls back to a CPU path: if librt_hip.so is missing or no GPU is
visible the calls raise.

Reference interfaces mirrored (file:line in shininglegend/cs420-ray-tracer):
  load_scene            include/scene_loader.h:27-135   -> Scene.load / Scene.parse
  Camera(pos, look, fov) include/camera.h:10-15          -> Camera.from_scene
  trace_ray pixel loop   src/main.cpp:146-157            -> Renderer.render
  launch_gpu_kernel      src/kernel.cu:185-200           -> Renderer.render_async
  write_ppm              src/main.cpp:69-91              -> write_ppm
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# RT_HIP_LIB selects an alternative build of the same ABI (tuning experiments).
LIB_PATH = os.environ.get("RT_HIP_LIB") or os.path.join(HERE, "librt_hip.so")
# Test builds of the same sources (csrc/Makefile), selected per context with
# Renderer(variant=...): "tuning" reads every layout / grid knob (RT_TUNING),
# "check" range-checks every indirect device index (RT_CHECK).  The product
# build reads only RT_HIP_LDS_SCENE and RT_HIP_CAM_GRID.
VARIANTS = {"tuning": os.path.join(HERE, "variants", "librt_hip_tuning.so"),
            "check": os.path.join(HERE, "variants", "librt_hip_check.so")}

RT_MAX_DEPTH = 64
ABI_VERSION = 12  # RT_HIP_ABI_VERSION in include/rt_hip.h
MAX_FRAMES = 32  # RT_MAX_FRAMES


class RtError(RuntimeError):
    def __init__(self, status: int, what: str, detail: str = ""):
        self.status = status
        super().__init__(f"{what}: {status_string(status)}" + (f" ({detail})" if detail else ""))


class rt_sphere(C.Structure):
    _fields_ = [("center", C.c_double * 3), ("radius", C.c_double), ("color", C.c_double * 3),
                ("reflectivity", C.c_double), ("shininess", C.c_double)]


class rt_light(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("color", C.c_double * 3), ("intensity", C.c_double)]


class rt_scene(C.Structure):
    _fields_ = [("num_spheres", C.c_int32), ("num_lights", C.c_int32),
                ("spheres", C.POINTER(rt_sphere)), ("lights", C.POINTER(rt_light)),
                ("ambient", C.c_double * 3), ("cam_position", C.c_double * 3),
                ("cam_look_at", C.c_double * 3), ("cam_fov", C.c_double),
                ("has_camera", C.c_int32), ("warnings", C.c_int32)]


class rt_camera(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("forward", C.c_double * 3), ("right", C.c_double * 3),
                ("up", C.c_double * 3), ("scale", C.c_double)]


class rt_info(C.Structure):
    _fields_ = [("cam_grid_last", C.c_int32), ("cam_grid_n", C.c_int32), ("cam_grid_builds", C.c_uint64),
                ("cam_grid_build_ms", C.c_double), ("tile_order_builds", C.c_uint64),
                ("tile_order_build_ms", C.c_double), ("upload_ms", C.c_double), ("launches", C.c_uint64),
                ("sphere_grids", C.c_int32), ("sphere_grid_n", C.c_int32), ("sphere_grid_entries", C.c_uint64),
                ("sphere_grid_build_ms", C.c_double), ("behind_grid", C.c_int32), ("behind_grid_last", C.c_int32),
                ("behind_grid_cells", C.c_uint64), ("behind_grid_entries", C.c_uint64),
                ("behind_grid_build_ms", C.c_double), ("bvh_build_ms", C.c_double),
                ("light_grid_build_ms", C.c_double), ("scratch_bytes", C.c_uint64),
                ("shadow_line_bounded", C.c_int32), ("reserved0", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class rt_tile(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("width", C.c_int32), ("height", C.c_int32)]


class rt_rows(C.Structure):
    _fields_ = [("band", C.c_int32), ("first", C.c_int32), ("stride", C.c_int32), ("count", C.c_int32)]


class rt_stats(C.Structure):
    _fields_ = [("rays_primary", C.c_uint64), ("rays_shadow", C.c_uint64), ("rays_reflect", C.c_uint64),
                ("negative_clamped", C.c_uint64), ("kernel_ms", C.c_double), ("tests_exact", C.c_uint64),
                ("tests_cull", C.c_uint64)]

    def as_dict(self):
        return {"primary": self.rays_primary, "shadow": self.rays_shadow, "reflect": self.rays_reflect,
                "negative": self.negative_clamped, "kernel_ms": self.kernel_ms, "tests_exact": self.tests_exact,
                "tests_cull": self.tests_cull}

    @property
    def rays(self) -> int:
        return self.rays_primary + self.rays_shadow + self.rays_reflect


# Every symbol include/rt_hip.h declares, with its ctypes signature.
_P = C.c_void_p
SIGNATURES = {
    "rt_scene_load": (C.c_int, [C.c_char_p, C.POINTER(rt_scene), C.c_int]),
    "rt_scene_parse": (C.c_int, [C.c_char_p, C.POINTER(rt_scene), C.c_int]),
    "rt_scene_free": (None, [C.POINTER(rt_scene)]),
    "rt_camera_from_scene": (C.c_int, [C.POINTER(rt_scene), C.POINTER(rt_camera)]),
    "rt_write_ppm": (C.c_int, [C.c_char_p, _P, C.c_int, C.c_int, C.c_int]),
    "rt_error_string": (C.c_char_p, [C.c_int]),
    "rt_abi_version": (C.c_int, []),
    "rt_rows_for_shard": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(rt_rows)]),
    "rt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rt_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "rt_destroy": (None, [_P]),
    "rt_last_error": (C.c_char_p, [_P]),
    "rt_set_stream": (C.c_int, [_P, _P]),
    "rt_upload_scene": (C.c_int, [_P, C.POINTER(rt_scene)]),
    "rt_set_culling": (C.c_int, [_P, C.c_int]),
    "rt_render": (C.c_int, [_P, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int, C.POINTER(rt_rows), _P,
                            C.c_int, C.POINTER(rt_stats)]),
    "rt_render_async": (C.c_int, [_P, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int, C.POINTER(rt_rows), _P]),
    "rt_render_stats": (C.c_int, [_P, C.POINTER(rt_stats)]),
    "rt_render_frames_async": (C.c_int, [_P, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(rt_rows), _P, C.c_size_t]),
    "rt_kernel_times": (C.c_int, [_P, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int)]),
    "rt_unpermute_rows": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "rt_render_tile": (C.c_int, [_P, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.c_int, _P]),
    "rt_render_tiles": (C.c_int, [_P, C.POINTER(rt_camera), C.c_int, C.c_int, C.c_int, C.POINTER(rt_tile), C.c_int,
                                  C.c_int, _P]),
    "rt_set_antialias": (C.c_int, [_P, C.c_int]),
    "rt_get_info": (C.c_int, [_P, C.POINTER(rt_info)]),
}

# include/rt_hip_compat.h: the reference's hybrid interface (src/kernel.cu:185-207),
# struct layouts of include/gpu_shared.h:84-171
class rt_float3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class rt_gpu_material(C.Structure):
    _fields_ = [("albedo", rt_float3), ("metallic", C.c_float), ("shininess", C.c_float)]


class rt_gpu_sphere(C.Structure):
    _fields_ = [("center", rt_float3), ("radius", C.c_float), ("material", rt_gpu_material)]


class rt_gpu_light(C.Structure):
    _fields_ = [("position", rt_float3), ("color", rt_float3), ("intensity", C.c_float)]


class rt_gpu_camera(C.Structure):
    _fields_ = [("origin", rt_float3), ("lower_left", rt_float3), ("horizontal", rt_float3),
                ("vertical", rt_float3), ("forward", rt_float3), ("right", rt_float3), ("up", rt_float3),
                ("fov", C.c_float)]


COMPAT_SIGNATURES = {
    "launch_gpu_kernel": (None, [C.POINTER(rt_float3), C.POINTER(rt_gpu_sphere), C.c_int, C.c_int,
                                 C.POINTER(rt_gpu_camera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, _P]),
    "upload_lights_and_ambience": (None, [C.POINTER(rt_gpu_light), C.c_int, rt_float3]),
    "rt_compat_status": (C.c_int, []),
}

# framebuffer formats of rt_render_tile (rt_hip.h)
RT_FB_RGB8, RT_FB_F32X3, RT_FB_F64X3 = 0, 1, 2

_libs = {}


def lib(path: str = LIB_PATH):
    """Load librt_hip.so (or a test variant of it; raises if it has not been built)."""
    _lib = _libs.get(path)
    if _lib is None:
        # torch bundles its own libamdhip64.so (SONAME libamdhip64.so.7).  If it
        # is importable, load it first so the dynamic linker binds librt_hip.so
        # to that same HIP runtime: two runtimes in one process cannot share
        # the device (torch then reports "No HIP GPUs are available").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run __graft_entry__.build() (no CPU fallback exists)")
        L = C.CDLL(path)
        for name, (res, args) in list(SIGNATURES.items()) + list(COMPAT_SIGNATURES.items()):
            if os.environ.get("RT_HIP_LIB") and not hasattr(L, name):
                continue  # an older diagnostic build (RT_HIP_LIB) may predate an entry point
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _libs[path] = _lib = L
    return _lib


def variant_lib(variant: str | None):
    """The library of a test variant ("tuning", "check") or the product's (None)."""
    if variant is None:
        return lib()
    if variant not in VARIANTS:
        raise ValueError(f"unknown librt_hip variant {variant!r} (one of {sorted(VARIANTS)})")
    return lib(VARIANTS[variant])


def status_string(status: int) -> str:
    try:
        return lib().rt_error_string(status).decode()
    except Exception:  # pragma: no cover - only when the library itself is missing
        return f"status {status}"


def _check(rc: int, what: str, ctx=None, L=None):
    if rc != 0:
        detail = (L or lib()).rt_last_error(ctx).decode() if ctx else ""
        raise RtError(rc, what, detail)


class Scene:
    """A parsed scene (owns the C arrays).  Mirrors load_scene(), scene_loader.h:27."""

    def __init__(self):
        self._s = rt_scene()
        self._owned = False

    @classmethod
    def load(cls, path: str, verbose: bool = False) -> "Scene":
        s = cls()
        _check(lib().rt_scene_load(os.fsencode(path), C.byref(s._s), int(verbose)), f"rt_scene_load({path})")
        s._owned = True
        return s

    @classmethod
    def parse(cls, text: str, verbose: bool = False) -> "Scene":
        s = cls()
        _check(lib().rt_scene_parse(text.encode(), C.byref(s._s), int(verbose)), "rt_scene_parse")
        s._owned = True
        return s

    @property
    def raw(self) -> rt_scene:
        return self._s

    @property
    def num_spheres(self) -> int:
        return self._s.num_spheres

    @property
    def num_lights(self) -> int:
        return self._s.num_lights

    @property
    def warnings(self) -> int:
        return self._s.warnings

    def sphere(self, i: int) -> dict:
        sp = self._s.spheres[i]
        return {"center": tuple(sp.center), "radius": sp.radius, "color": tuple(sp.color),
                "reflectivity": sp.reflectivity, "shininess": sp.shininess}

    def light(self, i: int) -> dict:
        L = self._s.lights[i]
        return {"position": tuple(L.position), "color": tuple(L.color), "intensity": L.intensity}

    def camera(self) -> rt_camera:
        cam = rt_camera()
        _check(lib().rt_camera_from_scene(C.byref(self._s), C.byref(cam)), "rt_camera_from_scene")
        return cam

    def close(self):
        if self._owned:
            lib().rt_scene_free(C.byref(self._s))
            self._owned = False

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def camera_array(cams) -> C.Array:
    """The rt_camera array rt_render_frames_async takes, built once (a caller
    that launches the same frames repeatedly keeps it off its launch path)."""
    return (rt_camera * len(cams))(*cams)


def rows_for_shard(height: int, band: int, rank: int, world: int) -> rt_rows:
    """Cyclic bands of `band` rows: rank r renders bands r, r+G, r+2G, ...
    (rt_rows_for_shard: the one layout ray_hip --gpus and bench.py share)."""
    rows = rt_rows()
    _check(lib().rt_rows_for_shard(height, band, rank, world, C.byref(rows)),
           f"rt_rows_for_shard({height}, {band}, {rank}, {world})")
    return rows


class Renderer:
    """One device context (rt_ctx).  Mirrors GPUResources + launch_gpu_kernel."""

    def __init__(self, device: int = 0, variant: str | None = None):
        """variant: None = the product library; "tuning" / "check" = a test build (VARIANTS)."""
        self._L = variant_lib(variant)
        self.variant = variant
        self._ctx = C.c_void_p()
        _check(self._L.rt_create(device, C.byref(self._ctx)), f"rt_create({device})", L=self._L)
        self.device = device

    @property
    def handle(self):
        return self._ctx

    def set_stream(self, stream_ptr: int | None):
        _check(self._L.rt_set_stream(self._ctx, C.c_void_p(stream_ptr or 0)), "rt_set_stream", self._ctx, L=self._L)

    def set_culling(self, enable: bool):
        _check(self._L.rt_set_culling(self._ctx, int(enable)), "rt_set_culling", self._ctx, L=self._L)

    def upload(self, scene: Scene):
        _check(self._L.rt_upload_scene(self._ctx, C.byref(scene.raw)), "rt_upload_scene", self._ctx, L=self._L)

    def render(self, cam: rt_camera, width: int, height: int, depth: int, rows: rt_rows | None = None,
               out=None, out_on_device: bool = False) -> tuple[object, rt_stats]:
        """Render into `out` (host bytearray/numpy if None) and return (buffer, stats)."""
        count = rows.count if rows is not None else height
        if out is None:
            out = bytearray(count * width * 3)
        ptr = _addr(out)
        st = rt_stats()
        _check(self._L.rt_render(self._ctx, C.byref(cam), width, height, depth,
                               C.byref(rows) if rows is not None else None, C.c_void_p(ptr), int(out_on_device),
                               C.byref(st)), "rt_render", self._ctx, L=self._L)
        return out, st

    def render_async(self, cam: rt_camera, width: int, height: int, depth: int, rows: rt_rows | None,
                     out_device_ptr: int):
        _check(self._L.rt_render_async(self._ctx, C.byref(cam), width, height, depth,
                                     C.byref(rows) if rows is not None else None, C.c_void_p(out_device_ptr)),
               "rt_render_async", self._ctx, L=self._L)

    def render_frames_async(self, cams, width: int, height: int, depth: int, rows: rt_rows | None,
                            out_device_ptr: int, frame_stride: int):
        """rt_render_frames_async: len(cams) frames (<= MAX_FRAMES) in one launch, frame f
        (seen through cams[f]) at out_device_ptr + f * frame_stride.  `cams` may
        be a ctypes array of rt_camera built beforehand (camera_array)."""
        arr = cams if isinstance(cams, C.Array) else (rt_camera * len(cams))(*cams)
        _check(self._L.rt_render_frames_async(self._ctx, arr, len(cams), width, height, depth,
                                            C.byref(rows) if rows is not None else None,
                                            C.c_void_p(out_device_ptr), frame_stride),
               "rt_render_frames_async", self._ctx, L=self._L)

    def set_antialias(self, samples: int):
        """1 = the serial path, 4 = the reference GPU's `-a` mode (main_gpu.cu:249-333)."""
        _check(self._L.rt_set_antialias(self._ctx, samples), "rt_set_antialias", self._ctx, L=self._L)

    def render_tile(self, cam: rt_camera, width: int, height: int, depth: int, tile_x: int, tile_y: int,
                    tile_w: int, tile_h: int, fb_format: int, fb_device_ptr: int):
        """launch_gpu_kernel tile semantics (kernel.cu:185-200) into a full-image device framebuffer."""
        _check(self._L.rt_render_tile(self._ctx, C.byref(cam), width, height, depth, tile_x, tile_y, tile_w, tile_h,
                                    fb_format, C.c_void_p(fb_device_ptr)), "rt_render_tile", self._ctx, L=self._L)

    def render_tiles(self, cam: rt_camera, width: int, height: int, depth: int, tiles, fb_format: int,
                     fb_device_ptr: int):
        """rt_render_tiles: every (x, y, w, h) tile of `tiles` in ONE launch (the 8x8 blocks covering them)."""
        arr = (rt_tile * max(1, len(tiles)))(*[rt_tile(*t) for t in tiles])
        _check(self._L.rt_render_tiles(self._ctx, C.byref(cam), width, height, depth, arr, len(tiles), fb_format,
                                     C.c_void_p(fb_device_ptr)), "rt_render_tiles", self._ctx, L=self._L)

    def stats(self) -> rt_stats:
        st = rt_stats()
        _check(self._L.rt_render_stats(self._ctx, C.byref(st)), "rt_render_stats", self._ctx, L=self._L)
        return st

    def info(self) -> rt_info:
        """rt_get_info: the host-side builds the render calls made (camera grid, tile order)."""
        inf = rt_info()
        _check(self._L.rt_get_info(self._ctx, C.byref(inf)), "rt_get_info", self._ctx, L=self._L)
        return inf

    def kernel_times(self, max_n: int = 256) -> list[float]:
        """Per-launch kernel durations (ms) since the previous call (syncs the stream)."""
        buf = (C.c_double * max_n)()
        n = C.c_int(0)
        _check(self._L.rt_kernel_times(self._ctx, buf, max_n, C.byref(n)), "rt_kernel_times", self._ctx, L=self._L)
        return list(buf[: n.value])

    def unpermute(self, gathered_ptr: int, image_ptr: int, width: int, height: int, band: int, shards: int,
                  rows_per_shard: int):
        _check(self._L.rt_unpermute_rows(self._ctx, C.c_void_p(gathered_ptr), C.c_void_p(image_ptr), width, height,
                                       band, shards, rows_per_shard), "rt_unpermute_rows", self._ctx, L=self._L)

    def close(self):
        if self._ctx:
            self._L.rt_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _addr(buf) -> int:
    if isinstance(buf, bytes):
        return C.cast(C.c_char_p(buf), C.c_void_p).value
    if isinstance(buf, bytearray):
        return C.addressof((C.c_char * len(buf)).from_buffer(buf))
    if hasattr(buf, "ctypes"):  # numpy
        return buf.ctypes.data
    if hasattr(buf, "data_ptr"):  # torch
        return buf.data_ptr()
    raise TypeError(type(buf))


def write_ppm(path: str, rgb, width: int, height: int, binary: bool = False):
    _check(lib().rt_write_ppm(os.fsencode(path), C.c_void_p(_addr(rgb)), width, height, int(binary)), "rt_write_ppm")


def device_count() -> int:
    n = C.c_int(0)
    lib().rt_device_count(C.byref(n))
    return n.value
