"""ctypes front end of oracle/liborc.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference render path (rt_oracle.c).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker / the timed CPU baseline -- never as a product path.
"""
from __future__ import annotations

import ctypes as C
import os
import time

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liborc.so")


class orc_vec3(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]


class orc_sphere(C.Structure):
    _fields_ = [("center", orc_vec3), ("radius", C.c_double), ("color", orc_vec3),
                ("reflectivity", C.c_double), ("shininess", C.c_double)]


class orc_light(C.Structure):
    _fields_ = [("position", orc_vec3), ("color", orc_vec3), ("intensity", C.c_double)]


class orc_scene(C.Structure):
    _fields_ = [("num_spheres", C.c_int), ("spheres", C.POINTER(orc_sphere)), ("num_lights", C.c_int),
                ("lights", C.POINTER(orc_light)), ("ambient", orc_vec3), ("cam_position", orc_vec3),
                ("cam_look_at", orc_vec3), ("cam_fov", C.c_double), ("has_camera", C.c_int),
                ("warnings", C.c_int)]


class orc_counts(C.Structure):
    _fields_ = [("primary", C.c_uint64), ("shadow", C.c_uint64), ("reflect", C.c_uint64),
                ("negative", C.c_uint64)]

    def as_dict(self):
        return {"primary": self.primary, "shadow": self.shadow, "reflect": self.reflect, "negative": self.negative}


class orc_camera(C.Structure):
    _fields_ = [("position", orc_vec3), ("forward", orc_vec3), ("right", orc_vec3), ("up", orc_vec3),
                ("scale", C.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise FileNotFoundError(f"{LIB} missing: run `make -C oracle`")
        L = C.CDLL(LIB)
        L.orc_load_scene.argtypes = [C.c_char_p, C.POINTER(orc_scene), C.c_int]
        L.orc_parse_scene.argtypes = [C.c_char_p, C.POINTER(orc_scene), C.c_int]
        L.orc_free_scene.argtypes = [C.POINTER(orc_scene)]
        L.orc_free_scene.restype = None
        L.orc_make_camera.argtypes = [C.POINTER(orc_scene), C.POINTER(orc_camera)]
        L.orc_make_camera.restype = None
        L.orc_intersect.argtypes = [C.POINTER(orc_sphere), orc_vec3, orc_vec3, C.POINTER(C.c_double)]
        L.orc_render.argtypes = [C.POINTER(orc_scene), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.c_void_p, C.c_void_p, C.POINTER(orc_counts), C.c_int]
        L.orc_render_cam.argtypes = [C.POINTER(orc_scene), C.POINTER(orc_camera), C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(orc_counts), C.c_int]
        L.orc_render_aa.argtypes = [C.POINTER(orc_scene), C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                    C.c_void_p, C.POINTER(orc_counts), C.c_int]
        L.orc_quantize.argtypes = [C.c_double]
        L.orc_tile_complexity.argtypes = [C.POINTER(orc_scene)] + [C.c_int] * 6
        _lib = L
    return _lib


class OracleScene:
    def __init__(self, path: str | None = None, text: str | None = None):
        self.s = orc_scene()
        if path is not None:
            if lib().orc_load_scene(os.fsencode(path), C.byref(self.s), 0) != 0:
                raise FileNotFoundError(path)
        else:
            lib().orc_parse_scene(text.encode(), C.byref(self.s), 0)

    def close(self):
        if self.s.spheres:
            lib().orc_free_scene(C.byref(self.s))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def camera(self) -> orc_camera:
        c = orc_camera()
        lib().orc_make_camera(C.byref(self.s), C.byref(c))
        return c

    def render(self, W, H, depth, band=1, first=0, stride=1, count=None, threads=1, want_fb=False, camera=None):
        """Returns (rgb bytes, counts dict, seconds[, fb doubles]).  `camera`: any
        object with position/forward/right/up (3 doubles) and scale (an
        rt_hip.rt_camera), else the scene's camera."""
        count = H if count is None else count
        rgb = (C.c_uint8 * (count * W * 3))()
        fb = (C.c_double * (count * W * 3))() if want_fb else None
        cnt = orc_counts()
        t0 = time.perf_counter()
        cam = None
        if isinstance(camera, orc_camera):
            cam = camera
        elif camera is not None:
            cam = orc_camera()
            for f in ("position", "forward", "right", "up"):
                v = getattr(camera, f)
                getattr(cam, f).x, getattr(cam, f).y, getattr(cam, f).z = v[0], v[1], v[2]
            cam.scale = camera.scale
        rc = lib().orc_render_cam(C.byref(self.s), C.byref(cam) if cam is not None else None, W, H, depth, band,
                                  first, stride, count, C.cast(rgb, C.c_void_p),
                                  C.cast(fb, C.c_void_p) if fb is not None else None, C.byref(cnt), threads)
        dt = time.perf_counter() - t0
        if rc != 0:
            raise ValueError("orc_render rejected its arguments")
        out = (bytes(rgb), cnt.as_dict(), dt)
        return out + (list(fb),) if want_fb else out


    def render_aa(self, W, H, depth, samples=4, threads=1, want_fb=False):
        """Antialias mode (main_gpu.cu:249-333, serial fp64 semantics), full frame.
        Returns (rgb bytes, counts dict, seconds[, fb doubles in PPM row order])."""
        rgb = (C.c_uint8 * (H * W * 3))()
        fb = (C.c_double * (H * W * 3))() if want_fb else None
        cnt = orc_counts()
        t0 = time.perf_counter()
        rc = lib().orc_render_aa(C.byref(self.s), W, H, depth, samples, C.cast(rgb, C.c_void_p),
                                 C.cast(fb, C.c_void_p) if fb is not None else None, C.byref(cnt), threads)
        dt = time.perf_counter() - t0
        if rc != 0:
            raise ValueError("orc_render_aa rejected its arguments")
        out = (bytes(rgb), cnt.as_dict(), dt)
        return out + (list(fb),) if want_fb else out


def hybrid_tiles(scene: "OracleScene", W: int, H: int, tile: int, threshold: int):
    """The hybrid driver's tile split (src/main_hybrid.cpp:351-395 / :487-527):
    tiles in scanline order of tile rows, (x0, y0, x1, y1, complexity, to_cpu)
    with to_cpu = complexity > threshold."""
    out = []
    for y in range(0, H, tile):
        for x in range(0, W, tile):
            x1, y1 = min(x + tile, W), min(y + tile, H)
            c = lib().orc_tile_complexity(C.byref(scene.s), x, y, x1, y1, W, H)
            out.append((x, y, x1, y1, c, c > threshold))
    return out


def intersect(center, radius, origin, direction):
    s = orc_sphere(orc_vec3(*center), radius, orc_vec3(0, 0, 0), 0.0, 0.0)
    t = C.c_double(0.0)
    hit = lib().orc_intersect(C.byref(s), orc_vec3(*origin), orc_vec3(*direction), C.byref(t))
    return bool(hit), t.value


def quantize(c: float) -> int:
    return lib().orc_quantize(c)
