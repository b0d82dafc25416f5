"""ctypes binding of the CPU restatement in oracle/rtp_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- as the checker / timed CPU baseline, never as
the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "librtp_oracle.so")

MAX_POINTS = 8192
MAX_QUADS = 2048
MAX_SPHERES = 2048
MAX_MATS = 16


class Scene(ctypes.Structure):
    """Mirror of rtpo_scene (rtp_oracle.h)."""

    _fields_ = [
        ("n_points", ctypes.c_int32),
        ("points", (ctypes.c_float * 3) * MAX_POINTS),
        ("n_quads", ctypes.c_int32),
        ("quad_ids", (ctypes.c_int32 * 5) * MAX_QUADS),
        ("quad_mat", ctypes.c_int32 * MAX_QUADS),
        ("quad_tex", ctypes.c_int32 * MAX_QUADS),
        ("n_spheres", ctypes.c_int32),
        ("sphere_point", ctypes.c_int32 * MAX_SPHERES),
        ("sphere_radius", ctypes.c_float * MAX_SPHERES),
        ("sphere_mat", ctypes.c_int32 * MAX_SPHERES),
        ("sphere_tex", ctypes.c_int32 * MAX_SPHERES),
        ("n_mat", ctypes.c_int32),
        ("mat_type", ctypes.c_int32 * MAX_MATS),
        ("n_tex_type", ctypes.c_int32),
        ("tex_type", ctypes.c_int32 * MAX_MATS),
        ("n_tex", ctypes.c_int32),
        ("tex", (ctypes.c_float * 3) * MAX_MATS),
        ("light_box_pointids", ctypes.c_int32 * 5),
        ("light_sphere_point", ctypes.c_int32),
        ("ior", ctypes.c_float),
        ("n_field", ctypes.c_int32),
        ("field", ctypes.c_float * (MAX_POINTS + 16)),
    ]

    # numpy views -------------------------------------------------------
    def points_np(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.points)[: self.n_points].copy()

    def quad_ids_np(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.quad_ids)[: self.n_quads].copy()


def build(force: bool = False) -> str:
    """Compile librtp_oracle.so with the committed Makefile (gcc)."""
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(
        os.path.getmtime(os.path.join(_HERE, f)) for f in ("rtp_oracle.c", "rtp_oracle.h", "Makefile")
    ):
        subprocess.run(["make", "-s", "-C", _HERE, "-B" if force else "librtp_oracle.so"], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        f32p = ctypes.POINTER(ctypes.c_float)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.rtpo_camera_setup.argtypes = [f32p, f32p, f32p, ctypes.c_float, ctypes.c_int32, ctypes.c_int32, f32p]
        L.rtpo_cornell_box.argtypes = [ctypes.c_int32, ctypes.POINTER(Scene)]
        L.rtpo_render_pixels.argtypes = [ctypes.POINTER(Scene), f32p, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, i64p, ctypes.c_int64,
                                         f32p, u32p, u32p, ctypes.c_int32]
        L.rtpo_render_soa.argtypes = [ctypes.POINTER(Scene), f32p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, f32p, u32p,
                                      u32p, ctypes.c_int32]
        L.rtpo_render_soa.restype = ctypes.c_int32
        L.rtpo_normalize.argtypes = [f32p, ctypes.c_int64, ctypes.c_int32]
        L.rtpo_wang32.argtypes = [ctypes.c_uint32]
        L.rtpo_wang32.restype = ctypes.c_uint32
        L.rtpo_randf.argtypes = [u32p]
        L.rtpo_randf.restype = ctypes.c_float
        L.rtpo_sinf.argtypes = [ctypes.c_float]
        L.rtpo_sinf.restype = ctypes.c_float
        L.rtpo_cosf.argtypes = [ctypes.c_float]
        L.rtpo_cosf.restype = ctypes.c_float
        L.rtpo_which.argtypes = [ctypes.c_uint32]
        L.rtpo_which.restype = ctypes.c_int32
        _lib = L
    return _lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _up(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def cornell_box(variant: int = 0) -> Scene:
    s = Scene()
    lib().rtpo_cornell_box(variant, ctypes.byref(s))
    return s


# main.cc:616-622 default camera
DEFAULT_CAMERA = dict(
    position=np.array([278 / 555.0, 278 / 555.0, -800 / 555.0], dtype=np.float32),
    look_at=np.array([278 / 555.0, 278 / 555.0, 278 / 555.0], dtype=np.float32),
    view_up=np.array([0, 1, 0], dtype=np.float32),
    fov_y=np.float32(40.0),
)


def camera_setup(nx: int, ny: int, position=None, look_at=None, view_up=None, fov_y=None) -> np.ndarray:
    c = DEFAULT_CAMERA
    pos = np.ascontiguousarray(c["position"] if position is None else position, dtype=np.float32)
    la = np.ascontiguousarray(c["look_at"] if look_at is None else look_at, dtype=np.float32)
    up = np.ascontiguousarray(c["view_up"] if view_up is None else view_up, dtype=np.float32)
    fov = float(c["fov_y"] if fov_y is None else fov_y)
    out = np.zeros(12, dtype=np.float32)
    lib().rtpo_camera_setup(_fp(pos), _fp(la), _fp(up), fov, nx, ny, _fp(out))
    return out


def render_pixels(scene: Scene, cam: np.ndarray, nx: int, ny: int, spp: int, depth: int, pixels,
                  seed_base: int = 0, nthreads: int = 0):
    """Scalar per-pixel oracle. Returns (rgba_sum[n,4], final_seed[n], live_bounces[n])."""
    pix = np.ascontiguousarray(pixels, dtype=np.int64)
    n = pix.size
    rgba = np.zeros((n, 4), dtype=np.float32)
    seeds = np.zeros(n, dtype=np.uint32)
    live = np.zeros(n, dtype=np.uint32)
    cam = np.ascontiguousarray(cam, dtype=np.float32)
    lib().rtpo_render_pixels(ctypes.byref(scene), _fp(cam), nx, ny, spp, depth, seed_base,
                             pix.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n, _fp(rgba), _up(seeds),
                             _up(live), nthreads)
    return rgba, seeds, live


def render_soa(scene: Scene, cam: np.ndarray, nx: int, ny: int, spp: int, depth: int, seed_base: int = 0,
               row_begin: int = 0, row_end: int | None = None, nthreads: int = 1):
    """Stage-structured oracle (the timed CPU baseline)."""
    row_end = ny if row_end is None else row_end
    n = (row_end - row_begin) * nx
    rgba = np.zeros((n, 4), dtype=np.float32)
    seeds = np.zeros(n, dtype=np.uint32)
    live = np.zeros(n, dtype=np.uint32)
    cam = np.ascontiguousarray(cam, dtype=np.float32)
    rc = lib().rtpo_render_soa(ctypes.byref(scene), _fp(cam), nx, ny, spp, depth, seed_base, row_begin, row_end,
                               _fp(rgba), _up(seeds), _up(live), nthreads)
    if rc != 0:
        raise ValueError("rtpo_render_soa: invalid arguments")
    return rgba, seeds, live


def normalize(rgba: np.ndarray, spp: int) -> np.ndarray:
    out = np.ascontiguousarray(rgba, dtype=np.float32).copy()
    lib().rtpo_normalize(_fp(out), out.shape[0], spp)
    return out


def wang32(x: int) -> int:
    return int(lib().rtpo_wang32(x))


def randf_stream(seed: int, n: int):
    s = ctypes.c_uint32(seed)
    vals = [float(lib().rtpo_randf(ctypes.byref(s))) for _ in range(n)]
    return vals, int(s.value)


# ------------------------------------------------------------ -direct mode ---
class DirectCam(ctypes.Structure):
    """Mirror of rtpo_direct_cam."""

    _fields_ = [("eye", ctypes.c_float * 3), ("nlook", ctypes.c_float * 3), ("dx", ctypes.c_float * 3),
                ("dy", ctypes.c_float * 3), ("nx", ctypes.c_int32), ("ny", ctypes.c_int32),
                ("sub_x0", ctypes.c_int32), ("sub_y0", ctypes.c_int32), ("sub_w", ctypes.c_int32),
                ("sub_h", ctypes.c_int32), ("vp", ctypes.c_float * 16), ("light", ctypes.c_float * 3),
                ("view_dir", ctypes.c_float * 3)]


AOV_COLOR, AOV_NORMALS, AOV_ALBEDO = 1, 2, 4

# main.cc:120-176: the 24-colour "pallet" handed to ColorTable(name, RGB, nan,
# rgbPoints, alphaPoints) -- read by VTK-m as (x, r, g, b) quadruples
_C1, _C2, _C3 = [0.65, 0.05, 0.05], [0.73, 0.73, 0.73], [0.12, 0.45, 0.15]
MAIN_PALLET = np.array(_C3 + _C1 + _C2 + _C2 * 21, dtype=np.float64)
MAIN_ALPHA = np.ones(24, dtype=np.float64)


def _direct_fns():
    L = lib()
    if not hasattr(L, "_direct_ready"):
        f32p = ctypes.POINTER(ctypes.c_float)
        d64p = ctypes.POINTER(ctypes.c_double)
        L.rtpo_direct_setup.argtypes = [ctypes.POINTER(Scene), f32p, f32p, f32p, ctypes.c_float, ctypes.c_float,
                                        ctypes.c_float, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(DirectCam)]
        L.rtpo_quad_scalars.argtypes = [ctypes.POINTER(Scene), f32p]
        L.rtpo_sample_color_table.argtypes = [d64p, ctypes.c_int32, d64p, ctypes.c_int32, d64p, ctypes.c_int32, f32p]
        L.rtpo_sample_color_table.restype = ctypes.c_int32
        L.rtpo_render_direct.argtypes = [ctypes.POINTER(Scene), ctypes.POINTER(DirectCam), f32p, f32p, ctypes.c_int32,
                                         f32p, ctypes.c_int32, ctypes.c_int32, f32p, f32p]
        L._direct_ready = True
    return L


def direct_setup(scene: Scene, nx: int, ny: int, position=None, look_at=None, view_up=None, fov_y=None,
                 clip=(0.1, 5.0)) -> DirectCam:
    c = DEFAULT_CAMERA
    pos = np.ascontiguousarray(c["position"] if position is None else position, dtype=np.float32)
    la = np.ascontiguousarray(c["look_at"] if look_at is None else look_at, dtype=np.float32)
    up = np.ascontiguousarray(c["view_up"] if view_up is None else view_up, dtype=np.float32)
    fov = float(c["fov_y"] if fov_y is None else fov_y)
    out = DirectCam()
    _direct_fns().rtpo_direct_setup(ctypes.byref(scene), _fp(pos), _fp(la), _fp(up), fov, clip[0], clip[1], nx, ny,
                                    ctypes.byref(out))
    return out


def quad_scalars(scene: Scene) -> np.ndarray:
    out = np.zeros(scene.n_quads, dtype=np.float32)
    _direct_fns().rtpo_quad_scalars(ctypes.byref(scene), _fp(out))
    return out


def sample_color_table(rgb_points=MAIN_PALLET, alpha_points=MAIN_ALPHA, n: int = 1024, nan=(0.0, 0.0, 0.0)):
    rgb = np.ascontiguousarray(rgb_points, dtype=np.float64)
    al = np.ascontiguousarray(alpha_points, dtype=np.float64)
    nanc = np.ascontiguousarray(nan, dtype=np.float64)
    out = np.zeros((n, 4), dtype=np.float32)
    d64 = ctypes.POINTER(ctypes.c_double)
    rc = _direct_fns().rtpo_sample_color_table(rgb.ctypes.data_as(d64), rgb.size, al.ctypes.data_as(d64), al.size,
                                               nanc.ctypes.data_as(d64), n, _fp(out))
    if rc != 0:
        raise ValueError("rtpo_sample_color_table: bad arguments")
    return out


def render_direct(scene: Scene, cam: DirectCam, aov: int, cmap=None, qscalar=None, bg=(0, 0, 0, 1),
                  composite: bool = True):
    """One -direct mapper render. Returns (rgba[n,4], depth[n])."""
    cmap = sample_color_table() if cmap is None else np.ascontiguousarray(cmap, dtype=np.float32)
    qs = quad_scalars(scene) if qscalar is None else np.ascontiguousarray(qscalar, dtype=np.float32)
    bgv = np.ascontiguousarray(bg, dtype=np.float32)
    n = cam.nx * cam.ny
    rgba = np.zeros((n, 4), dtype=np.float32)
    depth = np.zeros(n, dtype=np.float32)
    _direct_fns().rtpo_render_direct(ctypes.byref(scene), ctypes.byref(cam), _fp(qs), _fp(cmap), cmap.shape[0],
                                     _fp(bgv), int(composite), aov, _fp(rgba), _fp(depth))
    return rgba, depth
