"""ctypes binding of librtp.so (include/rtp.h).

There is no CPU fallback: if the HIP library is missing or fails to load,
every entry point raises.  The product path is the HIP path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTP_LIB_PATH") or os.path.join(_HERE, "librtp.so")  # override: experiments only

RTP_OK = 0
RTP_ERR_INVALID_ARGUMENT = -1
RTP_ERR_NO_SCENE = -2
RTP_ERR_DEVICE = -3
RTP_ERR_OUT_OF_MEMORY = -4

f32p = ctypes.POINTER(ctypes.c_float)
i32p = ctypes.POINTER(ctypes.c_int32)
u32p = ctypes.POINTER(ctypes.c_uint32)
i64p = ctypes.POINTER(ctypes.c_int64)


class RtpCamera(ctypes.Structure):
    _fields_ = [("position", ctypes.c_float * 3), ("look_at", ctypes.c_float * 3),
                ("view_up", ctypes.c_float * 3), ("fov_y_deg", ctypes.c_float)]


class RtpSceneDesc(ctypes.Structure):
    _fields_ = [
        ("points", f32p), ("n_points", ctypes.c_int32),
        ("quad_points", i32p), ("quad_mat", i32p), ("quad_tex", i32p), ("n_quads", ctypes.c_int32),
        ("sphere_point", i32p), ("sphere_radius", f32p), ("sphere_mat", i32p), ("sphere_tex", i32p),
        ("n_spheres", ctypes.c_int32),
        ("mat_type", i32p), ("n_mat", ctypes.c_int32),
        ("tex_type", i32p), ("n_tex_type", ctypes.c_int32),
        ("tex_rgb", f32p), ("n_tex", ctypes.c_int32),
        ("light_quad_points", ctypes.c_int32 * 4), ("light_sphere_point", ctypes.c_int32),
        ("ior", ctypes.c_float),
    ]


class RtpStats(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_uint64), ("live_bounces", ctypes.c_uint64),
                ("nan_pixels", ctypes.c_uint64), ("kernel_ms", ctypes.c_double)]


class RtpPixelAux(ctypes.Structure):
    _fields_ = [("final_seed", u32p), ("live_bounces", u32p)]


class RtpDirectDesc(ctypes.Structure):
    _fields_ = [("clip_near", ctypes.c_float), ("clip_far", ctypes.c_float), ("background", ctypes.c_float * 4),
                ("composite_background", ctypes.c_int32), ("quad_scalar", f32p), ("color_map", f32p),
                ("color_map_size", ctypes.c_int32)]


RTP_AOV_COLOR, RTP_AOV_NORMALS, RTP_AOV_ALBEDO = 1, 2, 4
RTP_FF_TABLES_AUTO, RTP_FF_TABLES_OFF, RTP_FF_TABLES_ON = 0, 1, 2


class RtpFfInfo(ctypes.Structure):
    _fields_ = [("policy", ctypes.c_int32), ("built", ctypes.c_int32), ("chain_tables", ctypes.c_int32),
                ("direct_first", ctypes.c_int32), ("direct_count", ctypes.c_int32), ("bytes", ctypes.c_uint64),
                ("alloc_ms", ctypes.c_double), ("build_ms", ctypes.c_double), ("samples_seen", ctypes.c_uint64),
                ("auto_samples", ctypes.c_uint64), ("auto_samples_direct", ctypes.c_uint64)]


EXPORTED_SYMBOLS = [
    "rtp_last_error", "rtp_abi_version", "rtp_create", "rtp_destroy", "rtp_set_scene", "rtp_render",
    "rtp_render_device", "rtp_render_tiles_device", "rtp_render_pixels", "rtp_normalize", "rtp_write_pnm", "rtp_cornell_box",
    "rtp_eval_primitive", "rtp_debug_counters", "rtp_verify_fast_math", "rtp_debug_closest_hit",
    "rtp_render_direct", "rtp_render_direct_device", "rtp_sample_color_table", "rtp_quad_scalars",
    "rtp_cornell_point_field", "rtp_write_pnm_depth", "rtp_eval_powf", "rtp_set_ff_tables", "rtp_get_ff_tables",
    "rtp_render_planned_device", "rtp_sphere_walk", "rtp_sphere_walk_oct_mask",
]


class RtpError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"rtp error {status}: {msg}")
        self.status = status


_lib = None


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load librtp.so (building it with hipcc first if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if not build_if_missing:
            raise RuntimeError(f"{LIB_PATH} is missing; run raytracingtherestofyourlife_amd/build.py")
        from . import build as _build
        _build.build()
    # One HIP runtime per process: torch bundles a libamdhip64 with the same
    # soname (libamdhip64.so.7) as /opt/rocm's.  Loading torch's first makes
    # librtp.so bind to it (soname match), so torch streams/allocations and
    # our launches share one runtime.  Without torch, /opt/rocm's is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    L.rtp_last_error.restype = ctypes.c_char_p
    L.rtp_abi_version.restype = ctypes.c_int32
    vp = ctypes.c_void_p
    L.rtp_create.argtypes = [ctypes.c_int32, ctypes.POINTER(vp)]
    L.rtp_destroy.argtypes = [vp]
    L.rtp_destroy.restype = None
    L.rtp_set_scene.argtypes = [vp, ctypes.POINTER(RtpSceneDesc)]
    L.rtp_render.argtypes = [vp, ctypes.POINTER(RtpCamera), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                             ctypes.c_int32, ctypes.c_uint32, f32p, ctypes.POINTER(RtpStats)]
    L.rtp_render_device.argtypes = [vp, ctypes.POINTER(RtpCamera), ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64,
                                    ctypes.c_int64, vp, vp, ctypes.POINTER(RtpPixelAux), vp,
                                    ctypes.POINTER(RtpStats)]
    L.rtp_render_tiles_device.argtypes = [vp, ctypes.POINTER(RtpCamera), ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int32,
                                          ctypes.c_int32, vp, vp, ctypes.POINTER(RtpStats)]
    L.rtp_render_pixels.argtypes = [vp, ctypes.POINTER(RtpCamera), ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, i64p, ctypes.c_int64, f32p,
                                    ctypes.POINTER(RtpPixelAux), ctypes.POINTER(RtpStats)]
    L.rtp_normalize.argtypes = [f32p, ctypes.c_int64, ctypes.c_int32]
    L.rtp_write_pnm.argtypes = [ctypes.c_char_p, f32p, ctypes.c_int32, ctypes.c_int32]
    L.rtp_cornell_box.argtypes = [ctypes.c_int32, ctypes.POINTER(RtpSceneDesc)]
    L.rtp_eval_primitive.argtypes = [vp, ctypes.c_int32, vp, vp, ctypes.c_int64]
    L.rtp_debug_closest_hit.argtypes = [vp, vp, ctypes.c_int64, vp]
    L.rtp_debug_counters.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
    L.rtp_verify_fast_math.argtypes = [vp, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]
    d64p = ctypes.POINTER(ctypes.c_double)
    L.rtp_render_direct.argtypes = [vp, ctypes.POINTER(RtpCamera), ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(RtpDirectDesc), f32p, f32p, f32p, f32p, ctypes.POINTER(RtpStats)]
    L.rtp_render_direct_device.argtypes = [vp, ctypes.POINTER(RtpCamera), ctypes.c_int32, ctypes.c_int32,
                                           ctypes.POINTER(RtpDirectDesc), vp, vp, vp, vp, vp,
                                           ctypes.POINTER(RtpStats)]
    L.rtp_sample_color_table.argtypes = [d64p, ctypes.c_int32, d64p, ctypes.c_int32, d64p, ctypes.c_int32, f32p]
    L.rtp_quad_scalars.argtypes = [f32p, ctypes.c_int32, i32p, ctypes.c_int32, f32p]
    L.rtp_cornell_point_field.argtypes = [ctypes.c_int32, ctypes.POINTER(f32p), ctypes.POINTER(ctypes.c_int32),
                                          ctypes.POINTER(i32p), ctypes.POINTER(ctypes.c_int32)]
    L.rtp_write_pnm_depth.argtypes = [ctypes.c_char_p, f32p, ctypes.c_int32, ctypes.c_int32]
    L.rtp_eval_powf.argtypes = [vp, f32p, ctypes.c_float, f32p, ctypes.c_int64]
    L.rtp_render_planned_device.argtypes = [vp, ctypes.POINTER(RtpCamera), ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64,
                                            ctypes.c_int64, vp, vp, ctypes.c_int32, vp, ctypes.POINTER(RtpPixelAux),
                                            vp, ctypes.POINTER(RtpStats)]
    L.rtp_set_ff_tables.argtypes = [vp, ctypes.c_int32]
    L.rtp_get_ff_tables.argtypes = [vp, ctypes.POINTER(RtpFfInfo)]
    L.rtp_sphere_walk.argtypes = [vp]
    L.rtp_sphere_walk_oct_mask.argtypes = [vp]
    for name in EXPORTED_SYMBOLS:
        if name not in ("rtp_last_error", "rtp_abi_version", "rtp_destroy"):
            getattr(L, name).restype = ctypes.c_int32
    _lib = L
    return L


def check(status: int) -> None:
    if status != RTP_OK:
        raise RtpError(status, load().rtp_last_error().decode(errors="replace"))
