"""MI355X-native Monte Carlo path tracer: the per-pixel sampling loop of
m-kim/raytracingtherestofyourlife (MapperPathTracer::RenderCellsImpl) as HIP
kernels for gfx950 behind a C ABI (include/rtp.h, librtp.so)."""
from ._lib import LIB_PATH, RtpError, load  # noqa: F401
from .mapper import (  # noqa: F401
    Camera, CanvasRayTracer, CellSet, CornellBox, DataSet, Device, ErrorBadValue, MapperPathTracer,
    Field, default_camera, normalize, runPath, save_pnm,
)
from .direct import (  # noqa: F401
    Actor, Color, ColorTable, MapperQuad, MapperQuadAlbedo, MapperQuadNormals, Scene, View3D, runAlbedo,
    runDirect, runNorms, runRay, save_depth_pnm,
)

__all__ = [
    "Camera", "CanvasRayTracer", "CellSet", "CornellBox", "DataSet", "Device", "ErrorBadValue",
    "MapperPathTracer", "RtpError", "default_camera", "load", "normalize", "runPath", "save_pnm", "LIB_PATH",
    "Field", "Actor", "Color", "ColorTable", "MapperQuad", "MapperQuadAlbedo", "MapperQuadNormals", "Scene",
    "View3D", "runAlbedo", "runDirect", "runNorms", "runRay", "save_depth_pnm",
]
