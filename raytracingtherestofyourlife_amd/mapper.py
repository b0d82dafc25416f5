"""Host-side mirror of the reference's MapperPathTracer API over librtp.so.

Names, argument meaning and error behaviour follow the reference so that
code written against ``vtkm::rendering::MapperPathTracer`` (and the parts of
main.cc that drive it) reads the same:

    cb = CornellBox(); cb.buildDataSet()
    canvas = CanvasRayTracer(nx, ny)
    cam = Camera(); cam.SetPosition(...); cam.SetLookAt(...); ...
    mapper = MapperPathTracer(spp, depth, cb.matIdx, cb.texIdx, cb.matType, cb.texType, cb.tex)
    mapper.SetCanvas(canvas)
    mapper.RenderCells(cb.ds.GetCellSet(), cb.coord, field, ct, cam, sr)
    normalize(canvas.GetColorBuffer(), spp)            # NormalizeFunctor
    save_pnm("output.pnm", canvas.GetColorBuffer(), nx, ny)

Reference: MapperPathTracer.h:44-159, MapperPathTracer.cxx:94-406,
main.cc:253-384, CornellBox.cpp:141-418.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import RtpCamera, RtpFfInfo, RtpPixelAux, RtpSceneDesc, RtpStats, check


class ErrorBadValue(ValueError):
    """vtkm::cont::ErrorBadValue."""


# ------------------------------------------------------------- camera --
class Camera:
    """The vtkm::rendering::Camera fields MapperPathTracer reads
    (pathtracing/Camera.cxx:624-637)."""

    def __init__(self):
        self.position = np.array([0.0, 0.0, 1.0], dtype=np.float32)
        self.look_at = np.zeros(3, dtype=np.float32)
        self.view_up = np.array([0.0, 1.0, 0.0], dtype=np.float32)
        self.fov = np.float32(60.0)
        self.zoom = np.float32(1.0)
        self.clipping = (0.01, 1000.0)

    def SetPosition(self, p):
        self.position = np.asarray(p, dtype=np.float32).reshape(3).copy()

    def SetLookAt(self, p):
        self.look_at = np.asarray(p, dtype=np.float32).reshape(3).copy()

    def SetViewUp(self, p):
        self.view_up = np.asarray(p, dtype=np.float32).reshape(3).copy()

    def SetFieldOfView(self, deg):
        self.fov = np.float32(deg)

    def SetZoom(self, z):  # RayGen is built with _zoom = 0: zoom never reaches the path
        self.zoom = np.float32(z)

    def SetClippingRange(self, near, far):  # unused by the path tracer
        self.clipping = (near, far)

    def GetPosition(self):
        return self.position.copy()

    def GetLookAt(self):
        return self.look_at.copy()

    def GetViewUp(self):
        return self.view_up.copy()

    def GetFieldOfView(self):
        return float(self.fov)

    def to_c(self) -> RtpCamera:
        c = RtpCamera()
        c.position[:] = [float(v) for v in self.position]
        c.look_at[:] = [float(v) for v in self.look_at]
        c.view_up[:] = [float(v) for v in self.view_up]
        c.fov_y_deg = float(self.fov)
        return c


def default_camera() -> Camera:
    """The camera of main.cc:616-622."""
    cam = Camera()
    cam.SetClippingRange(0.1, 5.0)
    cam.SetPosition([278 / 555.0, 278 / 555.0, -800 / 555.0])
    cam.SetFieldOfView(40.0)
    cam.SetViewUp([0, 1, 0])
    cam.SetLookAt([278 / 555.0, 278 / 555.0, 278 / 555.0])
    return cam


# ------------------------------------------------------------- canvas --
class Canvas:
    def __init__(self, nx: int, ny: int):
        self.width, self.height = int(nx), int(ny)

    def GetWidth(self):
        return self.width

    def GetHeight(self):
        return self.height


class CanvasRayTracer(Canvas):
    """Colour buffer = Vec4f per pixel, index j*nx + i (row 0 = camera bottom)."""

    def __init__(self, nx: int, ny: int):
        super().__init__(nx, ny)
        self.color = np.zeros((self.width * self.height, 4), dtype=np.float32)
        self.depth = np.full(self.width * self.height, np.float32(1.001), dtype=np.float32)

    def GetColorBuffer(self) -> np.ndarray:
        return self.color

    def GetDepthBuffer(self) -> np.ndarray:
        """Canvas depth (written by the -direct mappers; 1.001 = cleared)."""
        return self.depth


# -------------------------------------------------------------- scene --
@dataclass
class CellSet:
    """The parts of the explicit cell set the path tracer consumes: quad
    cells (QuadExtractor rows p0..p3) and vertex cells (sphere centres)."""

    quad_points: np.ndarray  # int32 [Q,4]
    sphere_points: np.ndarray  # int32 [S]
    quad_cells: np.ndarray | None = None  # int32 [Q]: QuadIds[0], the cell id of each quad


@dataclass
class Field:
    """vtkm::cont::Field (point association): a name and one value per entry."""

    name: str
    values: np.ndarray  # float32

    def GetName(self) -> str:
        return self.name

    def GetRange(self) -> tuple[float, float]:
        return float(self.values.min()), float(self.values.max())


@dataclass
class DataSet:
    cellset: CellSet
    coords: np.ndarray  # float32 [P,3]
    fields: dict = field(default_factory=dict)

    def GetCellSet(self) -> CellSet:
        return self.cellset

    def GetField(self, name: str) -> Field:
        if name not in self.fields:
            raise ErrorBadValue(f"No field with requested name: {name}")
        return self.fields[name]

    def AddField(self, f: Field) -> None:
        self.fields[f.name] = f


@dataclass
class CornellBox:
    """CornellBox (CornellBox.h:9-55); buildDataSet delegates to librtp's
    rtp_cornell_box (the same float/double arithmetic as CornellBox.cpp)."""

    variant: int = 0
    tex: np.ndarray | None = None
    matIdx: list = field(default_factory=list)
    texIdx: list = field(default_factory=list)
    matType: np.ndarray | None = None
    texType: np.ndarray | None = None
    coord: np.ndarray | None = None
    SphereRadii: np.ndarray | None = None
    ds: DataSet | None = None
    light_quad_points: tuple = (8, 9, 10, 11)
    light_sphere_point: int = 48
    ior: float = 1.5

    def buildDataSet(self) -> DataSet:
        L = _lib.load()
        d = RtpSceneDesc()
        check(L.rtp_cornell_box(self.variant, ctypes.byref(d)))
        npz = lambda ptr, n, dt: np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt).copy()
        self.coord = npz(d.points, 3 * d.n_points, np.float32).reshape(-1, 3)
        quads = npz(d.quad_points, 4 * d.n_quads, np.int32).reshape(-1, 4)
        spheres = npz(d.sphere_point, d.n_spheres, np.int32)
        self.SphereRadii = npz(d.sphere_radius, d.n_spheres, np.float32)
        self.matIdx = [npz(d.quad_mat, d.n_quads, np.int32), npz(d.sphere_mat, d.n_spheres, np.int32)]
        self.texIdx = [npz(d.quad_tex, d.n_quads, np.int32), npz(d.sphere_tex, d.n_spheres, np.int32)]
        self.matType = npz(d.mat_type, d.n_mat, np.int32)
        self.texType = npz(d.tex_type, d.n_tex_type, np.int32)
        self.tex = npz(d.tex_rgb, 3 * d.n_tex, np.float32).reshape(-1, 3)
        self.light_quad_points = tuple(int(v) for v in d.light_quad_points)
        self.light_sphere_point = int(d.light_sphere_point)
        self.ior = float(d.ior)
        fp, nf, qc, nq = _lib.f32p(), ctypes.c_int32(), _lib.i32p(), ctypes.c_int32()
        check(L.rtp_cornell_point_field(self.variant, ctypes.byref(fp), ctypes.byref(nf), ctypes.byref(qc),
                                        ctypes.byref(nq)))
        cells = npz(qc, nq.value, np.int32)
        self.ds = DataSet(CellSet(quads, spheres, cells), self.coord)
        self.ds.AddField(Field("point_var", npz(fp, nf.value, np.float32)))  # CornellBox.cpp:411-416
        return self.ds


# ------------------------------------------------------------- device --
class Device:
    """One rtp_context (one HIP device)."""

    def __init__(self, device: int = 0):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        check(self._L.rtp_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = device
        self._scene_key = None

    def close(self):
        if self.handle:
            self._L.rtp_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, coords, quad_points, quad_mat, quad_tex, sphere_points, sphere_radius, sphere_mat,
                  sphere_tex, mat_type, tex_type, tex, light_quad_points=(8, 9, 10, 11), light_sphere_point=48,
                  ior=1.5):
        arrs = dict(
            points=np.ascontiguousarray(coords, dtype=np.float32).reshape(-1),
            quad_points=np.ascontiguousarray(quad_points, dtype=np.int32).reshape(-1),
            quad_mat=np.ascontiguousarray(quad_mat, dtype=np.int32),
            quad_tex=np.ascontiguousarray(quad_tex, dtype=np.int32),
            sphere_point=np.ascontiguousarray(sphere_points, dtype=np.int32),
            sphere_radius=np.ascontiguousarray(sphere_radius, dtype=np.float32),
            sphere_mat=np.ascontiguousarray(sphere_mat, dtype=np.int32),
            sphere_tex=np.ascontiguousarray(sphere_tex, dtype=np.int32),
            mat_type=np.ascontiguousarray(mat_type, dtype=np.int32),
            tex_type=np.ascontiguousarray(tex_type, dtype=np.int32),
            tex_rgb=np.ascontiguousarray(tex, dtype=np.float32).reshape(-1),
        )
        d = RtpSceneDesc()
        fp = lambda a: a.ctypes.data_as(_lib.f32p)
        ip = lambda a: a.ctypes.data_as(_lib.i32p)
        d.points, d.n_points = fp(arrs["points"]), arrs["points"].size // 3
        d.quad_points, d.quad_mat, d.quad_tex = ip(arrs["quad_points"]), ip(arrs["quad_mat"]), ip(arrs["quad_tex"])
        d.n_quads = arrs["quad_mat"].size
        d.sphere_point, d.sphere_radius = ip(arrs["sphere_point"]), fp(arrs["sphere_radius"])
        d.sphere_mat, d.sphere_tex = ip(arrs["sphere_mat"]), ip(arrs["sphere_tex"])
        d.n_spheres = arrs["sphere_point"].size
        d.mat_type, d.n_mat = ip(arrs["mat_type"]), arrs["mat_type"].size
        d.tex_type, d.n_tex_type = ip(arrs["tex_type"]), arrs["tex_type"].size
        d.tex_rgb, d.n_tex = fp(arrs["tex_rgb"]), arrs["tex_rgb"].size // 3
        d.light_quad_points[:] = [int(v) for v in light_quad_points]
        d.light_sphere_point = int(light_sphere_point)
        d.ior = float(ior)
        check(self._L.rtp_set_scene(self.handle, ctypes.byref(d)))

    def set_cornell_box(self, variant: int = 0):
        d = RtpSceneDesc()
        check(self._L.rtp_cornell_box(variant, ctypes.byref(d)))
        check(self._L.rtp_set_scene(self.handle, ctypes.byref(d)))

    def render(self, camera: Camera, nx: int, ny: int, spp: int, depth: int, seed_base: int = 0):
        """Full canvas into host memory: (rgba_sum[nx*ny,4], stats)."""
        out = np.zeros((nx * ny, 4), dtype=np.float32)
        st = RtpStats()
        cam = camera.to_c()
        check(self._L.rtp_render(self.handle, ctypes.byref(cam), nx, ny, spp, depth, seed_base,
                                 out.ctypes.data_as(_lib.f32p), ctypes.byref(st)))
        return out, st

    def render_pixels(self, camera: Camera, nx: int, ny: int, spp: int, depth: int, pixels, seed_base: int = 0):
        """Arbitrary pixel subset: (rgba_sum[n,4], final_seed[n], live[n], stats)."""
        ids = np.ascontiguousarray(pixels, dtype=np.int64)
        n = ids.size
        out = np.zeros((n, 4), dtype=np.float32)
        seeds = np.zeros(n, dtype=np.uint32)
        live = np.zeros(n, dtype=np.uint32)
        aux = RtpPixelAux(seeds.ctypes.data_as(_lib.u32p), live.ctypes.data_as(_lib.u32p))
        st = RtpStats()
        cam = camera.to_c()
        check(self._L.rtp_render_pixels(self.handle, ctypes.byref(cam), nx, ny, spp, depth, seed_base,
                                        ids.ctypes.data_as(_lib.i64p), n, out.ctypes.data_as(_lib.f32p),
                                        ctypes.byref(aux), ctypes.byref(st)))
        return out, seeds, live, st

    def render_device(self, camera: Camera, nx: int, ny: int, spp: int, depth: int, out_ptr: int,
                      pixel_begin: int = 0, pixel_count: int | None = None, pixel_ids_ptr: int = 0,
                      seed_base: int = 0, stream: int = 0, seed_ptr: int = 0, live_ptr: int = 0,
                      timed: bool = False):
        """Device-resident render (out_ptr: device float4[pixel_count])."""
        if pixel_count is None:
            pixel_count = nx * ny - pixel_begin
        aux = RtpPixelAux(ctypes.cast(seed_ptr, _lib.u32p) if seed_ptr else None,
                          ctypes.cast(live_ptr, _lib.u32p) if live_ptr else None)
        st = RtpStats()
        cam = camera.to_c()
        check(self._L.rtp_render_device(self.handle, ctypes.byref(cam), nx, ny, spp, depth, seed_base,
                                        pixel_begin, pixel_count, ctypes.c_void_p(pixel_ids_ptr or None),
                                        ctypes.c_void_p(out_ptr), ctypes.byref(aux), ctypes.c_void_p(stream or None),
                                        ctypes.byref(st) if timed else None))
        return st

    def render_planned_device(self, camera: Camera, nx: int, ny: int, spp: int, depth: int, out_ptr: int,
                              pixel_count: int, wave_begin_ptr: int, n_waves: int, pixel_ids_ptr: int = 0,
                              pixel_begin: int = 0, seed_base: int = 0, stream: int = 0, seed_ptr: int = 0,
                              live_ptr: int = 0, timed: bool = False):
        """rtp_render_planned_device: wave w owns entries [wave_begin[w], wave_begin[w+1])."""
        aux = RtpPixelAux(ctypes.cast(seed_ptr, _lib.u32p) if seed_ptr else None,
                          ctypes.cast(live_ptr, _lib.u32p) if live_ptr else None)
        st = RtpStats()
        cam = camera.to_c()
        check(self._L.rtp_render_planned_device(self.handle, ctypes.byref(cam), nx, ny, spp, depth, seed_base,
                                                pixel_begin, pixel_count, ctypes.c_void_p(pixel_ids_ptr or None),
                                                ctypes.c_void_p(wave_begin_ptr), n_waves, ctypes.c_void_p(out_ptr),
                                                ctypes.byref(aux), ctypes.c_void_p(stream or None),
                                                ctypes.byref(st) if timed else None))
        return st

    def render_tiles_device(self, camera: Camera, nx: int, ny: int, spp: int, depth: int, out_ptr: int,
                            rank: int, world: int, seed_base: int = 0, stream: int = 0, timed: bool = False):
        """Device-resident render of rank's tiles of the round-robin 16x16
        tile deal (out_ptr: device float4[256 * tiles owned], each tile whole;
        on a canvas that is not whole tiles, shard.tile_entries gives the
        entries inside the canvas and their pixels)."""
        st = RtpStats()
        cam = camera.to_c()
        check(self._L.rtp_render_tiles_device(self.handle, ctypes.byref(cam), nx, ny, spp, depth, seed_base, rank,
                                              world, ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream or None),
                                              ctypes.byref(st) if timed else None))
        return st

    FF_POLICIES = {"auto": _lib.RTP_FF_TABLES_AUTO, "off": _lib.RTP_FF_TABLES_OFF, "on": _lib.RTP_FF_TABLES_ON}

    def sphere_walk(self) -> str:
        """How renders search the current scene's spheres (include/rtp.h
        rtp_sphere_walk): 'scan', 'global' (threaded BVH in global memory) or
        'lds' (the LDS-resident walk)."""
        return ("scan", "global", "lds")[self._L.rtp_sphere_walk(self.handle)]

    def sphere_walk_oct_mask(self) -> int:
        """The global sphere walk's octant mask (rtp_sphere_walk_oct_mask): 7
        = every direction octant walks its own near-to-far copy; -1 without a
        sphere BVH."""
        return int(self._L.rtp_sphere_walk_oct_mask(self.handle))

    def set_ff_tables(self, policy: str) -> dict:
        """RNG jump-table policy of this context (include/rtp.h rtp_set_ff_tables):
        'auto' (default), 'off', or 'on' (build now: a long-lived renderer).
        Returns ff_info()."""
        check(self._L.rtp_set_ff_tables(self.handle, self.FF_POLICIES[policy]))
        return self.ff_info()

    def ff_info(self) -> dict:
        """The device's jump tables: policy, what is built, bytes, setup cost."""
        i = RtpFfInfo()
        check(self._L.rtp_get_ff_tables(self.handle, ctypes.byref(i)))
        d = {k: getattr(i, k) for k, _ in RtpFfInfo._fields_}
        d["policy"] = {v: k for k, v in self.FF_POLICIES.items()}.get(d["policy"], d["policy"])
        return d

    DEBUG_COUNTERS = ("bounce_steps", "bounce_lanes", "ff_phases", "ff_lanes", "ff_iters", "cycles_bounce",
                      "cycles_ff", "cycles_total", "cycles_intersect", "cycles_bounce_call", "cycles_end",
                      "cycles_refill", "real_start", "real_end", "hw_id", "tail_steps", "tail_lanes",
                      "tail_cycles", "fallback_steps", "fallback_lanes", "refill_visits", "refill_lanes",
                      "hit_visits", "hit_lanes", "gen_visits", "gen_lanes", "cycles_gen", "cycles_pdf", "end_visits",
                      "end_lanes", "ffrad_visits", "ffrad_lanes", "ffrad_rows", "dead_lanes", "diel_visits", "diel_lanes",
                      "cycles_diel", "light_visits", "light_lanes", "box_free_steps", "box_lanes",
                      "max_wave_cycles")

    def debug_counters(self) -> dict:
        """Pool-kernel counters of the last launch made with RTP_DEBUG_STATS=1."""
        n = len(self.DEBUG_COUNTERS)
        out = (ctypes.c_uint64 * n)()
        waves = self._L.rtp_debug_counters(self.handle, out, n)
        d = {k: int(v) for k, v in zip(self.DEBUG_COUNTERS, out)}
        d["waves"] = int(waves)
        return d

    def verify_fast_math(self, kind: int, lo: float, hi: float) -> tuple[int, int]:
        """Exhaustive device check over every float in [lo, hi] (same sign)."""
        lb = int(np.float32(lo).view(np.uint32))
        hb = int(np.float32(hi).view(np.uint32))
        lb, hb = min(lb, hb), max(lb, hb)
        bad = ctypes.c_uint64(0)
        first = ctypes.c_uint32(0)
        check(self._L.rtp_verify_fast_math(self.handle, kind, lb, hb, ctypes.byref(bad), ctypes.byref(first)))
        return int(bad.value), int(first.value)

    def debug_wave_records(self) -> np.ndarray:
        """Raw per-wave counter records [waves, kDbgCounters] of the last stats launch."""
        n = len(self.DEBUG_COUNTERS) - 1
        waves = self.debug_counters()["waves"]
        buf = np.zeros((max(waves, 1), n), dtype=np.uint64)
        self._L.rtp_debug_counters(self.handle, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), -1)
        return buf[:waves]

    def eval_primitive(self, kind: int, values: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(values)
        assert a.dtype.itemsize == 4
        out = np.zeros_like(a)
        check(self._L.rtp_eval_primitive(self.handle, kind, a.ctypes.data_as(ctypes.c_void_p),
                                         out.ctypes.data_as(ctypes.c_void_p), a.size))
        return out

    def debug_closest_hit(self, rays: np.ndarray) -> np.ndarray:
        """(n, 6) float32 rays (o, d) -> (n, 7) uint32: prefiltered (t bits,
        kind, index), exact scan (t bits, kind, index), fell-back flag."""
        a = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        out = np.zeros((a.shape[0], 7), dtype=np.uint32)
        check(self._L.rtp_debug_closest_hit(self.handle, a.ctypes.data_as(ctypes.c_void_p), a.shape[0],
                                            out.ctypes.data_as(ctypes.c_void_p)))
        return out


# ------------------------------------------------------------- mapper --
class MapperPathTracer:
    """vtkm::rendering::MapperPathTracer (MapperPathTracer.h:44-159)."""

    def __init__(self, sc: int, dc: int, matIdx, texIdx, matType, texType, tex, device: int | Device = 0):
        self.samplecount = int(sc)
        self.depthcount = int(dc)
        self.MatIdx, self.TexIdx = matIdx, texIdx
        self.MatType, self.TexType, self.Tex = matType, texType, tex
        self._dev = device if isinstance(device, Device) else Device(device)
        self._canvas = None
        self.CompositeBackground = True
        self.last_stats = None

    def SetCanvas(self, canvas):  # MapperPathTracer.cxx:155-172
        if canvas is not None and not isinstance(canvas, CanvasRayTracer):
            raise ErrorBadValue("Ray Tracer: bad canvas type. Must be CanvasRayTracer")
        self._canvas = canvas

    def GetCanvas(self):
        return self._canvas

    def SetCompositeBackground(self, on: bool):
        self.CompositeBackground = bool(on)

    def StartScene(self):
        pass

    def EndScene(self):
        pass

    def NewCopy(self) -> "MapperPathTracer":  # shallow copy sharing Internals (:403-406)
        m = MapperPathTracer.__new__(MapperPathTracer)
        m.__dict__.update(self.__dict__)
        return m

    def RenderCells(self, cellset: CellSet, coords, scalarField=None, colorTable=None, camera: Camera = None,
                    scalarRange=None, light_quad_points=(8, 9, 10, 11), light_sphere_point=48, ior=1.5):
        """MapperPathTracer.cxx:356-383: the canvas colour buffer receives the
        un-normalised per-pixel sum over samplecount samples."""
        if self._canvas is None:
            raise ErrorBadValue("MapperPathTracer: SetCanvas was not called")
        if camera is None:
            raise ErrorBadValue("MapperPathTracer: no camera")
        radii = getattr(cellset, "sphere_radius", None)
        if radii is None:
            radii = np.full(len(cellset.sphere_points), np.float32(90 / 555.0), dtype=np.float32)  # extract(), :182
        self._dev.set_scene(coords, cellset.quad_points, self.MatIdx[0], self.TexIdx[0], cellset.sphere_points,
                            radii, self.MatIdx[1], self.TexIdx[1], self.MatType, self.TexType, self.Tex,
                            light_quad_points, light_sphere_point, ior)
        nx, ny = self._canvas.GetWidth(), self._canvas.GetHeight()
        out, st = self._dev.render(camera, nx, ny, self.samplecount, self.depthcount)
        self._canvas.color[...] = out
        self.last_stats = st


# -------------------------------------------------------- application --
def normalize(colors: np.ndarray, samplecount: int) -> np.ndarray:
    """NormalizeFunctor (main.cc:253-287), in place; returns colors."""
    a = colors
    if not (a.flags.c_contiguous and a.dtype == np.float32):
        raise ValueError("normalize: expects a C-contiguous float32 [N,4] buffer")
    check(_lib.load().rtp_normalize(a.ctypes.data_as(_lib.f32p), a.shape[0], int(samplecount)))
    return a


def save_pnm(path: str, colors: np.ndarray, nx: int, ny: int) -> None:
    """save() (main.cc:325-384): P3, buffer order, int(255.99*c)."""
    a = np.ascontiguousarray(colors, dtype=np.float32)
    check(_lib.load().rtp_write_pnm(path.encode(), a.ctypes.data_as(_lib.f32p), nx, ny))


def runPath(nx: int, ny: int, samplecount: int, depthcount: int, canvas: CanvasRayTracer, cam: Camera,
            cb: CornellBox, device: int | Device = 0) -> MapperPathTracer:
    """main.cc:289-323."""
    mapper = MapperPathTracer(samplecount, depthcount, cb.matIdx, cb.texIdx, cb.matType, cb.texType, cb.tex,
                              device=device)
    mapper.SetCanvas(canvas)
    cellset = cb.ds.GetCellSet()
    cellset.sphere_radius = cb.SphereRadii
    mapper.RenderCells(cellset, cb.coord, None, None, cam, None, cb.light_quad_points, cb.light_sphere_point,
                       cb.ior)
    normalize(canvas.GetColorBuffer(), samplecount)
    return mapper
