"""The -direct mode of main.cc (runRay / runNorms / runAlbedo, main.cc:120-251,
623-651; generate(), :386-431) over librtp.so.

Mirrors the reference's quad mappers and the VTK-m rendering objects main.cc
builds around them:

    scene = Scene(); scene.AddActor(Actor(cellset, coords, field, colorTable))
    view = View3D(scene, MapperQuad(), canvas, cam, background, foreground)
    view.Initialize(); view.Paint()          # canvas colour + depth buffers
    save_pnm("direct.pnm", canvas.GetColorBuffer(), nx, ny)
    save_depth_pnm("depth.pnm", canvas.GetDepthBuffer(), nx, ny)

MapperQuad / MapperQuadNormals / MapperQuadAlbedo (MapperQuad*.cxx:86-150)
each paint one AOV like the reference.  runDirect() is the MI355X path of
the whole -direct block: one launch intersects each camera ray once and
writes colour, normals, albedo and depth, each bit-identical to its own
mapper render.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import RtpDirectDesc, RtpStats, check
from .mapper import Camera, CanvasRayTracer, CellSet, CornellBox, Device, ErrorBadValue, Field


# ----------------------------------------------------------- colour table --
class ColorTable:
    """vtkm::cont::ColorTable(name, colorSpace, nanColor, rgbPoints, alphaPoints):
    rgbPoints are (x, r, g, b) quadruples, alphaPoints (x, alpha, midpoint,
    sharpness) quadruples (VTK-m's FillColorTableFromDataPointer)."""

    def __init__(self, name: str = "", color_space: str = "RGB", nan_color=(0.5, 0.0, 0.0), rgb_points=(),
                 alpha_points=(0.0, 1.0, 0.5, 0.0, 1.0, 1.0, 0.5, 0.0)):
        if color_space != "RGB":
            raise ErrorBadValue("ColorTable: only the RGB colour space is implemented")
        self.name = name
        self.nan_color = np.asarray(nan_color, dtype=np.float64).reshape(3)
        self.rgb_points = np.asarray(rgb_points, dtype=np.float64).reshape(-1)
        self.alpha_points = np.asarray(alpha_points, dtype=np.float64).reshape(-1)

    def Sample(self, n: int = 1024) -> np.ndarray:
        """Mapper::SetActiveColorTable: Sample(n) as Vec4ui_8, * (1/255.f)."""
        out = np.zeros((n, 4), dtype=np.float32)
        d64 = ctypes.POINTER(ctypes.c_double)
        check(_lib.load().rtp_sample_color_table(
            self.rgb_points.ctypes.data_as(d64), self.rgb_points.size, self.alpha_points.ctypes.data_as(d64),
            self.alpha_points.size, self.nan_color.ctypes.data_as(d64), n, out.ctypes.data_as(_lib.f32p)))
        return out


def norm_color_range(color_vals):
    """main.cc:114-119."""
    return [v / 255.0 for v in color_vals]


def main_pallet_color_table() -> ColorTable:
    """The ct_12_quad of runRay / runAlbedo (main.cc:150-176, 229-239):
    green, red, the light's fill (white) and 21 whites, alpha 24 x 1.0."""
    c1, c2, c3 = [0.65, 0.05, 0.05], [0.73, 0.73, 0.73], [0.12, 0.45, 0.15]
    num_quads = 12 + 6 + 6
    pallet = c3 + c1 + c2 + c2 * (num_quads - 3)
    return ColorTable("pallet_color_table", "RGB", (0, 0, 0), pallet, [1.0] * num_quads)


# ---------------------------------------------------------- scene / view --
class Color:
    def __init__(self, r=0.0, g=0.0, b=0.0, a=1.0):
        self.components = (float(r), float(g), float(b), float(a))


class Actor:
    """vtkm::rendering::Actor: cells, coordinates, scalar field, colour table;
    the scalar range is the field's range (Actor::Init)."""

    def __init__(self, cells: CellSet, coords, scalar_field: Field, color_table: ColorTable):
        self.cells, self.coords, self.field, self.color_table = cells, coords, scalar_field, color_table
        self.scalar_range = scalar_field.GetRange()


class Scene:
    def __init__(self):
        self.actors: list[Actor] = []

    def AddActor(self, actor: Actor) -> None:
        self.actors.append(actor)

    def Render(self, mapper, canvas, camera) -> None:
        """Scene::Render: StartScene, each actor's Render, EndScene."""
        mapper.StartScene()
        for a in self.actors:
            mapper.SetCanvas(canvas)
            mapper.SetActiveColorTable(a.color_table)
            mapper.RenderCells(a.cells, a.coords, a.field, a.color_table, camera, a.scalar_range)
        mapper.EndScene()


class View3D:
    """pathtracing::View3D (View3D.cxx:40-64): Paint clears the canvas and
    renders the scene with the mapper; annotations are not drawn."""

    def __init__(self, scene: Scene, mapper, canvas: CanvasRayTracer, camera: Camera, background: Color,
                 foreground: Color | None = None):
        self.scene, self.mapper, self.canvas, self.camera = scene, mapper, canvas, camera
        self.background = background
        self.foreground = foreground
        mapper.background = background.components

    def Initialize(self) -> None:
        pass

    def Paint(self) -> None:
        self.canvas.color[...] = 0.0  # Canvas::Clear
        self.canvas.depth[...] = np.float32(1.001)
        self.scene.Render(self.mapper, self.canvas, self.camera)


# ---------------------------------------------------------------- device --
def quad_scalars(field_values: np.ndarray, quad_cells: np.ndarray) -> np.ndarray:
    """QuadIntersector GetScalar per quad over the field's range."""
    f = np.ascontiguousarray(field_values, dtype=np.float32)
    c = np.ascontiguousarray(quad_cells, dtype=np.int32)
    out = np.zeros(c.size, dtype=np.float32)
    check(_lib.load().rtp_quad_scalars(f.ctypes.data_as(_lib.f32p), f.size, c.ctypes.data_as(_lib.i32p), c.size,
                                       out.ctypes.data_as(_lib.f32p)))
    return out


def render_direct(dev: Device, camera: Camera, nx: int, ny: int, qscalar: np.ndarray, cmap: np.ndarray | None,
                  aovs: int = 7, depth: bool = True, background=(0.0, 0.0, 0.0, 1.0), composite: bool = True):
    """One rtp_render_direct launch into host buffers: dict of 'color',
    'normals', 'albedo' (float32 [n,4]) and 'depth' (float32 [n]) for the
    requested AOVs, plus 'stats'."""
    n = nx * ny
    outs = {}
    for name, bit in (("color", 1), ("normals", 2), ("albedo", 4)):
        if aovs & bit:
            outs[name] = np.zeros((n, 4), dtype=np.float32)
    if depth:
        outs["depth"] = np.zeros(n, dtype=np.float32)
    qs = np.ascontiguousarray(qscalar, dtype=np.float32)
    cm = None if cmap is None else np.ascontiguousarray(cmap, dtype=np.float32)
    d = RtpDirectDesc()
    d.clip_near, d.clip_far = float(camera.clipping[0]), float(camera.clipping[1])
    d.background[:] = [float(v) for v in background]
    d.composite_background = int(bool(composite))
    d.quad_scalar = qs.ctypes.data_as(_lib.f32p)
    d.color_map = cm.ctypes.data_as(_lib.f32p) if cm is not None else None
    d.color_map_size = 0 if cm is None else cm.shape[0]
    st = RtpStats()
    cam = camera.to_c()
    ptr = lambda k: outs[k].ctypes.data_as(_lib.f32p) if k in outs else None
    check(dev._L.rtp_render_direct(dev.handle, ctypes.byref(cam), nx, ny, ctypes.byref(d), ptr("color"),
                                   ptr("normals"), ptr("albedo"), ptr("depth"), ctypes.byref(st)))
    outs["stats"] = st
    return outs


# ---------------------------------------------------------------- mappers --
class _MapperQuadBase:
    AOV = 1

    def __init__(self, device: int | Device = 0):
        self._dev = device if isinstance(device, Device) else Device(device)
        self._canvas = None
        self.CompositeBackground = True
        self.ColorMap = None
        self.background = (0.0, 0.0, 0.0, 1.0)
        self.last_stats = None

    def SetCanvas(self, canvas):  # MapperQuad.cxx:65-79
        if canvas is not None and not isinstance(canvas, CanvasRayTracer):
            raise ErrorBadValue("Ray Tracer: bad canvas type. Must be CanvasRayTracer")
        self._canvas = canvas

    def GetCanvas(self):
        return self._canvas

    def SetActiveColorTable(self, ct: ColorTable):
        """vtkm::rendering::Mapper::SetActiveColorTable: 1024 samples."""
        self.ColorMap = ct.Sample(1024)

    def SetCompositeBackground(self, on: bool):
        self.CompositeBackground = bool(on)

    def StartScene(self):
        pass

    def EndScene(self):
        pass

    def NewCopy(self):
        m = self.__class__.__new__(self.__class__)
        m.__dict__.update(self.__dict__)
        return m

    def RenderCells(self, cellset: CellSet, coords, scalarField: Field, colorTable, camera: Camera,
                    scalarRange=None):
        """MapperQuad.cxx:86-150: the canvas receives the mapper's AOV and depth."""
        if self._canvas is None:
            raise ErrorBadValue("MapperQuad: SetCanvas was not called")
        if cellset.quad_cells is None:
            raise ErrorBadValue("MapperQuad: the cell set carries no quad cell ids (QuadIds[0])")
        q = cellset.quad_points.shape[0]
        ones = np.ones(q, dtype=np.int32)
        zeros_r = np.zeros(0, dtype=np.float32)
        # the quad mappers draw quads only (QuadExtractor): no spheres, materials unused
        self._dev.set_scene(coords, cellset.quad_points, ones * 0, ones * 0, np.zeros(1, np.int32),
                            np.full(1, np.float32(1.0)), np.zeros(1, np.int32), np.zeros(1, np.int32),
                            np.zeros(1, np.int32), np.zeros(1, np.int32), np.zeros((1, 3), np.float32),
                            light_quad_points=tuple(cellset.quad_points[0]) if q else (0, 0, 0, 0),
                            light_sphere_point=0)
        del zeros_r
        qs = quad_scalars(scalarField.values, cellset.quad_cells) if q else np.zeros(0, np.float32)
        nx, ny = self._canvas.GetWidth(), self._canvas.GetHeight()
        outs = render_direct(self._dev, camera, nx, ny, qs, self.ColorMap if self.AOV == 1 else None,
                             aovs=self.AOV, depth=True, background=self.background,
                             composite=self.CompositeBackground)
        key = {1: "color", 2: "normals", 4: "albedo"}[self.AOV]
        self._canvas.color[...] = outs[key]
        self._canvas.depth[...] = outs["depth"]
        self.last_stats = outs["stats"]


class MapperQuad(_MapperQuadBase):
    """path::rendering::MapperQuad: VTK-m RayTracer colour (Phong over the colour map)."""

    AOV = 1


class MapperQuadNormals(_MapperQuadBase):
    """path::rendering::MapperQuadNormals (RayTracerNormals.cxx)."""

    AOV = 2


class MapperQuadAlbedo(_MapperQuadBase):
    """path::rendering::MapperQuadAlbedo (RayTracerAlbedo.cxx)."""

    AOV = 4


# ------------------------------------------------------------ application --
def _paint(mapper, nx, ny, canvas, cam, cb: CornellBox, ct: ColorTable):
    scene = Scene()
    scene.AddActor(Actor(cb.ds.GetCellSet(), cb.coord, cb.ds.GetField("point_var"), ct))
    view = View3D(scene, mapper, canvas, cam, Color(0, 0, 0, 1.0), Color(1, 1, 1, 1.0))
    view.Initialize()
    view.Paint()
    return mapper


def runRay(nx, ny, samplecount, depthcount, canvas: CanvasRayTracer, cam: Camera, cb: CornellBox, device=0):
    """main.cc:120-188."""
    return _paint(MapperQuad(device), nx, ny, canvas, cam, cb, main_pallet_color_table())


def runNorms(nx, ny, samplecount, depthcount, canvas: CanvasRayTracer, cam: Camera, cb: CornellBox, device=0):
    """main.cc:190-208 (COOL_TO_WARM_EXTENDED table: unused by the normals shade)."""
    return _paint(MapperQuadNormals(device), nx, ny, canvas, cam, cb, main_pallet_color_table())


def runAlbedo(nx, ny, samplecount, depthcount, canvas: CanvasRayTracer, cam: Camera, cb: CornellBox, device=0):
    """main.cc:210-251."""
    return _paint(MapperQuadAlbedo(device), nx, ny, canvas, cam, cb, main_pallet_color_table())


def runDirect(nx: int, ny: int, cam: Camera, cb: CornellBox, device: int | Device = 0) -> dict:
    """The whole -direct block of main.cc (runRay + depth + runNorms +
    runAlbedo) in one launch on the Cornell box: dict of float32 buffers
    'color', 'normals', 'albedo' ([nx*ny, 4]) and 'depth' ([nx*ny])."""
    dev = device if isinstance(device, Device) else Device(device)
    dev.set_cornell_box(cb.variant)
    qs = quad_scalars(cb.ds.GetField("point_var").values, cb.ds.GetCellSet().quad_cells)
    cmap = main_pallet_color_table().Sample(1024)
    return render_direct(dev, cam, nx, ny, qs, cmap, aovs=7, depth=True)


def save_depth_pnm(path: str, depth: np.ndarray, nx: int, ny: int) -> None:
    """save<vtkm::Float32> (main.cc:346-359)."""
    a = np.ascontiguousarray(depth, dtype=np.float32)
    check(_lib.load().rtp_write_pnm_depth(path.encode(), a.ctypes.data_as(_lib.f32p), nx, ny))
