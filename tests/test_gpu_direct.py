"""GPU parity of the -direct mode (main.cc:120-251): the HIP kernel
(rtp_render_direct through the C ABI) against the oracle and its committed
fixtures.  Bar: bit-exact colour, normals, albedo and depth buffers (NaN
matches NaN: in-subset misses have NaN depth in the reference too)."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from _util import same_bits_or_both_nan
from test_direct import FIXTURES, _load, _oracle_direct

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rtp():
    import raytracingtherestofyourlife_amd as m

    return m


def _camera(rtp, g):
    cam = rtp.default_camera()
    if "cam_position" in g:
        cam.SetPosition(g["cam_position"])
    if "cam_look_at" in g:
        cam.SetLookAt(g["cam_look_at"])
    if "cam_view_up" in g:
        cam.SetViewUp(g["cam_view_up"])
    if "cam_fov_y" in g:
        cam.SetFieldOfView(float(g["cam_fov_y"]))
    cam.SetClippingRange(*[float(c) for c in g["clip"]])
    return cam


def _assert_same(got, want, what):
    ok = same_bits_or_both_nan(got, want)
    if ok.ndim > 1:
        ok = ok.all(axis=1)
    bad = np.flatnonzero(~ok)
    assert bad.size == 0, f"{what}: {bad.size} pixels differ, first {bad[:6].tolist()}: {got[bad[:3]]} vs {want[bad[:3]]}"


@pytest.mark.parametrize("name", FIXTURES)
def test_direct_fixture_bit_exact(rtp, device, name):
    g = _load(name)
    variant, nx, ny = int(g["variant"]), int(g["nx"]), int(g["ny"])
    cb = rtp.CornellBox(variant=variant)
    cb.buildDataSet()
    device.set_cornell_box(variant)
    qs = rtp.direct.quad_scalars(cb.ds.GetField("point_var").values, cb.ds.GetCellSet().quad_cells)
    out = rtp.direct.render_direct(device, _camera(rtp, g), nx, ny, qs, g["cmap"], aovs=7, depth=True)
    for key in ("color", "normals", "albedo", "depth"):
        _assert_same(out[key], g[key], f"{name}/{key}")


def test_direct_single_aov_launches_match(rtp, device, oracle):
    """Each AOV rendered alone (one mapper per launch, as main.cc does) equals
    the fused launch and the oracle; hemisphere views of generate()."""
    cb = rtp.CornellBox(variant=0)
    cb.buildDataSet()
    device.set_cornell_box(0)
    qs = rtp.direct.quad_scalars(cb.ds.GetField("point_var").values, cb.ds.GetCellSet().quad_cells)
    cmap = oracle.sample_color_table()
    sc = oracle.cornell_box(0)
    r = -1078 / 555.0
    for phi, theta in ((0.0, 0.0), (0.2, 2.5132742), (0.6, 4.3982296), (0.93333334, 5.8643064)):
        pos = np.float32([r * np.cos(np.float32(theta)) * np.sin(np.float32(phi)) + 278 / 555.0,
                          r * np.sin(np.float32(theta)) * np.sin(np.float32(phi)) + 278 / 555.0,
                          r * np.cos(np.float32(phi)) + 278 / 555.0])
        cam = rtp.default_camera()
        cam.SetPosition(pos)
        ocam = oracle.direct_setup(sc, 72, 56, position=pos)
        fused = rtp.direct.render_direct(device, cam, 72, 56, qs, cmap, aovs=7, depth=True)
        for key, aov in (("color", 1), ("normals", 2), ("albedo", 4)):
            one = rtp.direct.render_direct(device, cam, 72, 56, qs, cmap, aovs=aov, depth=True)
            want, wdepth = oracle.render_direct(sc, ocam, aov, cmap=cmap)
            _assert_same(one[key], want, f"view {phi},{theta} {key}")
            _assert_same(fused[key], want, f"view {phi},{theta} fused {key}")
            _assert_same(one["depth"], wdepth, f"view {phi},{theta} depth")


def test_view3d_mapper_api(rtp, oracle):
    """runRay / runNorms / runAlbedo through View3D + MapperQuad* (main.cc's
    own sequence) fill the canvas like the oracle."""
    cb = rtp.CornellBox()
    cb.buildDataSet()
    canvas = rtp.CanvasRayTracer(80, 64)
    cam = rtp.default_camera()
    sc = oracle.cornell_box(0)
    ocam = oracle.direct_setup(sc, 80, 64)
    dev = rtp.Device(0)
    try:
        for fn, aov in ((rtp.runRay, 1), (rtp.runNorms, 2), (rtp.runAlbedo, 4)):
            fn(80, 64, 10, 5, canvas, cam, cb, device=dev)
            want, wdepth = oracle.render_direct(sc, ocam, aov)
            _assert_same(canvas.GetColorBuffer(), want, fn.__name__)
            _assert_same(canvas.GetDepthBuffer(), wdepth, fn.__name__ + " depth")
    finally:
        dev.close()


def test_device_powf_matches_libm(rtp, device):
    """Device glibc powf restatement vs the host libm's powf (called through
    ctypes: numpy's float32 power is its own SIMD code, not libm) over a
    sample of [0, 1.01], the values just below 1, and special values."""
    import ctypes

    libm = ctypes.CDLL("libm.so.6")
    libm.powf.restype = ctypes.c_float
    libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    x = np.concatenate([np.arange(0, 0x3F8147AE, 4099, dtype=np.uint32).view(np.float32),
                        np.arange(0x3F7F0000, 0x3F800400, 1, dtype=np.uint32).view(np.float32),
                        np.float32([0.0, -0.0, 1e-45, 1.0, np.inf, np.nan, 0.5, 0.999999])])
    got = np.zeros_like(x)
    check = rtp.load().rtp_eval_powf(device.handle, x.ctypes.data_as(rtp._lib.f32p), ctypes.c_float(20.0),
                                     got.ctypes.data_as(rtp._lib.f32p), x.size)
    assert check == 0
    want = np.array([libm.powf(float(v), 20.0) for v in x], dtype=np.float32)
    assert same_bits_or_both_nan(got, want).all()


def test_cpp_direct_cli_writes_reference_pnms(rtp, oracle, tmp_path):
    """examples/rtp_path -direct: direct/depth/normals/albedo.pnm equal the
    oracle's buffers through main.cc's save()."""
    exe = os.path.join(ROOT, "examples", "rtp_path")
    subprocess.run([exe, "-x", "48", "-y", "40", "-direct"], cwd=tmp_path, check=True, capture_output=True,
                   timeout=120)
    sc = oracle.cornell_box(0)
    ocam = oracle.direct_setup(sc, 48, 40)
    for name, aov in (("direct", 1), ("normals", 2), ("albedo", 4)):
        want, wdepth = oracle.render_direct(sc, ocam, aov)
        p = tmp_path / f"want_{name}.pnm"
        rtp.save_pnm(str(p), want, 48, 40)
        assert (tmp_path / f"{name}.pnm").read_text() == p.read_text(), name
    p = tmp_path / "want_depth.pnm"
    rtp.save_depth_pnm(str(p), wdepth, 48, 40)
    assert (tmp_path / "depth.pnm").read_text() == p.read_text()


@pytest.mark.parametrize("nx,ny,pos,look", [
    (1, 1, None, None),                                      # one pixel
    (7, 40, None, None),                                     # tall canvas: FovX from SetFieldOfView
    (33, 21, (0.5, 0.5, -3.0), (0.5, 0.5, -4.0)),            # looking away: FindSubset -> 1x1 at (0, 0)
    (40, 30, (0.5, 0.5, 0.5), (0.2, 0.9, 0.7)),             # camera inside the bounds: full canvas
])
def test_direct_edge_cameras(rtp, device, oracle, nx, ny, pos, look):
    cb = rtp.CornellBox()
    cb.buildDataSet()
    device.set_cornell_box(0)
    qs = rtp.direct.quad_scalars(cb.ds.GetField("point_var").values, cb.ds.GetCellSet().quad_cells)
    cmap = oracle.sample_color_table()
    cam = rtp.default_camera()
    kw = {}
    if pos is not None:
        cam.SetPosition(pos)
        cam.SetLookAt(look)
        kw = dict(position=np.float32(pos), look_at=np.float32(look))
    sc = oracle.cornell_box(0)
    ocam = oracle.direct_setup(sc, nx, ny, **kw)
    if pos is not None and pos[2] == -3.0:
        assert [ocam.sub_x0, ocam.sub_y0, ocam.sub_w, ocam.sub_h] == [0, 0, 1, 1]
    if pos is not None and pos[2] == 0.5:
        assert [ocam.sub_x0, ocam.sub_y0, ocam.sub_w, ocam.sub_h] == [0, 0, nx, ny]
    got = rtp.direct.render_direct(device, cam, nx, ny, qs, cmap, aovs=7, depth=True)
    for key, aov in (("color", 1), ("normals", 2), ("albedo", 4)):
        want, wdepth = oracle.render_direct(sc, ocam, aov, cmap=cmap)
        _assert_same(got[key], want, f"{nx}x{ny} {key}")
        _assert_same(got["depth"], wdepth, f"{nx}x{ny} depth")
