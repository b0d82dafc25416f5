"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same inputs.  Bar: bit-exact rgb sums (NaN-aware), identical final RNG state
and live-bounce count per pixel.  The final RNG state is the strongest check:
it encodes every draw the pixel consumed over all samples and depths, so it
only matches if every branch that decides a draw count matched."""
from __future__ import annotations

import numpy as np
import pytest

from _util import assert_render_equal, rmse_normalized, set_scene_from_oracle

pytestmark = pytest.mark.gpu


def _cam(rtp, **kw):
    cam = rtp.default_camera()
    for k, v in kw.items():
        getattr(cam, k)(v)
    return cam


@pytest.fixture(scope="module")
def rtp():
    import raytracingtherestofyourlife_amd as m

    return m


def _render_both(oracle, device, rtp, variant, nx, ny, spp, depth, pixels=None, seed_base=0, cam=None):
    cam = cam or rtp.default_camera()
    device.set_cornell_box(variant)
    sc = oracle.cornell_box(variant)
    ocam = oracle.camera_setup(nx, ny, cam.position, cam.look_at, cam.view_up, cam.fov)
    if pixels is None:
        pixels = np.arange(nx * ny, dtype=np.int64)
    got = device.render_pixels(cam, nx, ny, spp, depth, pixels, seed_base=seed_base)[:3]
    want = oracle.render_pixels(sc, ocam, nx, ny, spp, depth, pixels, seed_base=seed_base)
    return got, want


def test_device_sincos_match_glibc_restatement(oracle, device):
    """glibc-exact sinf/cosf port on the device == oracle restatement on every
    phi = float(2*pi*r) the samplers can produce from a sample of hashes, plus
    a dense sweep of [0, 2pi]."""
    rng = np.random.default_rng(1)
    r = (rng.integers(0, 2**32, size=1 << 20, dtype=np.uint64).astype(np.float32) / np.float32(4294967295.0))
    phi = (2 * np.pi * r.astype(np.float64)).astype(np.float32)
    sweep = np.linspace(0, 2 * np.pi, 1 << 20, dtype=np.float32)
    x = np.concatenate([phi, sweep, np.float32([0, 1e-30, 0.785398, 0.7853982, 6.2831855])])
    ds = device.eval_primitive(0, x)
    dc = device.eval_primitive(1, x)
    L = oracle.lib()
    os_ = np.array([L.rtpo_sinf(float(v)) for v in x[:20000]], dtype=np.float32)
    oc_ = np.array([L.rtpo_cosf(float(v)) for v in x[:20000]], dtype=np.float32)
    assert np.array_equal(ds[:20000].view(np.uint32), os_.view(np.uint32))
    assert np.array_equal(dc[:20000].view(np.uint32), oc_.view(np.uint32))
    # the rest against numpy float32 via libm (== restatement, see CPU test)
    import ctypes

    libm = ctypes.CDLL("libm.so.6")
    libm.sinf.restype = libm.cosf.restype = ctypes.c_float
    libm.sinf.argtypes = libm.cosf.argtypes = [ctypes.c_float]
    idx = np.random.default_rng(2).choice(x.size, 20000, replace=False)
    assert all(np.float32(libm.sinf(float(x[i]))).view(np.uint32) == ds[i].view(np.uint32) for i in idx)
    assert all(np.float32(libm.cosf(float(x[i]))).view(np.uint32) == dc[i].view(np.uint32) for i in idx)


def test_device_wang_and_rsqrt(oracle, device):
    rng = np.random.default_rng(3)
    u = rng.integers(0, 2**32, size=1 << 16, dtype=np.uint64).astype(np.uint32)
    got = device.eval_primitive(3, u)
    want = np.array([oracle.wang32(int(v)) for v in u[:4096]], dtype=np.uint32)
    assert np.array_equal(got[:4096], want)
    f = np.abs(rng.standard_normal(1 << 16).astype(np.float32)) * np.float32(3.0) + np.float32(1e-3)
    got = device.eval_primitive(2, f)
    want = (np.float32(1) / np.sqrt(f)).astype(np.float32)  # IEEE sqrt + div, correctly rounded
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_c1_full_image_bit_exact(oracle, device, rtp):
    """BASELINE config C1: Cornell Box 200x200, 10 spp, depth 10 -- full image."""
    got, want = _render_both(oracle, device, rtp, 0, 200, 200, 10, 10)
    assert_render_equal(got, want, "C1")
    assert rmse_normalized(got[0], want[0], 10) == 0.0


def test_visible_glass_sphere_bit_exact(oracle, device, rtp):
    """Dielectric path: variant 2 (clean glass sphere) and variant 1 (notebook
    cell 2 position, overlapping a box: NaN-poisoning stress case)."""
    got, want = _render_both(oracle, device, rtp, 2, 96, 96, 32, 20)
    assert_render_equal(got, want, "glass sphere v2")
    got, want = _render_both(oracle, device, rtp, 1, 96, 96, 16, 12)
    assert_render_equal(got, want, "glass sphere v1")
    # the dielectric really was exercised: the two scenes differ
    other = device.render_pixels(rtp.default_camera(), 96, 96, 16, 12, np.arange(96 * 96))[0]
    device.set_cornell_box(0)
    base = device.render_pixels(rtp.default_camera(), 96, 96, 16, 12, np.arange(96 * 96))[0]
    assert not np.array_equal(other, base)


def test_non_square_canvas_fov_quirk(oracle, device, rtp):
    """Non-square canvases use FovY for both axes (Camera.cxx:925-931)."""
    got, want = _render_both(oracle, device, rtp, 0, 72, 40, 6, 8)
    assert_render_equal(got, want, "72x40")
    got, want = _render_both(oracle, device, rtp, 0, 33, 65, 5, 6)
    assert_render_equal(got, want, "33x65")


def test_c2_camera_pixel_subset_full_depth(oracle, device, rtp):
    """C2 geometry (800x800, depth 50) on a random pixel subset, reduced spp."""
    rng = np.random.default_rng(7)
    pix = np.sort(rng.choice(800 * 800, 2048, replace=False)).astype(np.int64)
    got, want = _render_both(oracle, device, rtp, 0, 800, 800, 8, 50, pixels=pix)
    assert_render_equal(got, want, "C2 subset")


def test_edge_cases(oracle, device, rtp):
    for (nx, ny, spp, depth) in [(1, 1, 3, 1), (2, 3, 1, 2), (5, 4, 0, 3), (16, 16, 2, 1), (7, 9, 3, 64)]:
        got, want = _render_both(oracle, device, rtp, 0, nx, ny, spp, depth)
        assert_render_equal(got, want, f"{nx}x{ny} spp{spp} d{depth}")


def test_seed_base_stream_offset(oracle, device, rtp):
    """seed = seed_base + pixel (the derived streams of the sample-batch shard)."""
    got, want = _render_both(oracle, device, rtp, 0, 40, 40, 4, 10, seed_base=40 * 40 * 3)
    assert_render_equal(got, want, "seed_base")


def test_other_camera(oracle, device, rtp):
    cam = rtp.Camera()
    cam.SetPosition([0.9, 0.2, -0.9])
    cam.SetLookAt([0.4, 0.5, 0.6])
    cam.SetViewUp([0.1, 2.0, 0.0])  # non-unit up is normalised (Camera.cxx:767-776)
    cam.SetFieldOfView(55.0)
    got, want = _render_both(oracle, device, rtp, 1, 48, 48, 6, 10, cam=cam)
    assert_render_equal(got, want, "camera")


def test_render_device_matches_host_path(device, rtp):
    import torch

    device.set_cornell_box(0)
    cam = rtp.default_camera()
    nx = ny = 64
    out = torch.zeros((nx * ny, 4), dtype=torch.float32, device="cuda")
    seeds = torch.zeros(nx * ny, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    device.render_device(cam, nx, ny, 5, 10, out.data_ptr(), seed_ptr=seeds.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    host, hseed, _, _ = device.render_pixels(cam, nx, ny, 5, 10, np.arange(nx * ny))
    assert np.array_equal(out.cpu().numpy().view(np.uint32), host.view(np.uint32))
    assert np.array_equal(seeds.cpu().numpy().view(np.uint32), hseed)
    # contiguous sub-range == the same pixels of the full render
    part = torch.zeros((100, 4), dtype=torch.float32, device="cuda")
    device.render_device(cam, nx, ny, 5, 10, part.data_ptr(), pixel_begin=1000, pixel_count=100, stream=stream)
    torch.cuda.synchronize()
    assert np.array_equal(part.cpu().numpy().view(np.uint32), host[1000:1100].view(np.uint32))


def test_renders_on_two_streams_share_one_context(device, rtp):
    """Back-to-back asynchronous renders of one context on two streams (and a
    scene change while one is queued) are ordered by the context: the
    per-context history buffer and progress counter are never used by two
    kernels at once."""
    import torch

    cam = rtp.default_camera()
    nx = ny = 96
    device.set_cornell_box(0)
    want0 = device.render_pixels(cam, nx, ny, 6, 12, np.arange(nx * ny))[0]
    device.set_cornell_box(2)
    want2 = device.render_pixels(cam, nx, ny, 6, 12, np.arange(nx * ny))[0]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.zeros((nx * ny, 4), dtype=torch.float32, device="cuda")
    b = torch.zeros_like(a)
    c = torch.zeros_like(a)
    device.set_cornell_box(0)
    device.render_device(cam, nx, ny, 6, 12, a.data_ptr(), stream=s1.cuda_stream)
    device.render_device(cam, nx, ny, 6, 12, b.data_ptr(), stream=s2.cuda_stream)
    device.set_cornell_box(2)  # waits for the queued renders before replacing the scene
    device.render_device(cam, nx, ny, 6, 12, c.data_ptr(), stream=s1.cuda_stream)
    torch.cuda.synchronize()
    for got, want, name in ((a, want0, "stream 1"), (b, want0, "stream 2"), (c, want2, "after set_scene")):
        assert np.array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32)), name


def test_mapper_api_runpath(oracle, device, rtp):
    """The reference's own call sequence (main.cc:289-323) through the mirror."""
    cb = rtp.CornellBox()
    cb.buildDataSet()
    canvas = rtp.CanvasRayTracer(40, 30)
    cam = rtp.default_camera()
    rtp.runPath(40, 30, 4, 6, canvas, cam, cb, device=device)
    img = canvas.GetColorBuffer()
    sc = oracle.cornell_box(0)
    ocam = oracle.camera_setup(40, 30)
    want, _, _ = oracle.render_pixels(sc, ocam, 40, 30, 4, 6, np.arange(1200))
    want = oracle.normalize(want, 4)
    assert np.array_equal(img[:, :3].view(np.uint32), want[:, :3].view(np.uint32))
    with pytest.raises(rtp.ErrorBadValue):
        rtp.MapperPathTracer(1, 1, cb.matIdx, cb.texIdx, cb.matType, cb.texType, cb.tex,
                             device=device).SetCanvas(rtp.mapper.Canvas(2, 2))


def test_invalid_arguments(device, rtp):
    cam = rtp.default_camera()
    with pytest.raises(rtp.RtpError):
        device.render(cam, 0, 10, 1, 1)
    with pytest.raises(rtp.RtpError):
        device.render(cam, 10, 10, 1, 0)  # depthcount < 1
    bad = rtp.Camera()
    bad.SetFieldOfView(0.0)
    with pytest.raises(rtp.RtpError):
        device.render(bad, 4, 4, 1, 1)
    with pytest.raises(rtp.RtpError):
        device.render_pixels(cam, 4, 4, 1, 1, np.array([16], dtype=np.int64))
    with pytest.raises(rtp.RtpError):  # device bookkeeping limits (rtp_layout.hpp kMaxDepth / kMaxSpp)
        device.render(cam, 4, 4, 1, 16384)
    with pytest.raises(rtp.RtpError):
        device.render(cam, 4, 4, 8388608, 1)


def test_depth_at_the_bookkeeping_limit(oracle, device, rtp):
    """depthcount up to kMaxDepth = 16383 (s_rem's 14-bit count field): a
    deep render of a few pixels equals the oracle's, final seeds and
    live-bounce counts included (almost every depth is a dead one, so the
    fast-forward runs its full chain of jump tables and hashed steps)."""
    nx, ny = 6, 4
    pix = np.arange(nx * ny, dtype=np.int64)
    got, want = _render_both(oracle, device, rtp, 0, nx, ny, 3, 16383, pix)
    assert_render_equal(got, want, "depth 16383")


def test_empty_pixel_list_and_zero_spp(device, rtp):
    import torch

    cam = rtp.default_camera()
    out = torch.full((4, 4), 7.0, dtype=torch.float32, device="cuda")
    device.render_device(cam, 8, 8, 4, 5, out.data_ptr(), pixel_begin=0, pixel_count=0,
                         stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert bool((out == 7.0).all())  # nothing written
    rgba, _ = device.render(cam, 8, 8, 0, 5)  # spp 0: the canvas is zero
    assert not rgba[:, :3].any()


def test_c3_many_spheres_bvh_subset(oracle, device, rtp):
    """C3 geometry (2048x2048, 1000 spheres behind the BVH, depth 50): random
    pixel subset at full depth against the brute-force oracle."""
    nx = ny = 2048
    pix = np.sort(np.random.default_rng(33).choice(nx * ny, size=384, replace=False)).astype(np.int64)
    got, want = _render_both(oracle, device, rtp, 3, nx, ny, 4, 50, pix)
    assert_render_equal(got, want, "c3")
    assert (want[2] > 4).any()


@pytest.mark.parametrize("n", [2, 8, 9, 40])
def test_sphere_count_threshold_and_coincident_tie(oracle, device, rtp, n):
    """Below, at and above the BVH threshold (kBvhMinSpheres = 9), with the
    last sphere coincident with sphere 1 but another material: the reference's
    index-order scan keeps the lower index on equal t, and so must the BVH."""
    sc = oracle.cornell_box(3)
    sc.n_spheres = n
    sc.sphere_point[n - 1] = sc.sphere_point[1]
    sc.sphere_radius[n - 1] = sc.sphere_radius[1]
    sc.sphere_mat[n - 1] = 4 if sc.sphere_mat[1] != 4 else 1
    sc.sphere_tex[n - 1] = 0
    set_scene_from_oracle(device, sc)
    nx, ny = 96, 96
    cam = rtp.default_camera()
    pix = np.arange(nx * ny, dtype=np.int64)
    got = device.render_pixels(cam, nx, ny, 4, 12, pix)[:3]
    want = oracle.render_pixels(sc, oracle.camera_setup(nx, ny), nx, ny, 4, 12, pix)
    assert_render_equal(got, want, f"{n} spheres")
