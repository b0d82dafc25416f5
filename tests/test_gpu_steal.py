"""Work stealing in the pool kernel (rtp_kernels.hip pool_body kSteal): a
launch with more entries than the resident waves' pools hold runs the
resident waves, each refilling a finished pixel's slot with the next
unclaimed entry.  Per-pixel sample, draw and summation order are the same,
so the output must equal the generation schedule's (RTP_STEAL=0) bit for
bit, and the oracle's on any pixel."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from _util import assert_render_equal, same_bits_or_both_nan

pytestmark = pytest.mark.gpu


def _steals(npix: int, bvh: int) -> bool:
    from raytracingtherestofyourlife_amd import _lib

    L = _lib.load()
    L.rtp_plan_steal.restype = ctypes.c_int
    L.rtp_plan_steal.argtypes = [ctypes.c_int64, ctypes.c_int]
    return L.rtp_plan_steal(npix, bvh) > 0


def _render_range(device, nx, ny, spp, depth, begin, count, steal, monkeypatch):
    import torch

    import raytracingtherestofyourlife_amd as rtp

    monkeypatch.setenv("RTP_STEAL", "1" if steal else "0")
    out = torch.full((count, 4), 3.0, dtype=torch.float32, device="cuda")
    seeds = torch.zeros(count, dtype=torch.int32, device="cuda")
    live = torch.zeros(count, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    device.render_device(rtp.default_camera(), nx, ny, spp, depth, out.data_ptr(), pixel_begin=begin,
                         pixel_count=count, stream=s, seed_ptr=seeds.data_ptr(), live_ptr=live.data_ptr())
    torch.cuda.synchronize()
    return out.cpu().numpy(), seeds.cpu().numpy().view(np.uint32), live.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("variant,nx,ny,spp", [(0, 1920, 1080, 6), (3, 1024, 1024, 2)])
def test_steal_equals_generations(device, monkeypatch, variant, nx, ny, spp):
    """C4's canvas (2.07 M pixels) and a 1000-sphere canvas (BVH instance):
    the stealing schedule and the generation schedule agree on every pixel's
    sum, final RNG state and live-bounce count."""
    npix = nx * ny
    assert _steals(npix, 1 if variant == 3 else 0), "the launch must be large enough to steal"
    device.set_cornell_box(variant)
    try:
        a = _render_range(device, nx, ny, spp, 50, 0, npix, True, monkeypatch)
        b = _render_range(device, nx, ny, spp, 50, 0, npix, False, monkeypatch)
    finally:
        device.set_cornell_box(0)
    ok = same_bits_or_both_nan(a[0][:, :3], b[0][:, :3]).all(axis=1)
    assert ok.all(), f"{int((~ok).sum())} pixels differ, first {np.flatnonzero(~ok)[:8].tolist()}"
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])


def test_steal_matches_oracle(device, oracle, monkeypatch):
    """A stolen C4-canvas render (entries claimed in launch order after the
    initial pools) against the oracle on pixels from the whole range,
    including the last ones claimed."""
    nx, ny, spp, depth = 1920, 1080, 4, 50
    npix = nx * ny
    got = _render_range(device, nx, ny, spp, depth, 0, npix, True, monkeypatch)
    pix = np.unique(np.r_[np.random.default_rng(21).choice(npix, 192, replace=False), np.arange(npix - 64, npix),
                          np.arange(0, 32)]).astype(np.int64)
    want = oracle.render_pixels(oracle.cornell_box(0), oracle.camera_setup(nx, ny), nx, ny, spp, depth, pix)
    assert_render_equal((got[0][pix], got[1][pix], got[2][pix]), want, "stolen C4 canvas")


def test_steal_tile_deal(device, monkeypatch):
    """The tile-deal instance steals too (a one-rank deal of C4's canvas)."""
    import torch

    import raytracingtherestofyourlife_amd as rtp

    nx, ny = 1920, 1088  # whole 16x16 tiles
    n = nx * ny
    s = torch.cuda.current_stream().cuda_stream
    outs = []
    for steal in ("1", "0"):
        monkeypatch.setenv("RTP_STEAL", steal)
        o = torch.full((n, 4), 5.0, dtype=torch.float32, device="cuda")
        device.render_tiles_device(rtp.default_camera(), nx, ny, 3, 50, o.data_ptr(), 0, 1, stream=s)
        torch.cuda.synchronize()
        outs.append(o.cpu().numpy())
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
