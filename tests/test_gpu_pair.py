"""Two paths per lane (rtp_kernels.hip pool_body_pair, opt-in RTP_PAIR=1):
each lane of a 128-pixel pool carries two paths, and one closest-hit pass
tests every quad against both rays.  The pool protocol (queues, fast-forward
batch, per-pixel sample and summation order) is the single-path kernel's, so
every pixel's sum, final RNG state and live-bounce count must equal the
plain launch's bit for bit, and the oracle's.

Reference: MapperPathTracer.cxx:278-350 (each pixel's sample chain)."""
from __future__ import annotations

import numpy as np
import pytest

from _util import assert_render_equal, same_bits_or_both_nan

pytestmark = pytest.mark.gpu


def _render(device, monkeypatch, pair, nx, ny, spp, depth, begin=0, count=None, tiles=None):
    import torch

    import raytracingtherestofyourlife_amd as rtp

    monkeypatch.setenv("RTP_PAIR", "1" if pair else "0")
    if tiles is not None:
        rank, world = tiles
        n = 256 * len(range(rank, ((nx + 15) // 16) * ((ny + 15) // 16), world))
    else:
        n = count if count is not None else nx * ny
    out = torch.full((n, 4), 3.0, dtype=torch.float32, device="cuda")
    seeds = torch.zeros(n, dtype=torch.int32, device="cuda")
    live = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    if tiles is None:
        device.render_device(rtp.default_camera(), nx, ny, spp, depth, out.data_ptr(), pixel_begin=begin,
                             pixel_count=n, stream=s, seed_ptr=seeds.data_ptr(), live_ptr=live.data_ptr())
    else:
        device.render_tiles_device(rtp.default_camera(), nx, ny, spp, depth, out.data_ptr(), rank, world, stream=s)
    torch.cuda.synchronize()
    return out.cpu().numpy(), seeds.cpu().numpy().view(np.uint32), live.cpu().numpy().view(np.uint32)


def _assert_same(a, b, what):
    ok = same_bits_or_both_nan(a[0][:, :3], b[0][:, :3]).all(axis=1)
    assert ok.all(), f"{what}: {int((~ok).sum())} pixels differ, first {np.flatnonzero(~ok)[:8].tolist()}"
    assert np.array_equal(a[1], b[1]), f"{what}: final seeds differ"
    assert np.array_equal(a[2], b[2]), f"{what}: live counts differ"


@pytest.mark.parametrize("variant", [0, 2])
def test_pair_matches_oracle(device, oracle, monkeypatch, variant):
    """A small frame of the C2 scene (and the glass variant) against the oracle."""
    nx, ny, spp, depth = 96, 64, 16, 50
    device.set_cornell_box(variant)
    try:
        got = _render(device, monkeypatch, True, nx, ny, spp, depth)
    finally:
        device.set_cornell_box(0)
    want = oracle.render_pixels(oracle.cornell_box(variant), oracle.camera_setup(nx, ny), nx, ny, spp, depth,
                                np.arange(nx * ny, dtype=np.int64))
    assert_render_equal(got, want, f"two paths per lane, variant {variant}")


def test_pair_equals_plain_on_a_share(device, monkeypatch):
    """Rank 3 of 8's tile share of a 480x272 canvas at 256 spp (long chains,
    few waves: the launches this kernel is for), tile-deal instance, and a
    pixel range through the contiguous instance."""
    nx, ny, spp, depth = 480, 272, 256, 50
    a = _render(device, monkeypatch, True, nx, ny, spp, depth, tiles=(3, 8))
    b = _render(device, monkeypatch, False, nx, ny, spp, depth, tiles=(3, 8))
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), "tile share differs"
    a = _render(device, monkeypatch, True, nx, ny, spp, depth, begin=5000, count=20000)
    b = _render(device, monkeypatch, False, nx, ny, spp, depth, begin=5000, count=20000)
    _assert_same(a, b, "pixel range")
