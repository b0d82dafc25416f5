"""rtp_render_tiles_device (the tile deal computed in the kernel) against
rtp_render_device with shard.tile_pixels' explicit list: bit-identical
output, entry for entry, for every rank of several deals."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nx,ny,world,variant", [(64, 48, 1, 0), (64, 48, 2, 0), (80, 32, 3, 0), (48, 64, 5, 0),
                                                  (64, 48, 3, 3), (40, 30, 2, 0), (100, 36, 3, 0), (72, 40, 4, 3)])
def test_gpu_tile_deal_equals_pixel_list(device, nx, ny, world, variant):
    """Whole-tile canvases and clipped ones (the C4 case: 1080 rows): the
    entries inside the canvas (shard.tile_entries) equal the pixel-list
    render of shard.tile_pixels bit for bit."""
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard

    device.set_cornell_box(variant)  # 3: the 1000-sphere C3 scene (the BVH kernel instance)
    cam = rtp.default_camera()
    s = torch.cuda.current_stream().cuda_stream
    tiles = -(-nx // 16) * -(-ny // 16)
    for rank in range(world):
        ids_np = shard.tile_pixels(nx, ny, rank, world)
        ent, pix = shard.tile_entries(nx, ny, rank, world)
        assert np.array_equal(pix, ids_np)
        mine = len(range(rank, tiles, world))
        ids = torch.from_numpy(ids_np).cuda()
        a = torch.full((ids_np.size, 4), 7.0, dtype=torch.float32, device="cuda")
        b = torch.full((256 * mine + 64, 4), 9.0, dtype=torch.float32, device="cuda")  # (+64: no write past the tiles)
        device.render_device(cam, nx, ny, 5, 10, a.data_ptr(), pixel_count=ids_np.size, pixel_ids_ptr=ids.data_ptr(),
                             stream=s)
        device.render_tiles_device(cam, nx, ny, 5, 10, b.data_ptr(), rank, world, stream=s)
        torch.cuda.synchronize()
        an, bn = a.cpu().numpy(), b.cpu().numpy()
        assert np.array_equal(an.view(np.uint32), bn[ent].view(np.uint32)), (nx, ny, world, rank)
        assert (bn[256 * mine:] == 9.0).all(), "entries past the rank's tiles were written"
    device.set_cornell_box(0)


def test_gpu_tile_deal_rank_without_tiles(device):
    """More ranks than tiles (a 40x20 canvas has 6 tiles, 8 ranks): ranks 6
    and 7 own nothing -- the call succeeds and writes nothing; the others
    still match the pixel list."""
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard

    device.set_cornell_box(0)
    cam = rtp.default_camera()
    for rank in range(8):
        ent, pix = shard.tile_entries(40, 20, rank, 8)
        out = torch.full((256, 4), 3.0, dtype=torch.float32, device="cuda")
        device.render_tiles_device(cam, 40, 20, 2, 5, out.data_ptr(), rank, 8)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        if rank >= 6:
            assert ent.size == 0 and (o == 3.0).all()
            continue
        ids = torch.from_numpy(pix).cuda()
        a = torch.zeros((pix.size, 4), dtype=torch.float32, device="cuda")
        device.render_device(cam, 40, 20, 2, 5, a.data_ptr(), pixel_count=pix.size, pixel_ids_ptr=ids.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(a.cpu().numpy().view(np.uint32), o[ent].view(np.uint32)), rank


def test_gpu_tile_deal_rejects_bad_rank(device):
    import torch

    import raytracingtherestofyourlife_amd as rtp

    out = torch.empty((256, 4), dtype=torch.float32, device="cuda")
    with pytest.raises(Exception):
        device.render_tiles_device(rtp.default_camera(), 32, 32, 1, 5, out.data_ptr(), 2, 2)
    with pytest.raises(Exception):
        device.render_tiles_device(rtp.default_camera(), 32, 32, 1, 5, out.data_ptr(), -1, 2)


def test_launch_rejects_more_than_int32_entries(device):
    """The kernels index a launch's entries with 32-bit integers: a pixel list
    of 2^31 entries is refused before any allocation (rtp_host.cpp launch)."""
    import ctypes

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd._lib import RtpPixelAux, check

    device.set_cornell_box(0)
    cam = rtp.default_camera().to_c()
    L = rtp.load()
    st = L.rtp_render_device(device.handle, ctypes.byref(cam), 800, 800, 1, 5, 0, 0, 1 << 31,
                             ctypes.c_void_p(0x1000), ctypes.c_void_p(0x2000), ctypes.byref(RtpPixelAux()),
                             ctypes.c_void_p(None), None)
    assert st == rtp._lib.RTP_ERR_INVALID_ARGUMENT
    assert "2^31" in L.rtp_last_error().decode()
    with pytest.raises(rtp.RtpError):
        check(st)
