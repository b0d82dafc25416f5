"""The production schedule of the large configurations, at their full sample
counts.  C3 (2048^2 x 256 spp, 1000 spheres), C4 (1920x1080 x 4096 spp) and
a C5 frame (3840x2160) hold more pixels than the resident waves' pools
(5120 x 128 entries), so on one GPU they run the work-stealing instance of
the pool kernel (rtp_kernels.hip pool_body kSteal).  Each test renders the
WHOLE canvas (or a rank's whole share of it) through the default device path,
exactly as the timings of DESIGN.md 5 were taken, and checks the committed
full-S x D golden subsets (tools/make_golden.py, from the oracle) bit for
bit: rgb sums (NaN-aware), final RNG states and live-bounce counts.
Reference: MapperPathTracer.cxx:278-350 (the per-pixel sample loop)."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from _util import assert_render_equal

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def _steal_waves(npix: int, bvh: int) -> int:
    from raytracingtherestofyourlife_amd import _lib

    L = _lib.load()
    L.rtp_plan_steal.restype = ctypes.c_int
    L.rtp_plan_steal.argtypes = [ctypes.c_int64, ctypes.c_int]
    return L.rtp_plan_steal(npix, bvh)


@pytest.fixture
def tables_on(device):
    """The jump-table policy the configuration timings use (bench.py --ff-tables on)."""
    before = device.ff_info()["policy"]
    device.set_ff_tables("on")
    yield
    device.set_ff_tables(before)


@pytest.mark.parametrize("name,shard", [("c4_subset16k", None), ("c4_subset16k", (0, 2)), ("c3_subset4k", None),
                                        ("c5_shard3_2048spp", None)])
def test_full_canvas_on_the_stealing_schedule(device, tables_on, name, shard):
    """name: the golden subset; shard (rank, world): render that rank's share
    of the 16x16 tile deal as a pixel list (bench.py's N > 1 path for
    canvases that are not whole tiles), else the whole canvas as one range."""
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard as sh

    g = _load(name)
    variant, nx, ny = int(g["variant"]), int(g["nx"]), int(g["ny"])
    spp, depth, seed_base = int(g["spp"]), int(g["depth"]), int(g["seed_base"])
    ids = None if shard is None else sh.tile_pixels(nx, ny, shard[0], shard[1])
    n = nx * ny if ids is None else ids.size
    assert _steal_waves(n, 1 if variant == 3 else 0) > 0, "the launch must take the work-stealing schedule"
    device.set_cornell_box(variant)
    try:
        out = torch.full((n, 4), 5.0, dtype=torch.float32, device="cuda")
        seeds = torch.zeros(n, dtype=torch.int32, device="cuda")
        live = torch.zeros(n, dtype=torch.int32, device="cuda")
        d_ids = None if ids is None else torch.from_numpy(ids).cuda()
        device.render_device(rtp.default_camera(), nx, ny, spp, depth, out.data_ptr(), pixel_count=n,
                             pixel_ids_ptr=0 if d_ids is None else d_ids.data_ptr(), seed_base=seed_base,
                             stream=torch.cuda.current_stream().cuda_stream, seed_ptr=seeds.data_ptr(),
                             live_ptr=live.data_ptr(), timed=True)
        torch.cuda.synchronize()
        rgba = out.cpu().numpy()
        sd = seeds.cpu().numpy().view(np.uint32)
        lv = live.cpu().numpy().view(np.uint32)
    finally:
        device.set_cornell_box(0)
    assert not (rgba[:, 3] != 0).any(), "every entry is written (alpha 0), none left at the fill value"
    if ids is None:
        pos, pix = g["pixels"], np.arange(g["pixels"].size)
    else:  # the golden pixels in this rank's tiles, and where the list holds them
        order = np.argsort(ids)
        hit = np.isin(g["pixels"], ids)
        pix = np.flatnonzero(hit)
        pos = order[np.searchsorted(ids[order], g["pixels"][hit])]
        assert pix.size > g["pixels"].size // 4
    got = (rgba[pos], sd[pos], lv[pos])
    want = (np.c_[g["rgb"][pix], np.zeros(pix.size, np.float32)], g["final_seed"][pix], g["live"][pix])
    assert_render_equal(got, want, f"{name} shard={shard}")


@pytest.mark.parametrize("rank,world", [(0, 2), (5, 8)])
def test_c4_share_through_the_tile_instance(device, tables_on, rank, world):
    """bench.py's N > 1 path on C4's 1080 rows: rtp_render_tiles_device renders
    the rank's tiles whole (clipped edge tiles included; the 1/2 share steals,
    the 1/8 share does not), and the entries inside the canvas
    (shard.tile_entries) match the c4_subset16k golden pixels bit for bit."""
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from _util import same_bits_or_both_nan
    from raytracingtherestofyourlife_amd import shard as sh

    g = _load("c4_subset16k")
    nx, ny, spp, depth = int(g["nx"]), int(g["ny"]), int(g["spp"]), int(g["depth"])
    assert int(g["variant"]) == 0 and int(g["seed_base"]) == 0 and ny % 16 != 0
    ent, ids = sh.tile_entries(nx, ny, rank, world)
    n_tiles = len(range(rank, -(-nx // 16) * -(-ny // 16), world))
    out = torch.full((256 * n_tiles, 4), 5.0, dtype=torch.float32, device="cuda")
    device.set_cornell_box(0)
    device.render_tiles_device(rtp.default_camera(), nx, ny, spp, depth, out.data_ptr(), rank, world,
                               stream=torch.cuda.current_stream().cuda_stream, timed=True)
    torch.cuda.synchronize()
    rgba = out.cpu().numpy()
    assert not (rgba[:, 3] != 0).any(), "every entry of the owned tiles is written"
    order = np.argsort(ids)
    hit = np.isin(g["pixels"], ids)
    pix = np.flatnonzero(hit)
    pos = ent[order[np.searchsorted(ids[order], g["pixels"][hit])]]
    assert pix.size > g["pixels"].size // (2 * world)
    ok = same_bits_or_both_nan(rgba[pos, :3], g["rgb"][pix]).all(axis=1)
    assert ok.all(), f"{int((~ok).sum())} of {pix.size} golden pixels differ"


@pytest.mark.skipif(not os.path.exists(os.path.join(GOLD, "c4_full_digest.npz")),
                    reason="tests/golden/c4_full_digest.npz not generated (tools/make_golden_digest.py)")
@pytest.mark.parametrize("launch", ["contiguous", "tiles"])
def test_c4_whole_frame_digest(device, tables_on, launch):
    """The WHOLE C4 frame (1920x1080, 4096 spp, depth 50: 8.5e9 samples, the
    tile shard's configuration) against the oracle's, every pixel: the
    SHA-256 of the rgb sums (NaN canonical), the NaN pixel list, and -- for
    the contiguous work-stealing launch, which carries them -- the digests of
    the final seeds and live-bounce counts.  `tiles`: the tile instance every
    rank of a C4 run launches (rank 0 of 1, clipped edge tiles rendered
    whole), its in-canvas entries scattered (shard.tile_entries)."""
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard as sh

    from _util import canonical_rgb_sha256, sha256_u32

    g = _load("c4_full_digest")
    device.set_cornell_box(int(g["variant"]))
    nx, ny, spp, depth = int(g["nx"]), int(g["ny"]), int(g["spp"]), int(g["depth"])
    n = nx * ny
    cam = rtp.default_camera()
    s = torch.cuda.current_stream().cuda_stream
    if launch == "contiguous":
        out = torch.empty((n, 4), dtype=torch.float32, device="cuda")
        seeds = torch.empty(n, dtype=torch.int32, device="cuda")
        live = torch.empty(n, dtype=torch.int32, device="cuda")
        device.render_device(cam, nx, ny, spp, depth, out.data_ptr(), stream=s, seed_ptr=seeds.data_ptr(),
                             live_ptr=live.data_ptr())
        torch.cuda.synchronize()
        rgb = out[:, :3].cpu().numpy()
        sd, lv = seeds.cpu().numpy().view(np.uint32), live.cpu().numpy().view(np.uint32)
        assert sha256_u32(sd) == bytes(g["seed_sha256"]), "final RNG states differ"
        assert sha256_u32(lv) == bytes(g["live_sha256"]), "live-bounce counts differ"
        assert int(lv.astype(np.uint64).sum()) == int(g["live_sum"])
    else:
        ent, pix = sh.tile_entries(nx, ny, 0, 1)
        n_tiles = -(-nx // 16) * -(-ny // 16)
        out = torch.empty((256 * n_tiles, 4), dtype=torch.float32, device="cuda")
        device.render_tiles_device(cam, nx, ny, spp, depth, out.data_ptr(), 0, 1, stream=s)
        torch.cuda.synchronize()
        rgb = np.empty((n, 3), np.float32)
        rgb[pix] = out[:, :3].cpu().numpy()[ent]
    nan = np.flatnonzero(np.isnan(rgb).any(1))
    assert np.array_equal(nan, g["nan_pixels"]), f"NaN pixels: {nan.size} vs {g['nan_pixels'].size}"
    assert canonical_rgb_sha256(rgb) == bytes(g["rgb_sha256"]), (
        f"rgb sums differ: channel sums {np.nansum(rgb.astype(np.float64), 0)} vs {g['rgb_sum']}")


C5_DIGESTS = [n for n in ("c5_shard3_full_digest", "c5_shard3_band_digest")
              if os.path.exists(os.path.join(GOLD, n + ".npz"))][:1]  # the whole canvas when generated


@pytest.mark.skipif(not C5_DIGESTS, reason="no C5 share digest generated (tools/make_golden_digest.py)")
@pytest.mark.parametrize("name", C5_DIGESTS)
def test_c5_rank_share_whole_canvas_digest(device, tables_on, name):
    """Rank 3 of 8's share of the C5 frame (3840x2160, 2048 of 16384 spp on
    the derived stream seed = pixel + 3 * 8294400: what bench.py's rank 3
    renders per step at N = 8) against the oracle's digests over the
    fixture's pixels -- the whole canvas (1.7e10 samples), or its leading band
    of rows (`pixel_count`, tools/make_golden_digest.py --assemble-first) --:
    rgb sums (NaN canonical), NaN pixels, final seeds, live counts."""
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard as sh

    from _util import canonical_rgb_sha256, sha256_u32

    g = _load(name)
    device.set_cornell_box(int(g["variant"]))
    nx, ny, spp, depth, sb = int(g["nx"]), int(g["ny"]), int(g["spp"]), int(g["depth"]), int(g["seed_base"])
    b = sh.sample_batches(16384, 8, nx * ny)[3]
    assert (b.spp, b.seed_base) == (spp, sb)  # the bench's rank 3 of 8
    n = int(g.get("pixel_count", nx * ny))
    assert int(g.get("pixel_begin", 0)) == 0
    out = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    seeds = torch.empty(n, dtype=torch.int32, device="cuda")
    live = torch.empty(n, dtype=torch.int32, device="cuda")
    device.render_device(rtp.default_camera(), nx, ny, spp, depth, out.data_ptr(), pixel_count=n, seed_base=sb,
                         stream=torch.cuda.current_stream().cuda_stream, seed_ptr=seeds.data_ptr(),
                         live_ptr=live.data_ptr())
    torch.cuda.synchronize()
    rgb = out[:, :3].cpu().numpy()
    assert sha256_u32(seeds.cpu().numpy().view(np.uint32)) == bytes(g["seed_sha256"]), "final RNG states differ"
    assert sha256_u32(live.cpu().numpy().view(np.uint32)) == bytes(g["live_sha256"]), "live-bounce counts differ"
    assert np.array_equal(np.flatnonzero(np.isnan(rgb).any(1)), g["nan_pixels"])
    assert canonical_rgb_sha256(rgb) == bytes(g["rgb_sha256"]), "rgb sums differ"


C3_DIGESTS = [n for n in ("c3_full16_digest", "c3_band256_digest") if os.path.exists(os.path.join(GOLD, n + ".npz"))]


@pytest.mark.skipif(not C3_DIGESTS, reason="no C3 digest generated (tools/make_golden_digest.py)")
@pytest.mark.parametrize("name", C3_DIGESTS)
def test_c3_whole_canvas_digest(device, tables_on, name):
    """C3 (2048^2, 1000 spheres, depth 50) against the oracle's digests over
    the fixture's pixels: c3_full16_digest, the whole canvas at 16 spp (the
    oracle's full-spp frame would take ~8 h on the host); c3_band256_digest,
    a leading band of rows at the full 256 spp (`pixel_count`,
    tools/make_golden_digest.py --assemble-first); c3_subset4k covers 4096
    scattered pixels at 256.  Every pixel goes through the sphere-BVH walk on
    the work-stealing schedule: rgb sums (NaN canonical), NaN pixels, final
    seeds, live counts."""
    import torch

    import raytracingtherestofyourlife_amd as rtp

    from _util import canonical_rgb_sha256, sha256_u32

    g = _load(name)
    device.set_cornell_box(int(g["variant"]))
    nx, ny, spp, depth = int(g["nx"]), int(g["ny"]), int(g["spp"]), int(g["depth"])
    n = int(g["pixel_count"])
    assert int(g.get("pixel_begin", 0)) == 0 and int(g["seed_base"]) == 0 and 0 < n <= nx * ny
    out = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    seeds = torch.empty(n, dtype=torch.int32, device="cuda")
    live = torch.empty(n, dtype=torch.int32, device="cuda")
    device.render_device(rtp.default_camera(), nx, ny, spp, depth, out.data_ptr(), pixel_count=n,
                         stream=torch.cuda.current_stream().cuda_stream, seed_ptr=seeds.data_ptr(),
                         live_ptr=live.data_ptr())
    torch.cuda.synchronize()
    rgb = out[:, :3].cpu().numpy()
    assert sha256_u32(seeds.cpu().numpy().view(np.uint32)) == bytes(g["seed_sha256"]), "final RNG states differ"
    lv = live.cpu().numpy().view(np.uint32)
    assert sha256_u32(lv) == bytes(g["live_sha256"]), "live-bounce counts differ"
    assert int(lv.astype(np.uint64).sum()) == int(g["live_sum"])
    assert np.array_equal(np.flatnonzero(np.isnan(rgb).any(1)), g["nan_pixels"])
    assert canonical_rgb_sha256(rgb) == bytes(g["rgb_sha256"]), (
        f"rgb sums differ: channel sums {np.nansum(rgb.astype(np.float64), 0)} vs {g['rgb_sum']}")
