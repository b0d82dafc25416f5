"""Multi-GPU decomposition (raytracingtherestofyourlife_amd/shard.py) on CPU:
world-size-2 gloo groups, the oracle standing in for each rank's device
render.  Tile sharding + one sum reduce must reproduce the unsharded image
bit-for-bit; the sample-batch schedule must equal its per-shard renders summed."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NX, NY, SPP, DEPTH, VARIANT = 48, 32, 6, 8, 1  # variant 1: NaN-heavy scene (NaN must survive the reduce)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_render():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, ROOT)
    import oracle_ctypes as oc

    sc, cam = oc.cornell_box(VARIANT), oc.camera_setup(NX, NY)

    def render(ids, spp, seed_base):
        if ids is None:
            ids = np.arange(NX * NY, dtype=np.int64)
        return oc.render_pixels(sc, cam, NX, NY, spp, DEPTH, ids, seed_base=seed_base, nthreads=1)[0]

    return render


def _worker(rank, world, port, mode, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from raytracingtherestofyourlife_amd import shard

    canvas = torch.zeros((NX * NY, 4), dtype=torch.float32)
    render = _oracle_render()
    if mode == "tiles":
        shard.render_tile_shard(render, canvas, NX, NY, SPP, rank, world)
    else:
        shard.render_sample_shard(render, canvas, NX * NY, SPP, rank, world)
    shard.reduce_canvas(canvas, dist)
    if rank == 0:
        np.save(out_path, canvas.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _run(mode, tmp_path, world=2):
    out = str(tmp_path / f"{mode}.npy")
    mp.start_processes(_worker, args=(world, _free_port(), mode, out), nprocs=world, join=True, start_method="spawn")
    return np.load(out)


def _same(a, b):
    return bool(((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))).all())


def test_tile_plan_covers_every_pixel_once():
    from raytracingtherestofyourlife_amd import shard

    for world in (1, 2, 3, 4, 8):
        ids = np.concatenate([shard.tile_pixels(800, 1600, r, world) for r in range(world)])
        assert ids.size == 800 * 1600 and np.array_equal(np.sort(ids), np.arange(800 * 1600))
        sizes = [shard.tile_pixels(800, 1600, r, world).size for r in range(world)]
        assert max(sizes) - min(sizes) <= 256  # at most one tile apart
    # canvases that are not a multiple of the tile (C4: 1080 rows = 67.5 tiles): edge tiles are clipped
    for nx, ny, world in ((1920, 1080, 8), (100, 64, 2), (17, 33, 3)):
        parts = [shard.tile_pixels(nx, ny, r, world) for r in range(world)]
        ids = np.concatenate(parts)
        assert np.array_equal(np.sort(ids), np.arange(nx * ny))
    with pytest.raises(ValueError):
        shard.tile_pixels(0, 64, 0, 2)
    with pytest.raises(ValueError):
        shard.tile_pixels(64, 64, 2, 2)


def test_tile_entries_match_the_kernel_layout():
    """rtp_render_tiles_device renders every owned tile whole: entry 256 q + e
    is pixel (16 tx + e % 16, 16 ty + e // 16) of the q-th owned tile.
    tile_entries picks the entries inside the canvas, in tile_pixels order."""
    from raytracingtherestofyourlife_amd import shard

    for nx, ny, world in ((1920, 1080, 8), (100, 64, 2), (17, 33, 3), (64, 48, 1)):
        tx, ty = -(-nx // 16), -(-ny // 16)
        for r in range(world):
            ent, pix = shard.tile_entries(nx, ny, r, world)
            assert np.array_equal(pix, shard.tile_pixels(nx, ny, r, world))
            owned = np.arange(tx * ty)[r::world]
            q, e = np.divmod(ent, 256)
            ox, oy = owned[q] % tx, owned[q] // tx
            assert np.array_equal(pix, (oy * 16 + e // 16) * nx + ox * 16 + e % 16)
            assert ent.size == 0 or ent.max() < 256 * owned.size
            if nx % 16 == 0 and ny % 16 == 0:
                assert np.array_equal(ent, np.arange(256 * owned.size))
    ent, pix = shard.tile_entries(40, 20, 7, 8)  # 6 tiles, 8 ranks: rank 7 owns none
    assert ent.size == 0 and pix.size == 0
    with pytest.raises(ValueError):
        shard.tile_entries(64, 64, 2, 2)


def test_sample_batches_partition():
    from raytracingtherestofyourlife_amd import shard

    b = shard.sample_batches(16384, 8, 3840 * 2160)
    assert sum(x.spp for x in b) == 16384 and {x.spp for x in b} == {2048}
    assert [x.seed_base for x in b] == [(k * 3840 * 2160) & 0xFFFFFFFF for k in range(8)]
    b = shard.sample_batches(10, 4, 7)
    assert [x.spp for x in b] == [3, 3, 2, 2]
    with pytest.raises(ValueError):
        shard.sample_batches(2, 4, 7)


def test_tile_shards_reduce_to_unsharded_image(tmp_path):
    got = _run("tiles", tmp_path)
    want = _oracle_render()(None, SPP, 0)
    assert np.isnan(want[:, :3]).any()  # the reduce must carry NaN pixels through
    assert _same(got[:, :3], want[:, :3])


def test_sample_shards_reduce_to_summed_shards(tmp_path):
    from raytracingtherestofyourlife_amd import shard

    got = _run("samples", tmp_path)
    render = _oracle_render()
    parts = [render(None, b.spp, b.seed_base) for b in shard.sample_batches(SPP, 2, NX * NY)]
    want = parts[0] + parts[1]
    assert _same(got[:, :3], want[:, :3])


def _overlap_worker(rank, world, port, overlap, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from raytracingtherestofyourlife_amd import shard

    n = 64
    canvas = torch.zeros((n, 4), dtype=torch.float32)
    red = shard.OverlappedCanvasReduce(canvas, dist, overlap=overlap)
    ids = torch.arange(rank, n, world)
    last = None
    for step in range(5):
        part = torch.full((ids.numel(), 4), float(100 * step + rank + 1))
        last = red.step(ids, part)
    red.drain()
    if rank == 0:
        np.save(out_path, last.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_overlapped_canvas_reduce(tmp_path, overlap):
    """bench.py's per-step reduce, async on two alternating canvases (the
    RCCL path, here with gloo's async reduce) or synchronous on one: rank 0
    ends with the last step's entries of every rank, nothing left over from
    earlier steps."""
    world = 2
    out = str(tmp_path / "ov.npy")
    mp.start_processes(_overlap_worker, args=(world, _free_port(), overlap, out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    want = np.zeros((64, 4), np.float32)
    for r in range(world):
        want[r::world] = 100 * 4 + r + 1
    assert np.array_equal(got, want)


def _overlap_samples_worker(rank, world, port, overlap, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from raytracingtherestofyourlife_amd import shard

    render = _oracle_render()
    b = shard.sample_batches(SPP, world, NX * NY)[rank]
    part = torch.from_numpy(render(None, b.spp, b.seed_base))
    canvas = torch.zeros((NX * NY, 4), dtype=torch.float32)
    red = shard.OverlappedCanvasReduce(canvas, dist, overlap=overlap)
    last = None
    for step in range(3):  # bench.py's C5 steps: the rank's whole-canvas sample batch, one reduce each
        last = red.step(None, part)
    red.drain()
    if rank == 0:
        np.save(out_path, last.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_overlapped_reduce_of_sample_batches(tmp_path, overlap):
    """bench.py's C5 path (--workload c5, N > 1) on CPU: each rank's sample
    batch of every pixel (seed_base k*N, the oracle standing in for the
    device) goes through shard.OverlappedCanvasReduce as a whole canvas
    (ids None) for several steps; rank 0 ends with the shards' sum, NaN
    pixels carried through."""
    from raytracingtherestofyourlife_amd import shard

    world = 2
    out = str(tmp_path / "ovs.npy")
    mp.start_processes(_overlap_samples_worker, args=(world, _free_port(), overlap, out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    render = _oracle_render()
    parts = [render(None, b.spp, b.seed_base) for b in shard.sample_batches(SPP, world, NX * NY)]
    want = parts[0] + parts[1]
    assert np.isnan(want[:, :3]).any()
    assert _same(got[:, :3], want[:, :3])


def _tree_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from raytracingtherestofyourlife_amd import shard

    buf = torch.from_numpy(_tree_parts(world)[rank].copy())
    shard.tree_reduce_(dist, buf, torch.empty_like(buf), rank, world)
    if rank == 0:
        np.save(out_path, buf.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _tree_parts(world):
    # magnitudes spread over many binades: float32 sums of more than two of
    # them depend on the association
    rng = np.random.default_rng(11)
    return [(rng.standard_normal((256, 4)) * 10.0 ** rng.integers(-3, 4, (256, 4))).astype(np.float32)
            for _ in range(world)]


@pytest.mark.parametrize("world", [2, 3, 4, 5])
def test_tree_reduce_fixed_association(tmp_path, world):
    """shard.tree_reduce_ (bench.py's and render_dist's framebuffer sum) over
    gloo: rank 0 ends with the pairwise-tree sum ((s0 + s1) + (s2 + s3)) + ...
    bit for bit (shard.tree_sum, the checker's side), whatever the world size,
    including a rank left without a partner."""
    from raytracingtherestofyourlife_amd import shard

    out = str(tmp_path / "tree.npy")
    mp.start_processes(_tree_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    got = np.load(out)
    parts = _tree_parts(world)
    want = shard.tree_sum(parts)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    if world >= 4:  # (three ranks: (s0 + s1) + s2 IS rank order) the test data tells the associations apart
        chain = parts[0].copy()
        for p in parts[1:]:
            chain = chain + p
        assert not np.array_equal(chain.view(np.uint32), want.view(np.uint32))


def test_tree_sum_matches_bench_pairwise_tree():
    import bench
    from raytracingtherestofyourlife_amd import shard

    for world in (3, 4, 6, 8):
        parts = _tree_parts(world)
        assert np.array_equal(bench.association_sums(parts)["pairwise_tree"], shard.tree_sum(parts))
    s = _tree_parts(6)
    want = ((s[0] + s[1]) + (s[2] + s[3])) + (s[4] + s[5])
    assert np.array_equal(shard.tree_sum(s).view(np.uint32), want.view(np.uint32))
