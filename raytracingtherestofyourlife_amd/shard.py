"""Multi-GPU decomposition of the render, one process per GPU.

Pixels are independent (own seed = pixel index, own sequential S x D stream,
MapperPathTracer.cxx:265-267), so the path shards with no data exchange until
the framebuffer sum:

* image tiles (C2/C4): 16x16 tiles, tile t -> rank t mod G (static,
  interleaved so every rank gets the same mix of cheap and expensive image
  regions).  Each rank renders its pixel list into a zeroed canvas; ONE
  reduce(sum) of the float4 canvas to rank 0.  Bit-exact: x + 0 == x and
  NaN / Inf pass through the sum unchanged.
* sample batches (C5): rank k renders S_k samples of every pixel with
  seed = pixel + k*N (seed_base = k*N), then the same reduce.  A Wang-hash
  stream has no jump-ahead and a pixel's sample-s state depends on every
  earlier sample's variable draw count, so this is a documented derived
  stream, exact against the oracle run on the same schedule.

The render itself is a callback so the planner and the reduce are testable
on CPU (gloo) with the oracle standing in for the device.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import numpy as np

TILE = 16


def tile_pixels(nx: int, ny: int, rank: int, world: int, tile: int = TILE) -> np.ndarray:
    """Pixel ids (int64, j*nx + i) of the tiles owned by `rank`; each tile in
    row-major order, so a 64-lane wave covers a 16x4 block.  Tiles on the
    right and top edges are clipped to the canvas (1080 rows = 67.5 tiles)."""
    if nx <= 0 or ny <= 0:
        raise ValueError("empty canvas")
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    tx, ty = -(-nx // tile), -(-ny // tile)
    tiles = np.arange(tx * ty)
    mine = tiles[tiles % world == rank]
    oy, ox = np.divmod(mine, tx)
    ly, lx = np.divmod(np.arange(tile * tile), tile)
    rows = (oy[:, None] * tile + ly[None, :]).astype(np.int64)
    cols = (ox[:, None] * tile + lx[None, :]).astype(np.int64)
    keep = (rows < ny) & (cols < nx)
    return (rows * nx + cols)[keep]


def tile_entries(nx: int, ny: int, rank: int, world: int, tile: int = TILE) -> tuple[np.ndarray, np.ndarray]:
    """rtp_render_tiles_device's output layout: it renders the rank's tiles
    whole (256 entries each, clipped edge tiles included), so its output has
    256 * (tiles owned) entries.  Returns (entries, pixels): the indices of the
    entries that lie inside the canvas and their pixel ids -- `pixels` equals
    tile_pixels(nx, ny, rank, world), and out[entries] is its render."""
    if nx <= 0 or ny <= 0:
        raise ValueError("empty canvas")
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    tx, ty = -(-nx // tile), -(-ny // tile)
    tiles = np.arange(tx * ty)
    mine = tiles[tiles % world == rank]
    oy, ox = np.divmod(mine, tx)
    ly, lx = np.divmod(np.arange(tile * tile), tile)
    rows = (oy[:, None] * tile + ly[None, :]).astype(np.int64)
    cols = (ox[:, None] * tile + lx[None, :]).astype(np.int64)
    keep = ((rows < ny) & (cols < nx)).reshape(-1)
    return np.flatnonzero(keep).astype(np.int64), (rows * nx + cols).reshape(-1)[keep]


@dataclass(frozen=True)
class SampleBatch:
    rank: int
    spp: int        # samples this rank renders per pixel
    seed_base: int  # seed = pixel + seed_base (mod 2^32)


def sample_batches(spp: int, world: int, npix: int) -> list[SampleBatch]:
    """Split spp over `world` ranks (the first spp % world ranks take one more)."""
    if spp < world:
        raise ValueError("fewer samples than ranks")
    base, extra = divmod(spp, world)
    return [SampleBatch(k, base + (1 if k < extra else 0), (k * npix) & 0xFFFFFFFF) for k in range(world)]


# render callbacks: (pixel_ids or None for all, spp, seed_base) -> float32 [n, 4] RGBA sums
RenderFn = Callable[[np.ndarray | None, int, int], "np.ndarray"]


def render_tile_shard(render: RenderFn, canvas, nx: int, ny: int, spp: int, rank: int, world: int):
    """This rank's tiles into `canvas` (float32 [nx*ny, 4], numpy or torch),
    zero elsewhere.  Returns the canvas."""
    ids = tile_pixels(nx, ny, rank, world)
    part = render(ids, spp, 0)
    canvas[...] = 0
    _scatter(canvas, ids, part)
    return canvas


def render_sample_shard(render: RenderFn, canvas, npix: int, spp: int, rank: int, world: int):
    """This rank's sample batch of every pixel into `canvas`."""
    b = sample_batches(spp, world, npix)[rank]
    canvas[...] = _as_like(canvas, render(None, b.spp, b.seed_base))
    return canvas


def reduce_canvas(canvas, dist) -> None:
    """The one collective: sum the float4 canvases onto rank 0."""
    if dist.get_world_size() > 1:
        dist.reduce(canvas, dst=0, op=dist.ReduceOp.SUM)


class OverlappedCanvasReduce:
    """The per-step canvas reduce of bench.py, overlapped with the next
    step: the rank's entries are scattered into one of two canvases, whose
    reduce (async) runs while the next step renders; a canvas is reused only
    after its reduce has been waited on.  overlap=False: one canvas, a
    synchronous reduce (gloo reduces host tensors: `host_copy` moves a device
    canvas through the host).  force: run the collective even on one rank
    (a world-size-1 RCCL group exercises the same calls on a one-GPU box)."""

    def __init__(self, canvas, dist, overlap: bool, host_copy: bool = False, force: bool = False):
        import torch

        self.dist, self.overlap, self.host_copy = dist, overlap, host_copy
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.collective = dist.is_initialized() and (self.world > 1 or force)
        self.canvases = [canvas, torch.zeros_like(canvas)] if overlap and self.collective else [canvas]
        self.pending = [None] * len(self.canvases)
        self.steps = 0

    def step(self, ids, part):
        """Zero the next canvas, scatter `part` at `ids`, start its reduce;
        returns that canvas (rank 0 holds the sum once drained)."""
        slot = self.steps % len(self.canvases)
        self.steps += 1
        if self.pending[slot] is not None:
            self.pending[slot].wait()
            self.pending[slot] = None
        c = self.canvases[slot]
        c.zero_()
        c.index_copy_(0, ids, part)
        if self.collective:
            if len(self.canvases) > 1:
                self.pending[slot] = self.dist.reduce(c, dst=0, op=self.dist.ReduceOp.SUM, async_op=True)
            elif self.host_copy:
                host = c.cpu()
                self.dist.reduce(host, dst=0, op=self.dist.ReduceOp.SUM)
                if self.rank == 0:
                    c.copy_(host)
            else:
                self.dist.reduce(c, dst=0, op=self.dist.ReduceOp.SUM)
        return c

    def drain(self) -> None:
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None


def _as_like(canvas, a):
    if isinstance(canvas, np.ndarray):
        return np.asarray(a, dtype=np.float32)
    import torch

    return torch.as_tensor(a, dtype=torch.float32, device=canvas.device)


def _scatter(canvas, ids, part) -> None:
    if isinstance(canvas, np.ndarray):
        canvas[ids] = part
    else:
        import torch

        idx = torch.as_tensor(ids, device=canvas.device)
        canvas.index_copy_(0, idx, _as_like(canvas, part))
