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

The reduce (tree_reduce_) sums in ONE fixed association, the pairwise tree
((s0 + s1) + (s2 + s3)) + ..., by point-to-point sends.  A collective reduce
would leave the association of N > 2 float32 shards to the library: RCCL's
rings follow the node's xGMI topology and split the buffer over channels
with rings of their own, so the reduced bits would depend on the node.

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


def tree_reduce_(dist, buf, tmp, rank: int, world: int) -> None:
    """Sum every rank's `buf` into rank 0's `buf` in a fixed association, the
    pairwise tree ((s0 + s1) + (s2 + s3)) + ... (bench.association_sums
    "pairwise_tree"; a rank left without a partner passes its partial up
    unchanged).  Round j (step 2^j): a rank r = 0 mod 2^(j+1) receives rank
    r + 2^j's partial into `tmp` and adds it (IEEE addition commutes, so only
    the association is fixed); a rank r = 2^j mod 2^(j+1) sends its partial
    and is done.  log2(N) rounds of point-to-point transfers, each waiting
    only on higher ranks: no cycle.  `tmp`: same shape as `buf` (receiving
    ranks only).  Over RCCL the calls only enqueue: the current stream waits
    on each transfer on the device."""
    step = 1
    while step < world:
        if rank % (2 * step):
            dist.send(buf, dst=rank - step)
            return
        if rank + step < world:
            dist.recv(tmp, src=rank + step)
            buf.add_(tmp)
        step *= 2


def tree_sum(parts):
    """The float32 sum of the ranks' partials (rank order) in tree_reduce_'s
    association, on the host: the checker's side of the reduce."""
    lvl = [np.asarray(p, np.float32) for p in parts]
    while len(lvl) > 1:
        lvl = [lvl[i] + lvl[i + 1] if i + 1 < len(lvl) else lvl[i] for i in range(0, len(lvl), 2)]
    return lvl[0].copy()


def reduce_canvas(canvas, dist) -> None:
    """The framebuffer sum: the ranks' float4 canvases onto rank 0 (tree_reduce_)."""
    world = dist.get_world_size()
    if world > 1:
        tree_reduce_(dist, canvas, canvas.new_empty(canvas.shape), dist.get_rank(), world)


class OverlappedCanvasReduce:
    """The per-step canvas reduce of bench.py, overlapped with the next
    step: the rank's entries are scattered into one of two canvases, whose
    reduce (tree_reduce_) runs on a communication stream while the next step
    renders; a canvas is reused only after its reduce has finished (an event
    the render stream waits on, on the device).  Without overlap (host
    tensors; gloo): one canvas, a synchronous reduce (`host_copy` moves a
    device canvas through the host).  force: run the reduce's calls even on
    one rank (a world-size-1 group, where the tree has no transfers)."""

    def __init__(self, canvas, dist, overlap: bool, host_copy: bool = False, force: bool = False):
        import torch

        self.dist, self.host_copy = dist, host_copy
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.collective = dist.is_initialized() and (self.world > 1 or force)
        # the overlapped path needs device tensors (a stream of its own)
        self.overlap = overlap and self.collective and canvas.is_cuda and not host_copy
        self.canvases = [canvas, torch.zeros_like(canvas)] if self.overlap else [canvas]
        self.tmp = torch.empty_like(canvas) if self.collective and not host_copy else None
        self.stream = torch.cuda.Stream(device=canvas.device) if self.overlap else None
        self.pending = [None] * len(self.canvases)
        self.steps = 0

    def _wait(self, slot: int) -> None:
        import torch

        if self.pending[slot] is not None:
            torch.cuda.current_stream().wait_event(self.pending[slot])
            self.pending[slot] = None

    def step(self, ids, part):
        """Zero the next canvas, scatter `part` at `ids` (ids None: `part` is
        a whole canvas -- a sample batch of every pixel -- and is copied),
        start its reduce; returns that canvas (rank 0 holds the sum once
        drained)."""
        import torch

        slot = self.steps % len(self.canvases)
        self.steps += 1
        self._wait(slot)
        c = self.canvases[slot]
        if ids is None:
            c.copy_(part)
        else:
            c.zero_()
            c.index_copy_(0, ids, part)
        if self.collective:
            if self.overlap:
                self.stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.stream):
                    tree_reduce_(self.dist, c, self.tmp, self.rank, self.world)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                self.pending[slot] = ev
            elif self.host_copy:
                host = c.cpu()
                tree_reduce_(self.dist, host, torch.empty_like(host), self.rank, self.world)
                if self.rank == 0:
                    c.copy_(host)
            else:
                tree_reduce_(self.dist, c, self.tmp, self.rank, self.world)
        return c

    def drain(self) -> None:
        for i in range(len(self.pending)):
            self._wait(i)


def sample_shard_consistency(single: np.ndarray, shards: list, spp: int) -> dict:
    """Monte Carlo consistency of a sample-sharded image with the single-stream
    image of the same frame (SURVEY.md 8(e) C5 "statistical vs the unsharded
    reference"; shard.sample_batches).  single: the float32 [n, 4] sums of spp
    samples per pixel on the reference's stream (seed_base 0); shards: G
    arrays, each the sums of spp/G samples on its derived stream (seed_base
    k*n).  The two images are two independent estimates of each pixel's mean
    radiance, so their per-pixel difference D = (single - sum(shards)) / spp
    has mean 0 and variance 2 sigma^2 / spp, with sigma^2 the per-sample
    variance.  sigma^2 / (spp/G) is estimated per pixel from the spread of
    the G shard means (ddof 1), so Var(D) ~ 2 s^2 / G.  Pixels that are NaN in
    either image (a non-finite attenuation: the sum stays NaN, MapperPathTracer
    .cxx:350; NormalizeFunctor zeroes it) are counted, not compared.
    Returns: n (pixels compared), z_total (sum D / sqrt(sum Var D): ~N(0,1)),
    ratio (sum D^2 / sum Var D: ~1), outliers (fraction with |D| > 5 sd),
    norm_ratio (the same ratio after NormalizeFunctor, delta method:
    Var(sqrt m) ~ Var(m) / (4 m)), nan_single / nan_sharded."""
    G = len(shards)
    x = np.asarray(single, np.float64)[:, :3]
    ys = np.stack([np.asarray(s, np.float64)[:, :3] for s in shards])  # [G, n, 3]
    nan = np.isnan(x).any(1) | np.isnan(ys).any((0, 2))
    keep = ~nan
    x, ys = x[keep], ys[:, keep]
    mx = x / spp
    my = ys.sum(0) / spp
    means = ys / (spp / G)  # per-shard means
    var_d = 2.0 * means.var(0, ddof=1) / G  # [n, 3]
    d = mx - my
    live = var_d > 0
    z = np.zeros_like(d)
    z[live] = d[live] / np.sqrt(var_d[live])
    m = np.maximum(0.5 * (mx + my), 1e-12)
    nx_, ny_ = np.sqrt(mx), np.sqrt(my)
    return {
        "n": int(keep.sum()),
        "z_total": float(d[live].sum() / np.sqrt(var_d[live].sum())),
        "ratio": float((d[live] ** 2).sum() / var_d[live].sum()),
        "outliers": float((np.abs(z) > 5).mean()),
        "zero_var_nonzero_d": int(((~live) & (d != 0)).sum()),
        "norm_ratio": float(((nx_ - ny_)[live] ** 2).sum() / (var_d[live] / (4 * m[live])).sum()),
        "nan_single": int(np.isnan(np.asarray(single)[:, :3]).any(1).sum()),
        "nan_sharded": int(np.isnan(np.stack([np.asarray(s)[:, :3] for s in shards])).any((0, 2)).sum()),
    }


def sample_shard_ttest(single: np.ndarray, shards_sum: np.ndarray, spp: int, blocks: int = 256) -> dict:
    """Frame-level test that a sample-sharded image (shards_sum: the G shards'
    sums, spp samples per pixel in all) and the single-stream image of the
    same pixels estimate the same radiance, with no per-pixel variance
    estimate (the per-pixel one of sample_shard_consistency is unstable when
    few shards hold a rare light hit).  The pixels (in the given order) are
    cut into `blocks` groups; each group's mean difference of the per-pixel
    means is an independent, near-Gaussian draw with mean 0 under the null, so
    t = mean / (sd / sqrt(blocks)) per channel is Student-t with blocks - 1
    degrees of freedom.  Pixels NaN in either image are left out (counted).
    Returns t per channel, max |t|, the relative difference of the frame means
    per channel, and the counts."""
    x = np.asarray(single, np.float64)[:, :3] / spp
    y = np.asarray(shards_sum, np.float64)[:, :3] / spp
    keep = ~(np.isnan(x).any(1) | np.isnan(y).any(1))
    d = (x - y)[keep]
    B = max(2, min(blocks, d.shape[0] // 2))
    m = np.stack([g.mean(0) for g in np.array_split(d, B)])  # [B, 3]
    sd = m.std(0, ddof=1)
    t = np.where(sd > 0, m.mean(0) / np.where(sd > 0, sd, 1.0) * np.sqrt(B), 0.0)
    mx = x[keep].mean(0)
    rel = np.where(mx != 0, (y[keep].mean(0) - mx) / np.where(mx != 0, mx, 1.0), 0.0)
    return {"n": int(keep.sum()), "blocks": int(B), "t": [round(float(v), 3) for v in t],
            "t_max": float(np.abs(t).max()), "rel_diff_frame_mean": [float(v) for v in rel],
            "nan_single": int(np.isnan(x).any(1).sum()), "nan_sharded": int(np.isnan(y).any(1).sum())}


def ttest_consistent(st: dict, t_max: float = 4.5) -> bool:
    """sample_shard_ttest's verdict: every channel within t_max standard
    errors (Student-t, >= 64 blocks: |t| > 4.5 has p < 1e-4) and NaN pixel
    counts within Poisson noise of each other."""
    a, b = st["nan_single"], st["nan_sharded"]
    return bool(st["n"] > 0 and st["t_max"] < t_max and abs(a - b) <= 5 * np.sqrt(a + b) + 3)


def shards_consistent(st: dict) -> bool:
    """The frame-level bounds of tests/_util.assert_shards_consistent (the
    per-pixel outlier bound needs G >= 4 shards: with fewer the per-pixel
    variance estimate has too few degrees of freedom for a 5-sd test)."""
    if st["n"] <= 0 or abs(st["z_total"]) >= 4 or not 0.5 < st["ratio"] < 2.0 or not 0.3 < st["norm_ratio"] < 3.0:
        return False
    a, b = st["nan_single"], st["nan_sharded"]
    return bool(abs(a - b) <= 5 * np.sqrt(a + b) + 3)


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
