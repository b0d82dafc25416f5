"""Multi-GPU render of one image: one process per GPU,
RCCL over xGMI, the shard plans of shard.py.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m raytracingtherestofyourlife_amd.render_dist --nx 1920 --ny 1080 --spp 4096 --shard tiles
    ... --nx 3840 --ny 2160 --spp 16384 --shard samples --out c5.pnm

--shard tiles (BASELINE configs[3], C4): 16x16 tiles round-robin over the
    ranks; each rank renders its tiles (rtp_render_tiles_device: each entry's
    pixel computed in the kernel) into a zeroed canvas; one reduce(sum) to
    rank 0.  The image is
    bit-identical to a one-GPU render (x + 0 == x, NaN passes through).
--shard samples (configs[4], C5): rank k renders spp_k samples of every
    pixel from the derived stream seed = pixel + k*N (shard.sample_batches);
    the reduce sums the ranks' partial sums.  Exact against the oracle run on
    the same schedule; vs a one-GPU render it is a different (documented)
    random stream.

Rank 0 normalises the sum (NormalizeFunctor, main.cc:253-287), optionally
writes the PNM (save(), main.cc:325-384), and prints one JSON line: strong
scaling (the image's total work is fixed), Msamples/s of the whole job from
the slowest rank's wall time between two barriers.

--backend gloo --share-gpu rehearses the same code with every rank on device
0 and a host-side reduce (a one-GPU box).  --check makes rank 0 re-render the
reference and compare: bit-exact for tiles; for samples the ranks' shard
renders summed in the reduce's own association (shard.tree_reduce_'s
pairwise tree), bit for bit.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--nx", type=int, default=1920)
    ap.add_argument("--ny", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--variant", type=int, default=0, help="rtp_cornell_box variant (0: the reference scene)")
    ap.add_argument("--shard", choices=["tiles", "samples"], default="tiles")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl")
    ap.add_argument("--share-gpu", action="store_true")
    ap.add_argument("--out", default="", help="PNM path written by rank 0")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    from . import mapper, shard
    from .mapper import Device, default_camera

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = 0 if a.share_gpu else local
    torch.cuda.set_device(gpu)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    n = a.nx * a.ny
    dev = Device(gpu)
    dev.set_cornell_box(a.variant)
    cam = default_camera()
    stream = torch.cuda.current_stream()
    canvas = torch.zeros((n, 4), dtype=torch.float32, device="cuda")

    if a.shard == "tiles":
        # the rank's tiles through the tile instance (each entry's pixel
        # computed in the kernel, clipped edge tiles rendered whole); the
        # entries inside the canvas go to their pixels (shard.tile_entries)
        ent_np, ids_np = shard.tile_entries(a.nx, a.ny, rank, world)
        ids = torch.from_numpy(ids_np).cuda()
        ent = torch.from_numpy(ent_np).cuda()
        n_tiles = len(range(rank, -(-a.nx // shard.TILE) * -(-a.ny // shard.TILE), world))
        part = torch.empty((shard.TILE * shard.TILE * max(n_tiles, 1), 4), dtype=torch.float32, device="cuda")
        spp_mine, seed_base = a.spp, 0
    else:
        b = shard.sample_batches(a.spp, world, n)[rank]
        ids, part = None, canvas
        spp_mine, seed_base = b.spp, b.seed_base

    def reduce():  # the fixed-association tree sum (shard.tree_reduce_)
        if world == 1:
            return
        if a.backend == "nccl":
            shard.tree_reduce_(dist, canvas, torch.empty_like(canvas), rank, world)
        else:
            host = canvas.cpu()
            shard.tree_reduce_(dist, host, torch.empty_like(host), rank, world)
            if rank == 0:
                canvas.copy_(host)

    # one-pixel warm-up: builds the device's RNG jump tables and scratch outside the timed region
    dev.render_device(cam, a.nx, a.ny, 1, a.depth, part.data_ptr(), pixel_count=1, stream=stream.cuda_stream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if ids is not None:
        st = dev.render_tiles_device(cam, a.nx, a.ny, spp_mine, a.depth, part.data_ptr(), rank, world,
                                     stream=stream.cuda_stream, timed=True)
        canvas.index_copy_(0, ids, part.index_select(0, ent))
    else:
        st = dev.render_device(cam, a.nx, a.ny, spp_mine, a.depth, part.data_ptr(), pixel_count=n, seed_base=seed_base,
                               stream=stream.cuda_stream, timed=True)
    reduce()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, st.kernel_ms], dtype=torch.float64,
                         device="cuda" if a.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kmax = float(t[0].item()), float(t[1].item())
    else:
        kmax = st.kernel_ms

    if rank == 0:
        line = {"metric": "Msamples/s (whole job, strong scaling)", "value": round(n * a.spp / elapsed / 1e6, 3),
                "n_gpus": world, "shard": a.shard, "backend": a.backend, "seconds": round(elapsed, 4),
                "max_kernel_ms": round(kmax, 3), "config": {"nx": a.nx, "ny": a.ny, "spp": a.spp, "depth": a.depth,
                                                             "variant": a.variant}}
        if a.check:
            line["check"] = _check(a, dev, cam, canvas, world, stream)
        img = canvas.cpu().numpy()
        if a.out:
            mapper.normalize(img, a.spp)
            mapper.save_pnm(a.out, img, a.nx, a.ny)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _check(a, dev, cam, canvas, world, stream) -> bool:
    """Rank 0: the reduced canvas against a one-process render of the same plan."""
    import torch

    from . import shard

    n = a.nx * a.ny
    got = canvas[:, :3].cpu().numpy()
    if a.shard == "tiles":
        full = torch.empty((n, 4), dtype=torch.float32, device="cuda")
        dev.render_device(cam, a.nx, a.ny, a.spp, a.depth, full.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize()
        want = full[:, :3].cpu().numpy()
        return bool(((got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))).all())
    one = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    parts = []
    for b in shard.sample_batches(a.spp, world, n):
        dev.render_device(cam, a.nx, a.ny, b.spp, a.depth, one.data_ptr(), seed_base=b.seed_base,
                          stream=stream.cuda_stream)
        torch.cuda.synchronize()
        parts.append(one[:, :3].cpu().numpy())
    want = shard.tree_sum(parts)  # the reduce's own association
    return bool(((got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))).all())


if __name__ == "__main__":
    sys.exit(main())
