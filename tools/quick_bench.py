"""Quick C2-geometry timing of the HIP render kernel (development tool)."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import raytracingtherestofyourlife_amd as rtp

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=800)
ap.add_argument("--ny", type=int, default=800)
ap.add_argument("--spp", type=int, default=50)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--variant", type=int, default=0)
ap.add_argument("--tiles", action="store_true", help="the tile-deal instance bench.py runs (rank 0 of 1), no live counters")
ap.add_argument("--world", type=int, default=1, help="--tiles: the deal over this many ranks")
ap.add_argument("--rank", type=int, default=0, help="--tiles: the rank whose share is rendered")
ap.add_argument("--ff-tables", default="on", choices=["on", "auto", "off"], help="RNG jump-table policy")
ap.add_argument("--list-tiles", action="store_true", help="the pixel-list path over the tile deal's order")
ap.add_argument("--list-contig", action="store_true", help="the pixel-list path over the contiguous order")
ap.add_argument("--share", action="store_true",
                help="the pixel-list path over rank --rank's tiles of the --world deal (shard.tile_pixels: any canvas, "
                     "clipped edge tiles; bench.py's path for canvases that are not whole tiles, e.g. C4's 1080 rows)")
ap.add_argument("--seed-base", type=int, default=0)
a = ap.parse_args()
ids = None
if a.share:
    from raytracingtherestofyourlife_amd import shard
    ids = torch.from_numpy(shard.tile_pixels(a.nx, a.ny, a.rank, a.world)).cuda()
if a.list_contig:
    ids = torch.arange(a.nx * a.ny, dtype=torch.int64, device="cuda")
if a.list_tiles:
    from raytracingtherestofyourlife_amd import shard
    ids = torch.from_numpy(shard.tile_pixels(a.nx, a.ny, 0, 1)).cuda()
dev = rtp.Device(0)
dev.set_cornell_box(a.variant)
dev.set_ff_tables(a.ff_tables)
cam = rtp.default_camera()
n = a.nx * a.ny if ids is None else int(ids.numel())
# --tiles renders the rank's tiles whole (clipped edge tiles included)
n_out = 256 * len(range(a.rank, -(-a.nx // 16) * -(-a.ny // 16), a.world)) if a.tiles else n
out = torch.zeros((max(n, n_out), 4), dtype=torch.float32, device="cuda")
live = torch.zeros(n, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for r in range(a.reps):
    t = time.time()
    if ids is not None:
        st = dev.render_device(cam, a.nx, a.ny, a.spp, a.depth, out.data_ptr(), pixel_count=n, pixel_ids_ptr=ids.data_ptr(),
                               stream=s, live_ptr=live.data_ptr(), timed=True, seed_base=a.seed_base)
    elif a.tiles:
        st = dev.render_tiles_device(cam, a.nx, a.ny, a.spp, a.depth, out.data_ptr(), a.rank, a.world, stream=s,
                                     timed=True)
    else:
        st = dev.render_device(cam, a.nx, a.ny, a.spp, a.depth, out.data_ptr(), stream=s, live_ptr=live.data_ptr(),
                               timed=True, seed_base=a.seed_base)
    torch.cuda.synchronize()
    wall = time.time() - t
    L = live.to(torch.int64).sum().item() / (n * a.spp)
    Lp = (live.to(torch.float64) / a.spp).cpu().numpy()
    nr = n  # (--share: n is already the rank's pixels)
    if a.tiles:  # the rank's pixels inside the canvas
        from raytracingtherestofyourlife_amd import shard as _sh
        nr = int(_sh.tile_pixels(a.nx, a.ny, a.rank, a.world).size)
    print(json.dumps(dict(rep=r, npix=nr, kernel_ms=st.kernel_ms, wall_s=wall, msamples_per_s=nr * a.spp / (st.kernel_ms / 1e3) / 1e6,
                          live_per_sample=L, nan_px=int(torch.isnan(out[:, :3]).any(1).sum().item()),
                          L_pixel_pct={q: round(float(np.percentile(Lp, q)), 3) for q in (50, 90, 99, 99.9, 100)})), flush=True)
