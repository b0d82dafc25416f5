"""Cost-grouped wave plans (development experiment).

A pixel's samples are one sequential chain, so a wave whose pixels have very
different path lengths ends with a few lanes running the long chains (the
"tail").  Grouping pixels of similar cost into the same wave -- expensive
pixels 64 to a wave, cheap ones up to 128 -- keeps every lane busy to the
end.  This tool times, on rank R's share of the C2 tile deal:
  base   the pixel-list render in deal order (rtp_render_device);
  oracle a plan from the exact per-pixel live-bounce counts of the base render
         (an upper bound: the cost is known in advance);
  est    a plan from a cheap pre-pass (P spp on a different seed stream),
         smoothed over 5x5 pixels;
and checks that every planned render equals the base render bit for bit.

    python tools/plan_experiment.py [--world N --rank R] [--pre-spp 16] [--ff 1.0]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402
from raytracingtherestofyourlife_amd import shard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=800)
ap.add_argument("--ny", type=int, default=800)
ap.add_argument("--spp", type=int, default=1000)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--pre-spp", type=int, default=16)
ap.add_argument("--ff", type=float, default=1.0, help="per-sample overhead in bounce steps (fast-forward, refill)")
ap.add_argument("--resident", type=int, default=5120)
ap.add_argument("--cap", type=int, default=128, help="most pixels per wave (64: grouping only, no packing)")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

dev = rtp.Device(0)
dev.set_cornell_box(0)
dev.set_ff_tables("on")
cam = rtp.default_camera()
ids_np = shard.tile_pixels(a.nx, a.ny, a.rank, a.world)
n = ids_np.size
ids = torch.from_numpy(ids_np).cuda()
s = torch.cuda.current_stream().cuda_stream


def render_list(pix, spp, seed_base=0, live=None, out=None):
    out = torch.zeros((pix.numel(), 4), dtype=torch.float32, device="cuda") if out is None else out
    st = dev.render_device(cam, a.nx, a.ny, spp, a.depth, out.data_ptr(), pixel_count=pix.numel(),
                           pixel_ids_ptr=pix.data_ptr(), seed_base=seed_base, stream=s,
                           live_ptr=0 if live is None else live.data_ptr(), timed=True)
    return out, st.kernel_ms


def plan(cost):
    """cost: expected chain length (bounce steps) per entry -> (order, wave_begin)."""
    order = np.argsort(-cost, kind="stable")
    c = cost[order]
    T = max(c.max(), c.sum() / (64 * a.resident))
    w = np.maximum(c / (64 * T), 1 / (a.cap - 0.5))
    start = np.concatenate([[0.0], np.cumsum(w)[:-1]])
    wid = np.floor(start).astype(np.int64)
    nw = int(wid[-1]) + 1
    wb = np.searchsorted(wid, np.arange(nw + 1), side="left").astype(np.int32)
    assert wb[-1] == n and (np.diff(wb) <= a.cap).all() and (np.diff(wb) > 0).all()
    return order, wb, T


def run_plan(order, wb):
    pix = torch.from_numpy(ids_np[order]).cuda()
    wbt = torch.from_numpy(wb).cuda()
    out = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    best = 1e9
    for _ in range(a.reps):
        st = dev.render_planned_device(cam, a.nx, a.ny, a.spp, a.depth, out.data_ptr(), n, wbt.data_ptr(),
                                       len(wb) - 1, pixel_ids_ptr=pix.data_ptr(), stream=s, timed=True)
        best = min(best, st.kernel_ms)
    back = np.empty((n, 4), np.float32)
    back[order] = out.cpu().numpy()
    return back, best


live = torch.zeros(n, dtype=torch.int32, device="cuda")
base_ms = 1e9
for _ in range(a.reps):
    out, ms = render_list(ids, a.spp, live=live)
    base_ms = min(base_ms, ms)
base = out.cpu().numpy()
L = live.cpu().numpy().astype(np.float64)
res = {"world": a.world, "rank": a.rank, "pixels": n, "base_ms": round(base_ms, 2)}


def same(x):
    return bool(((x[:, :3].view(np.uint32) == base[:, :3].view(np.uint32)) |
                 (np.isnan(x[:, :3]) & np.isnan(base[:, :3]))).all())


order, wb, T = plan(L + a.spp * a.ff)
got, ms = run_plan(order, wb)
res["oracle"] = {"ms": round(ms, 2), "waves": len(wb) - 1, "T": round(T, 1), "equal": same(got)}

t = time.perf_counter()
pre_live = torch.zeros(n, dtype=torch.int32, device="cuda")
_, pre_ms = render_list(ids, a.pre_spp, seed_base=0x9E3779B9, live=pre_live)
est = np.zeros(a.nx * a.ny)
est[ids_np] = pre_live.cpu().numpy()
img = est.reshape(a.ny, a.nx)
mask = np.zeros_like(img)
mask.reshape(-1)[ids_np] = 1
k = 2
pad = lambda x: np.pad(x, k, mode="edge")
acc = sum(np.roll(np.roll(pad(img), dy, 0), dx, 1) for dy in range(-k, k + 1) for dx in range(-k, k + 1))[k:-k, k:-k]
cnt = sum(np.roll(np.roll(pad(mask), dy, 0), dx, 1) for dy in range(-k, k + 1) for dx in range(-k, k + 1))[k:-k, k:-k]
sm = (acc / np.maximum(cnt, 1)).reshape(-1)[ids_np] * (a.spp / a.pre_spp)
host_ms = (time.perf_counter() - t) * 1e3 - pre_ms
order, wb, T = plan(sm + a.spp * a.ff)
got, ms = run_plan(order, wb)
res["est"] = {"ms": round(ms, 2), "pre_ms": round(pre_ms, 2), "host_plan_ms": round(host_ms, 1),
              "waves": len(wb) - 1, "T": round(T, 1), "equal": same(got),
              "corr_est_vs_true": round(float(np.corrcoef(sm, L)[0, 1]), 3)}
print(json.dumps(res), flush=True)
