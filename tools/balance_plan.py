"""Cost-balanced wave plans for a full chip (development experiment).

At N = 1 the frame fills every resident wave and a wave's loop iterations
are ~1.1x its lane bound (its pixels' live bounces / 64), so the slowest wave
is the one that drew the most work.  This times planned launches
(rtp_render_planned_device) whose waves get equal work:
  random  pixels in a random order, 125 per wave (control: same instance);
  snake   pixels sorted by their live-bounce count (from a first render: the
          cost a renderer knows from its previous frame) and dealt to the
          waves boustrophedon (0..W-1, W-1..0, ...), so every wave gets the
          same mix of expensive and cheap pixels;
and the production tile-deal render, and checks the planned renders equal
the base render bit for bit.

    python tools/balance_plan.py [--reps 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=800)
ap.add_argument("--spp", type=int, default=1000)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--waves", type=int, default=5120)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

dev = rtp.Device(0)
dev.set_cornell_box(0)
dev.set_ff_tables("on")
cam = rtp.default_camera()
n = a.n * a.n
W = a.waves
s = torch.cuda.current_stream().cuda_stream
out = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
live = torch.zeros(n, dtype=torch.int32, device="cuda")
dev.render_device(cam, a.n, a.n, a.spp, a.depth, out.data_ptr(), stream=s, live_ptr=live.data_ptr())
torch.cuda.synchronize()
base = out.cpu().numpy().copy()
L = live.cpu().numpy().astype(np.int64)
res = {"pixels": n, "waves": W}


def best_of(fn):
    return round(min(fn() for _ in range(a.reps)), 2)


tiles = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
res["tiles_ms"] = best_of(lambda: dev.render_tiles_device(cam, a.n, a.n, a.spp, a.depth, tiles.data_ptr(), 0, 1,
                                                          stream=s, timed=True).kernel_ms)
res["list_ms"] = best_of(lambda: dev.render_device(cam, a.n, a.n, a.spp, a.depth, out.data_ptr(), stream=s,
                                                   timed=True).kernel_ms)


def run_plan(name, order):
    cnt = np.full(W, n // W, np.int64)
    cnt[: n - cnt.sum()] += 1
    wb = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
    pix = torch.from_numpy(order.astype(np.int64)).cuda()
    wbt = torch.from_numpy(wb).cuda()
    po = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    ms = best_of(lambda: dev.render_planned_device(cam, a.n, a.n, a.spp, a.depth, po.data_ptr(), n, wbt.data_ptr(), W,
                                                   pixel_ids_ptr=pix.data_ptr(), stream=s, timed=True).kernel_ms)
    back = np.empty((n, 4), np.float32)
    back[order] = po.cpu().numpy()
    eq = bool(((back[:, :3].view(np.uint32) == base[:, :3].view(np.uint32)) |
               (np.isnan(back[:, :3]) & np.isnan(base[:, :3]))).all())
    work = np.array([L[order[wb[w]:wb[w + 1]]].sum() / 64.0 for w in range(W)])
    chain = np.array([L[order[wb[w]:wb[w + 1]]].max() for w in range(W)])
    res[name] = {"ms": ms, "equal": eq, "lane_bound_max": round(float(work.max()), 1),
                 "lane_bound_p50": round(float(np.median(work)), 1), "chain_max": int(chain.max()),
                 "bound_max": round(float(np.maximum(work, chain).max()), 1)}


run_plan("random", np.random.default_rng(3).permutation(n))
srt = np.argsort(-L, kind="stable")
# boustrophedon deal: rank r goes to wave (r mod W) on even passes, W-1-(r mod W) on odd ones;
# the plan's entries are grouped by wave
r = np.arange(n)
p, q = r // W, r % W
wave = np.where(p % 2 == 0, q, W - 1 - q)
order = srt[np.argsort(wave, kind="stable")]
run_plan("snake", order)
# the production interleave (entry k -> wave k mod W) as a plan, for the instance's own cost
inter = np.argsort(np.arange(n) % W, kind="stable")
run_plan("interleave", inter)
print(json.dumps(res), flush=True)
