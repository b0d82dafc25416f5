"""How close each wave runs to its pixels' sample-chain floor (development tool).

A pixel's samples are one sequential RNG chain, and a sample with L live
depths takes L loop iterations of its wave, so a wave can never finish in
fewer iterations than the largest live-bounce count among its pixels (its
"chain").  With the pool's fair-share queue the critical pixel of a wave runs
almost without waiting; then the wave's iteration count is close to that
chain, and no redistribution of the other pixels (tail consolidation) can
shorten it.  This renders rank R's share of the frame with the statistics
build (RTP_DEBUG_STATS=1, per-wave iteration counts) and the per-pixel
live-bounce counters, and reports per wave: iterations / chain.

    python tools/chain_floor.py [--world N --rank R] [--spp 1000]
"""
import argparse
import json
import os
import sys

os.environ["RTP_DEBUG_STATS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402
from raytracingtherestofyourlife_amd import shard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=800)
ap.add_argument("--spp", type=int, default=1000)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--rank", type=int, default=0)
a = ap.parse_args()

dev = rtp.Device(0)
dev.set_cornell_box(0)
dev.set_ff_tables("on")
ids_np = shard.tile_pixels(a.n, a.n, a.rank, a.world) if a.world > 1 else None
npix = a.n * a.n if ids_np is None else ids_np.size
ids = None if ids_np is None else torch.from_numpy(ids_np).cuda()
out = torch.zeros((npix, 4), dtype=torch.float32, device="cuda")
live = torch.zeros(npix, dtype=torch.int32, device="cuda")
st = dev.render_device(rtp.default_camera(), a.n, a.n, a.spp, a.depth, out.data_ptr(), pixel_count=npix,
                       pixel_ids_ptr=0 if ids is None else ids.data_ptr(),
                       stream=torch.cuda.current_stream().cuda_stream, live_ptr=live.data_ptr(), timed=True)
rec = dev.debug_wave_records()
W = rec.shape[0]
L = live.cpu().numpy().astype(np.int64)
steps = rec[:, 0].astype(np.int64)
cycles = rec[:, 7].astype(np.float64)
k = np.arange(npix)
chain = np.zeros(W, np.int64)
np.maximum.at(chain, k % W, L)  # entry k belongs to wave k mod W (interleaved pool)
ratio = steps / np.maximum(chain, 1)
slow = int(np.argmax(cycles))
res = {
    "workload": f"{a.n}x{a.n}x{a.spp} depth {a.depth}, rank {a.rank}/{a.world}: {npix} px, {W} waves",
    "kernel_ms_stats_build": round(st.kernel_ms, 2),
    "pixel_chain_max": int(L.max()),
    "pixel_chain_p50": float(np.median(L)),
    "wave_iterations_max": int(steps.max()),
    "iterations_over_chain": {q: round(float(np.percentile(ratio, q)), 4) for q in (0, 10, 50, 90, 100)},
    "slowest_wave": {"iterations": int(steps[slow]), "chain": int(chain[slow]),
                     "ratio": round(float(ratio[slow]), 4), "pixels": int((k % W == slow).sum())},
    "lane_bound_iterations_p50": float(np.median(np.bincount(k % W, weights=L, minlength=W) / 64.0)),
}
print(json.dumps(res), flush=True)
