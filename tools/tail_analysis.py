"""Which waves of the pool kernel finish last, and why (development tool).

Renders C2 (contiguous pixels) with RTP_DEBUG_STATS=2 (wave start/end
stamps in the production kernel) and the per-pixel live-bounce counts, then
relates each wave's finish time to its pixels: the wave's total work (sum of
live bounces), and its longest sample chain (max over its pixels of
live bounces + samples, i.e. bounce iterations + one fast-forward per sample).
Wave w owns entries k = j * W + w (j < slots), as in rtp_render_pool.
usage: python tools/tail_analysis.py [--spp 1000]
"""
import argparse
import json
import os
import sys

os.environ["RTP_DEBUG_STATS"] = "2"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=1000)
ap.add_argument("--depth", type=int, default=50)
a = ap.parse_args()
dev = rtp.Device(0)
dev.set_cornell_box(0)
n = 800 * 800
out = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
live = torch.zeros(n, dtype=torch.int32, device="cuda")
st = dev.render_device(rtp.default_camera(), 800, 800, a.spp, a.depth, out.data_ptr(),
                       stream=torch.cuda.current_stream().cuda_stream, live_ptr=live.data_ptr(), timed=True)
torch.cuda.synchronize()
rec = dev.debug_wave_records()
W = len(rec)
start, end = rec[:, 12].astype(np.int64), rec[:, 13].astype(np.int64)
fin = (end - start.min()) / 100.0  # us
lv = live.cpu().numpy().astype(np.int64)
k = np.arange(n)
w_of = k % W
work = np.bincount(w_of, weights=lv, minlength=W)            # live bounces of the wave
chain = np.zeros(W)
np.maximum.at(chain, w_of, lv + a.spp)                       # longest pixel chain (iterations)
order = np.argsort(fin)
last = order[-W // 20:]  # last 5% of waves to finish
first = order[: W // 2]
res = dict(kernel_ms=st.kernel_ms, waves=W,
           finish_us_pct={q: round(float(np.percentile(fin, q)), 1) for q in (0, 10, 50, 90, 99, 100)},
           corr_finish_chain=round(float(np.corrcoef(fin, chain)[0, 1]), 3),
           corr_finish_work=round(float(np.corrcoef(fin, work)[0, 1]), 3),
           chain_last5pct_mean=round(float(chain[last].mean()), 1), chain_first50pct_mean=round(float(chain[first].mean()), 1),
           work_last5pct_mean=round(float(work[last].mean()), 1), work_first50pct_mean=round(float(work[first].mean()), 1),
           chain_pct={q: round(float(np.percentile(chain, q)), 1) for q in (0, 50, 90, 99, 100)},
           iterations_est_per_wave=round(float(work.mean() / 60.0 + 0), 1))
print(json.dumps(res))
