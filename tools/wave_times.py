"""Per-wave lifetime / placement of the production pool kernel (RTP_DEBUG_STATS=2)."""
import os, sys, json, argparse
os.environ["RTP_DEBUG_STATS"] = "2"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import raytracingtherestofyourlife_amd as rtp

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=1000)
ap.add_argument("--depth", type=int, default=50)
a = ap.parse_args()
dev = rtp.Device(0)
dev.set_cornell_box(0)
n = 800 * 800
out = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
st = dev.render_device(rtp.default_camera(), 800, 800, a.spp, a.depth, out.data_ptr(),
                       stream=torch.cuda.current_stream().cuda_stream, timed=True)
torch.cuda.synchronize()
rec = dev.debug_wave_records()
start, end, hw = rec[:, 12].astype(np.int64), rec[:, 13].astype(np.int64), rec[:, 14].astype(np.int64)
t0 = start.min()
fin = (end - t0) / 100.0
life = (end - start) / 100.0
slot = hw & 0xF
simd = (hw >> 4) & 3
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
print(json.dumps(dict(kernel_ms=st.kernel_ms, waves=int(len(rec)),
                      finish_us_pct={q: round(float(np.percentile(fin, q)), 1) for q in (0, 10, 50, 90, 100)},
                      avg_over_max=round(float(life.mean() / life.max()), 4),
                      by_slot={int(s): round(float(life[slot == s].mean()), 1) for s in np.unique(slot)},
                      by_se={int(s): round(float(fin[se == s].max()), 1) for s in np.unique(se)})))
