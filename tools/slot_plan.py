"""Wave-slot balance experiment (development tool).

The SIMD arbiter favours older waves: in a C2 launch the waves in hardware
slot 0 of their SIMD finish ~1/3 earlier than the waves in slot 4, and the
SIMDs run their last tens of milliseconds with fewer waves.  This tool times
planned launches (rtp_render_planned_device) on a random pixel subset:
  uniform  every wave the same number of pixels;
  slot     pixels per wave in proportion to the measured speed of its slot
           (1 / mean lifetime of the slot's waves in the uniform launch);
and reports the wave lifetimes by slot (RTP_DEBUG_STATS=2 timestamps) and
whether the wave -> slot placement is the same from launch to launch.

    python tools/slot_plan.py [--pixels-per-wave 80] [--reps 3]
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
ap.add_argument("--n", type=int, default=800)
ap.add_argument("--spp", type=int, default=1000)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--waves", type=int, default=5120)
ap.add_argument("--pixels-per-wave", type=int, default=80)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--power", type=float, default=1.0, help="weight = speed**power")
a = ap.parse_args()

dev = rtp.Device(0)
dev.set_cornell_box(0)
dev.set_ff_tables("on")
cam = rtp.default_camera()
W = a.waves
n = min(a.n * a.n, W * a.pixels_per_wave)
perm = np.random.default_rng(7).permutation(a.n * a.n)[:n].astype(np.int64)
ids = torch.from_numpy(perm).cuda()
s = torch.cuda.current_stream().cuda_stream
out = torch.zeros((n, 4), dtype=torch.float32, device="cuda")


def run(counts):
    wb = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    assert wb[-1] == n and (counts >= 1).all() and (counts <= 128).all()
    wbt = torch.from_numpy(wb).cuda()
    best, recs = 1e9, []
    for _ in range(a.reps):
        st = dev.render_planned_device(cam, a.n, a.n, a.spp, a.depth, out.data_ptr(), n, wbt.data_ptr(), W,
                                       pixel_ids_ptr=ids.data_ptr(), stream=s, timed=True)
        best = min(best, st.kernel_ms)
        recs.append(dev.debug_wave_records())
    res = out.cpu().numpy().copy()
    return best, recs, res


def by_slot(rec):
    start, end = rec[:, 12].astype(np.int64), rec[:, 13].astype(np.int64)
    life = (end - start) / 100.0
    slot = rec[:, 14].astype(np.int64) & 0xF
    return slot, life, {int(k): round(float(life[slot == k].mean()), 1) for k in np.unique(slot)}


uni = np.full(W, n // W, np.int64)
uni[: n - uni.sum()] += 1
ms_u, recs_u, img_u = run(uni)
slot0, life0, tab0 = by_slot(recs_u[0])
stable = [float((by_slot(r)[0] == slot0).mean()) for r in recs_u[1:]]
res = {"pixels": n, "waves": W, "uniform": {"ms": round(ms_u, 2), "life_by_slot_us": tab0,
                                            "slot_same_as_first": stable}}
speed = {k: 1.0 / v for k, v in tab0.items()}
wgt = np.array([speed[int(k)] for k in slot0]) ** a.power
cnt = np.clip(np.floor(wgt / wgt.sum() * n).astype(np.int64), 1, 128)
rem = n - cnt.sum()
order = np.argsort(-wgt, kind="stable")
i = 0
while rem != 0:  # hand out / take back the rounding remainder, fastest waves first
    w = order[i % W]
    if rem > 0 and cnt[w] < 128:
        cnt[w] += 1
        rem -= 1
    elif rem < 0 and cnt[w] > 1:
        cnt[w] -= 1
        rem += 1
    i += 1
ms_s, recs_s, img_s = run(cnt)
res["slot"] = {"ms": round(ms_s, 2), "life_by_slot_us": by_slot(recs_s[0])[2],
               "pixels_by_slot": {int(k): round(float(cnt[slot0 == k].mean()), 1) for k in np.unique(slot0)}}
# the pixels are the same, only their waves differ: renders must be equal bit for bit
res["equal"] = bool((img_u[:, :3].view(np.uint32) == img_s[:, :3].view(np.uint32)).all() |
                    (np.isnan(img_u[:, :3]) & np.isnan(img_s[:, :3])).all())
res["speedup"] = round(ms_u / ms_s, 4)
print(json.dumps(res), flush=True)
