"""Fallback rates of the closest-hit culls in a real render (stats build,
RTP_DEBUG_STATS=1): per bounce step, how often some lane of the wave ran the
prefilter's exact scan of the axis-plane quads, and how often some lane ran
the rotated box's exact scan (box cull undecided), with the lanes that did.

    RTP_DEBUG_STATS=1 python tools/box_cull_rate.py [--spp 16] [--variant 0]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=800)
ap.add_argument("--ny", type=int, default=800)
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--variant", type=int, default=0)
a = ap.parse_args()
if os.environ.get("RTP_DEBUG_STATS") != "1":
    raise SystemExit("run with RTP_DEBUG_STATS=1 (the stats build of the pool kernel)")
dev = rtp.Device(0)
dev.set_cornell_box(a.variant)
pix = np.arange(a.nx * a.ny, dtype=np.int64)
dev.render_pixels(rtp.default_camera(), a.nx, a.ny, a.spp, a.depth, pix)
c = dev.debug_counters()
steps, lanes = c["bounce_steps"], c["bounce_lanes"]
print(json.dumps({"config": f"{a.nx}x{a.ny} x {a.spp} spp, depth {a.depth}, variant {a.variant}",
                  "box_cull": dev.box_cull(), "bounce_steps": steps, "live_lanes_per_step": lanes / max(steps, 1),
                  "prefilter_fallback_step_frac": c["fallback_steps"] / max(steps, 1),
                  "prefilter_fallback_lane_frac": c["fallback_lanes"] / max(lanes, 1),
                  "box_fallback_step_frac": c["boxfb_steps"] / max(steps, 1),
                  "box_fallback_lane_frac": c["boxfb_lanes"] / max(lanes, 1)}))
dev.close()
