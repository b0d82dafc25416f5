"""Fall-back rate of the closest-hit prefilter (rtp_debug_closest_hit) per ray
population of tests/test_gpu_prefilter.stress_rays, and the implied share of
64-lane waves that run the exact scan (1 - (1 - p)^57 at ~57 live lanes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402
from test_gpu_prefilter import scene_quads, stress_rays  # noqa: E402

dev = rtp.Device(0)
dev.set_cornell_box(0)
rays = stress_rays(scene_quads(0), 1 << 21, 11)
got = dev.debug_closest_hit(rays)
k = len(rays) // 8
names = ["edge-aimed", "from surfaces", "grazing", "on planes/axis", "unnormalised", "out of range", "camera",
         "to light"]
for i, n in enumerate(names):
    p = (got[i * k:(i + 1) * k, 6] == 1).mean()
    print(f"{n:16s} fallback {p:.5f}  waves {1 - (1 - p) ** 57:.3f}  mismatches "
          f"{int((got[i * k:(i + 1) * k, 0:3] != got[i * k:(i + 1) * k, 3:6]).any(1).sum())}")
