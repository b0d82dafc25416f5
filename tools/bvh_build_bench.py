"""Sphere-BVH build time (rtp_set_scene wall time) with the host SAH builder
and the device LBVH builder (RTP_BVH_BUILD=host|gpu), for random sphere
scenes of growing size, plus the render time of a small C3-style view with
each tree.  One JSON line per (n, builder)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle_ctypes as oc  # noqa: E402  (scene walls only)
import raytracingtherestofyourlife_amd as rtp  # noqa: E402
from test_gpu_bvh import _random_sphere_scene, _upload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sizes", default="1000,16384,131072,1048576")
ap.add_argument("--spp", type=int, default=4)
ap.add_argument("--res", type=int, default=512)
a = ap.parse_args()
dev = rtp.Device(0)
n_px = a.res * a.res
out = torch.zeros((n_px, 4), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for n in [int(v) for v in a.sizes.split(",")]:
    scene = _random_sphere_scene(oc, n, 11)
    for build in ("host", "gpu"):
        os.environ["RTP_BVH_BUILD"] = build
        t = time.time()
        _upload(dev, *scene)
        torch.cuda.synchronize()
        t_build = time.time() - t
        st = dev.render_device(rtp.default_camera(), a.res, a.res, a.spp, 50, out.data_ptr(), stream=s, timed=True)
        print(json.dumps(dict(n=n, build=build, set_scene_s=round(t_build, 4), render_ms=st.kernel_ms,
                              msamples_per_s=n_px * a.spp / (st.kernel_ms / 1e3) / 1e6)), flush=True)
