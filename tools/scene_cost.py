"""Where a fresh process's scene upload time goes (development tool).

Times, in one new process: context creation, the host scene build
(rtp_cornell_box), the first and a second rtp_set_scene, and the first and a
second tiny render (8x8, 1 spp).  One JSON line.

    python tools/scene_cost.py [--variant 0]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402
from raytracingtherestofyourlife_amd import _lib  # noqa: E402
from raytracingtherestofyourlife_amd.mapper import check  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variant", type=int, default=0)
a = ap.parse_args()
torch.zeros(1, device="cuda")  # the HIP runtime up, as in bench.py
res = {}


def tick(name, fn):
    t = time.perf_counter()
    r = fn()
    res[name] = round((time.perf_counter() - t) * 1e3, 2)
    return r


dev = tick("create_ms", lambda: rtp.Device(0))
d = _lib.RtpSceneDesc()
tick("host_scene_ms", lambda: check(dev._L.rtp_cornell_box(a.variant, ctypes.byref(d))))
tick("set_scene_1_ms", lambda: check(dev._L.rtp_set_scene(dev.handle, ctypes.byref(d))))
tick("set_scene_2_ms", lambda: check(dev._L.rtp_set_scene(dev.handle, ctypes.byref(d))))
dev.set_ff_tables("off")
cam = rtp.default_camera()
tick("render_1_ms", lambda: dev.render(cam, 8, 8, 1, 50))
tick("render_2_ms", lambda: dev.render(cam, 8, 8, 1, 50))
print(json.dumps(res), flush=True)
dev.close()
