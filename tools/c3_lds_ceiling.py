"""C3's scene cut to its first N spheres (development tool): how much the LDS
walk gains over the global walk when the one-sphere-leaf tree's 8 octant
copies fit the block's LDS (N ~ 300), i.e. the ceiling of moving the walk's
gathers off the texture path without changing the tree.

    RTP_BVH_LDS=0|1 [RTP_LIB_PATH=...] python tools/c3_lds_ceiling.py [--spheres 300] [--spp 16] [--reps 3]

Prints one JSON line per rep: kernel ms, the walk in use, Msamples/s."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402
from raytracingtherestofyourlife_amd import _lib  # noqa: E402
from raytracingtherestofyourlife_amd._lib import RtpSceneDesc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spheres", type=int, default=300)
ap.add_argument("--n", type=int, default=2048)
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

dev = rtp.Device(0)
dev.set_ff_tables("on")
L = _lib.load()
d = RtpSceneDesc()
_lib.check(L.rtp_cornell_box(3, ctypes.byref(d)))
d.n_spheres = min(a.spheres, d.n_spheres)  # the first N of C3's spheres (sphere 0 stays the light-sphere target)
_lib.check(L.rtp_set_scene(dev.handle, ctypes.byref(d)))
walk = dev.sphere_walk()
n = a.n * a.n
out = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
for rep in range(a.reps):
    st = dev.render_device(rtp.default_camera(), a.n, a.n, a.spp, a.depth, out.data_ptr(), timed=True)
    print(json.dumps({"rep": rep, "spheres": d.n_spheres, "walk": walk, "kernel_ms": st.kernel_ms,
                      "msamples_per_s": n * a.spp / st.kernel_ms / 1e3}), flush=True)
dev.close()
