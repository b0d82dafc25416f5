"""Timing of the -direct kernel (rtp_render_direct_kernel): all three AOVs +
depth of the default Cornell-box view in one launch, device-resident outputs,
HIP-event kernel time.  Prints one JSON line per repetition.

Algorithmic HBM bytes per pixel: 3 x 16 B (colour, normals, albedo float4) +
4 B depth = 52 B written; the scene (49 KB) and colour map (16 KB) are read
through the scalar cache once per wave."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402

import torch  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402
from raytracingtherestofyourlife_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=800)
ap.add_argument("--ny", type=int, default=800)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--aovs", type=int, default=7)
a = ap.parse_args()
dev = rtp.Device(0)
dev.set_cornell_box(0)
cb = rtp.CornellBox()
cb.buildDataSet()
qs = rtp.direct.quad_scalars(cb.ds.GetField("point_var").values, cb.ds.GetCellSet().quad_cells)
cmap = rtp.direct.main_pallet_color_table().Sample(1024)
n = a.nx * a.ny
bufs = {k: torch.zeros((n, 4), dtype=torch.float32, device="cuda") for k, bit in
        (("color", 1), ("normals", 2), ("albedo", 4)) if a.aovs & bit}
depth = torch.zeros(n, dtype=torch.float32, device="cuda")
d = _lib.RtpDirectDesc()
d.clip_near, d.clip_far = 0.1, 5.0
d.background[:] = [0.0, 0.0, 0.0, 1.0]
d.composite_background = 1
d.quad_scalar = qs.ctypes.data_as(_lib.f32p)
d.color_map = cmap.ctypes.data_as(_lib.f32p)
d.color_map_size = cmap.shape[0]
cam = rtp.default_camera().to_c()
s = torch.cuda.current_stream().cuda_stream
vp = ctypes.c_void_p
ptr = lambda k: vp(bufs[k].data_ptr()) if k in bufs else None
bytes_px = 16 * len(bufs) + 4
for r in range(a.reps):
    st = _lib.RtpStats()
    _lib.check(dev._L.rtp_render_direct_device(dev.handle, ctypes.byref(cam), a.nx, a.ny, ctypes.byref(d),
                                               ptr("color"), ptr("normals"), ptr("albedo"), vp(depth.data_ptr()),
                                               vp(s), ctypes.byref(st)))
    ms = st.kernel_ms
    print(json.dumps(dict(rep=r, nx=a.nx, ny=a.ny, aovs=a.aovs, kernel_ms=ms, mrays_per_s=n / (ms / 1e3) / 1e6,
                          gb_per_s=n * bytes_px / (ms / 1e3) / 1e9)), flush=True)
torch.cuda.synchronize()
