"""End-to-end cost of a render in a FRESH process (development tool).

main.cc renders once per process and its timer covers the whole run
(main.cc:584-585, 653, 661-663).  This times, in one new process: context
creation, scene upload, the first render (which includes any RNG jump-table
build the library's policy triggers), then a few more renders of the same
workload (steady state).  One JSON line.

    python tools/setup_cost.py [--nx 800 --ny 800 --spp 1000 --depth 50] [--renders 3]
"""
import argparse
import json
import os
import sys
import time

t_start = time.perf_counter()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracingtherestofyourlife_amd as rtp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=800)
ap.add_argument("--ny", type=int, default=800)
ap.add_argument("--spp", type=int, default=1000)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--renders", type=int, default=3)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--ff-tables", default="auto", choices=["on", "auto", "off"], help="RNG jump-table policy")
a = ap.parse_args()
# the HIP runtime's first-use initialisation (first host-to-device copy) is
# process start, as in bench.py
torch.ones(1).cuda()
torch.cuda.synchronize()
t_import = time.perf_counter() - t_start

t = time.perf_counter()
dev = rtp.Device(0)
t_create = time.perf_counter() - t
t = time.perf_counter()
dev.set_cornell_box(0)
t_scene = time.perf_counter() - t
t = time.perf_counter()
dev.set_ff_tables(a.ff_tables)
t_ff = time.perf_counter() - t
cam = rtp.default_camera()
n = a.nx * a.ny
out = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
s = torch.cuda.current_stream().cuda_stream
walls, kms = [], []
for r in range(a.renders):
    t = time.perf_counter()
    st = dev.render_tiles_device(cam, a.nx, a.ny, a.spp, a.depth, out.data_ptr(), a.rank, a.world, stream=s,
                                 timed=True)
    torch.cuda.synchronize()
    walls.append((time.perf_counter() - t) * 1e3)
    kms.append(st.kernel_ms)
info = dev.ff_info()
samples = n // a.world * a.spp
print(json.dumps(dict(
    env={k: v for k, v in os.environ.items() if k.startswith("RTP_")},
    workload=f"{a.nx}x{a.ny}x{a.spp} depth {a.depth}, tiles rank {a.rank}/{a.world}",
    import_s=round(t_import, 3), create_ms=round(t_create * 1e3, 2), scene_ms=round(t_scene * 1e3, 2),
    ff_policy_ms=round(t_ff * 1e3, 2),
    render_wall_ms=[round(x, 2) for x in walls], kernel_ms=[round(x, 2) for x in kms],
    first_render_msamples_s=round(samples / walls[0] / 1e3, 1),
    end_to_end_msamples_s=round(samples / (t_create + t_scene + t_ff + walls[0] / 1e3) / 1e6, 1),
    steady_msamples_s=round(samples / min(kms[1:] or kms) / 1e3, 1),
    ff=info)), flush=True)
dev.close()
