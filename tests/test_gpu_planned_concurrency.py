"""rtp_render_planned_device against rtp_render_device, and two
contexts rendering from two host threads while one of them moves the shared
per-device RNG jump tables through their AUTO stages (the tables
are published only after their build finished, and a launch holds a snapshot).

Reference: MapperPathTracer.cxx:278-350 (each pixel's sample chain); the plan
and the tables only change the schedule and the RNG fast-forward, never a
result, so every render here must equal the plain one bit for bit."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _same(a, b):
    a, b = np.asarray(a)[:, :3], np.asarray(b)[:, :3]
    return bool(((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))).all())


def test_planned_render_equals_device_render(device):
    """A wave plan of ragged ranges (1..128 entries per wave, in order) gives
    the same pixels, final seeds and live counts as the interleaved launch."""
    import torch

    import raytracingtherestofyourlife_amd as rtp

    device.set_cornell_box(0)
    cam = rtp.default_camera()
    nx, ny, spp, depth = 96, 64, 16, 50
    n = nx * ny
    rng = np.random.default_rng(5)
    sizes = []
    while sum(sizes) < n:
        sizes.append(int(min(rng.integers(1, 129), n - sum(sizes))))
    begin = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    out = {}
    for mode in ("plain", "planned"):
        rgba = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
        seed = torch.zeros(n, dtype=torch.int32, device="cuda")
        live = torch.zeros(n, dtype=torch.int32, device="cuda")
        if mode == "plain":
            device.render_device(cam, nx, ny, spp, depth, rgba.data_ptr(), seed_ptr=seed.data_ptr(),
                                 live_ptr=live.data_ptr())
        else:
            wb = torch.from_numpy(begin).cuda()
            device.render_planned_device(cam, nx, ny, spp, depth, rgba.data_ptr(), n, wb.data_ptr(), len(sizes),
                                         seed_ptr=seed.data_ptr(), live_ptr=live.data_ptr())
        torch.cuda.synchronize()
        out[mode] = (rgba.cpu().numpy(), seed.cpu().numpy(), live.cpu().numpy())
    assert _same(out["planned"][0], out["plain"][0])
    assert np.array_equal(out["planned"][1], out["plain"][1])
    assert np.array_equal(out["planned"][2], out["plain"][2])


@pytest.mark.parametrize("bad", ["not_monotone", "range_over_128", "short_end", "long_end"])
def test_planned_render_rejects_bad_plans(device, bad):
    """The host checks a plan before launching it: monotone, at most 128
    entries per wave, ending exactly at pixel_count."""
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd._lib import RtpError

    device.set_cornell_box(0)
    n = 1024
    plans = {
        "not_monotone": [0, 100, 50, 1024],
        "range_over_128": [0, 200, 1024] + [],
        "short_end": list(range(0, 1000, 100)) + [1000],
        "long_end": list(range(0, 1024, 128)) + [1100],
    }
    wb = torch.tensor(plans[bad], dtype=torch.int32, device="cuda")
    rgba = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    with pytest.raises(RtpError):
        device.render_planned_device(rtp.default_camera(), 32, 32, 4, 10, rgba.data_ptr(), n, wb.data_ptr(),
                                     wb.numel() - 1)


_TWO_THREADS = r"""
import threading, numpy as np, torch
import raytracingtherestofyourlife_amd as rtp
cam = rtp.default_camera()
nx, ny, spp, depth = 64, 64, 8, 50
ref = rtp.Device(0); ref.set_cornell_box(0); ref.set_ff_tables("off")
want = ref.render(cam, nx, ny, spp, depth)[0]
ref.close()
results, errors = {}, []
def work(name, rounds):
    try:
        d = rtp.Device(0); d.set_cornell_box(0)
        s = torch.cuda.Stream()
        got = []
        for _ in range(rounds):
            o = torch.zeros((nx * ny, 4), dtype=torch.float32, device="cuda")
            d.render_device(cam, nx, ny, spp, depth, o.data_ptr(), stream=s.cuda_stream)
            s.synchronize()
            got.append((o.cpu().numpy(), d.ff_info()["built"]))
        results[name] = got
        d.close()
    except Exception as e:
        errors.append(repr(e))
ts = [threading.Thread(target=work, args=(k, 6)) for k in ("a", "b")]
[t.start() for t in ts]; [t.join() for t in ts]
assert not errors, errors
def same(a, b):
    a, b = a[:, :3], b[:, :3]
    return bool(((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))).all())
stages = sorted({b for v in results.values() for _, b in v})
ok = all(same(o, want) for v in results.values() for o, _ in v)
print("stages", stages, "ok", ok)
"""


def test_two_contexts_race_an_auto_stage_build():
    """Two contexts in two threads (each on its own non-blocking stream)
    render while their shared tables go none -> chain -> direct under AUTO
    (break-even counts lowered in a child process): every frame equals the
    table-free render, whichever tables it ran with."""
    env = dict(os.environ, RTP_FF_AUTO_SAMPLES="60000,200000", RTP_FF_TABLES="1", RTP_FF_DIRECT="1")
    out = subprocess.run([sys.executable, "-c", _TWO_THREADS], env=env, capture_output=True, text=True, timeout=280,
                         cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    last = out.stdout.strip().splitlines()[-1]
    assert last.endswith("ok True"), last
    assert "2" in last.split("stages")[1].split("ok")[0], f"the direct stage was never reached: {last}"
