"""The RNG jump-table policy of include/rtp.h (rtp_set_ff_tables), AUTO:
a one-shot render builds nothing, and the two stages (chain tables, then the
direct block) come at their break-even sample counts.  The tables are per
device and process, so this file runs first (its name sorts before every
other test file) while no test has built them yet."""
from __future__ import annotations

import os

import pytest

pytestmark = pytest.mark.gpu


def test_policy_auto_leaves_one_shot_renders_alone():
    """A fresh context on the default policy renders a small frame without
    building (or using) tables; the samples are counted toward break-even."""
    import raytracingtherestofyourlife_amd as rtp

    d = rtp.Device(0)
    try:
        i0 = d.ff_info()
        assert i0["policy"] == "auto"
        if i0["built"]:
            pytest.skip("tables already built in this process")
        d.set_cornell_box(0)
        d.render(rtp.default_camera(), 32, 32, 4, 10)
        i1 = d.ff_info()
        assert i1["built"] == 0 and i1["samples_seen"] == i0["samples_seen"] + 32 * 32 * 4
    finally:
        d.close()


def test_policy_auto_stages():
    """AUTO builds the chain tables, then the direct block, at the break-even
    counts (lowered here through RTP_FF_AUTO_SAMPLES in a child process)."""
    import subprocess
    import sys

    code = (
        "import raytracingtherestofyourlife_amd as rtp\n"
        "d = rtp.Device(0); d.set_cornell_box(0); cam = rtp.default_camera()\n"
        "seen = []\n"
        "for _ in range(3):\n"
        "    d.render(cam, 64, 64, 8, 10); seen.append(d.ff_info()['built'])\n"
        "print(seen)\n")
    env = dict(os.environ, RTP_FF_AUTO_SAMPLES="40000,70000", RTP_FF_TABLES="1", RTP_FF_DIRECT="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-2000:]
    # 32768 samples per render: none, then chain (65536 >= 40000), then direct (98304 >= 70000)
    assert out.stdout.strip().splitlines()[-1] == "[0, 1, 2]"


def test_policy_auto_direct_stage_follows_measured_allocation():
    """The default thresholds, unlowered: C2 frames (6.4e8 samples each) in a
    fresh child process.  The chain tables come with the 12th frame (7.5e9
    samples); from then on the direct stage's break-even is the chain stage's
    count + (0.07 s + 2.5x the chain tables' measured allocation time) /
    1.23e-11 s per sample (rtp_host.cpp ff_auto_samples), and the direct
    block is built on the frame that reaches it."""
    import json
    import subprocess
    import sys

    code = (
        "import json, raytracingtherestofyourlife_amd as rtp\n"
        "d = rtp.Device(0); d.set_cornell_box(0); cam = rtp.default_camera()\n"
        "rec = []\n"
        "for _ in range(60):\n"
        "    d.render(cam, 800, 800, 1000, 50); i = d.ff_info()\n"
        "    rec.append([i['samples_seen'], i['built'], i['auto_samples'], i['auto_samples_direct'], i['alloc_ms']])\n"
        "    if i['built'] == 2: break\n"
        "print(json.dumps(rec))\n")
    env = {k: v for k, v in os.environ.items() if not k.startswith("RTP_FF")}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-2000:]
    _wait_for_device_memory()  # (the child's 224 GiB come back after it exits, not at once)
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    per = 800 * 800 * 1000
    built = [r[1] for r in rec]
    assert rec[0][2] == 7_500_000_000 and built[:11] == [0] * 11 and built[11] >= 1
    assert all(r[3] == 300_000_000_000 for r in rec[:11])  # before the chain stage: the fixed count
    chain_at, alloc_ms = rec[11][0], rec[11][4]
    want = chain_at + int((0.07 + 2.5 * alloc_ms / 1e3) / 1.23e-11)
    if built[11] == 1:
        assert abs(rec[11][3] - want) <= 1, (rec[11], want)
    reach = next((k for k in range(11, 60) if chain_at + (k - 11) * per >= want), None)
    if reach is None:
        pytest.skip(f"the chain tables' allocation took {alloc_ms:.0f} ms: the direct stage is beyond 60 frames")
    assert built[reach] == 2 and built[reach - 1] < 2, (reach, built)


def _wait_for_device_memory(timeout_s: float = 60.0) -> None:
    """Until the device's free memory is back to what a fresh process sees
    (within 16 GiB): later tests in this process build the full tables."""
    import time

    import torch

    t0 = time.time()
    while time.time() - t0 < timeout_s:
        free, total = torch.cuda.mem_get_info(0)
        if free > total - (16 << 30):
            return
        time.sleep(0.5)
    free, total = torch.cuda.mem_get_info(0)
    pytest.fail(f"the child's jump tables were not released within {timeout_s:.0f} s: "
                f"{free / 2**30:.1f} of {total / 2**30:.1f} GiB free (later table builds would fail with an "
                f"unrelated out-of-memory error)")
