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
