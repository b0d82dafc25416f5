"""The sphere hit normal (p - c) / r as Markstein divisions by RN(1/r)
(rtp_kernels.hip shade_hit under RTP_SPH_NORMAL_MK, rtp_device.hpp
div_markstein) against IEEE float division, on the host (tests/cpp/
markstein_check.c, gcc with hardware FMA): every float numerator with |a| in
[2^-40, 2^40], both signs, for C2's glass-sphere radius (90/555) and the ends
of C3's radius range (8/555, 30/555); 3e8 random (a, r) pairs over the whole
range the kernel admits (r in [2^-20, 2^20]).  Markstein's theorem (Muller et
al., Thm 5.8) is the argument; this is the check."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "markstein_check.c")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    with open("/proc/cpuinfo") as f:
        if " fma " not in f.read():
            pytest.skip("host CPU without FMA3")
    exe = str(tmp_path_factory.mktemp("mk") / "markstein_check")
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-o", exe, SRC, "-lm"], check=True)
    return exe


@pytest.mark.parametrize("radius", [90 / 555.0, 8 / 555.0, 30 / 555.0])
def test_markstein_normal_exhaustive(checker, radius):
    r = float(np.float32(radius)).hex()
    out = subprocess.run([checker, "exhaustive", r], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK ")


def test_markstein_normal_sampled(checker):
    out = subprocess.run([checker, "sampled", "300000000", "7"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip() == "OK 300000000"
