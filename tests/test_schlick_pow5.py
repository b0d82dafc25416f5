"""schlick's x^5 (EmitWorklet.h:153-158: pow((double)(1 - cosine), 5.0)) on
the device is rtp_device.hpp pow5_exact, a double-double product, not a pow
call.  Two host checks pin it (tests/cpp/pow5_check.cpp, every float x):
  - it is the correctly rounded x^5 for every float |x| in [2^-24, 2] (the
    range of 1 - cosine: 0 or >= 2^-24, <= 2.5);
  - the float reflect probability it gives equals the one glibc's pow gives
    (the reference's, and the oracle's) for every float |x| <= 4 at the
    reference's ior 1.5 (MapperPathTracer.cxx:467) and at 1.3 -- although
    glibc's pow itself is not correctly rounded for ~0.09% of these x."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def pow5_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pow5") / "pow5_check")
    src = os.path.join(ROOT, "tests", "cpp", "pow5_check.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", src, "-o", exe, "-lquadmath", "-lpthread"],
                   check=True)
    return exe


def _run(exe, *args):
    out = subprocess.run([exe, *args], capture_output=True, text=True, check=True, timeout=600).stdout
    assert out.startswith("mismatches 0 "), (args, out)


def test_pow5_exact_is_correctly_rounded(pow5_check):
    _run(pow5_check, "cr", "33800000", "40000000")  # [2^-24, 2]
    _run(pow5_check, "cr", "b3800000", "c0000000")  # [-2, -2^-24]


@pytest.mark.parametrize("ior", ["1.5", "1.3"])
def test_schlick_float_equals_glibc_pow(pow5_check, ior):
    _run(pow5_check, "schlick", ior, "00000000", "40800000")  # [0, 4]
    _run(pow5_check, "schlick", ior, "80000000", "c0800000")  # [-4, -0]
