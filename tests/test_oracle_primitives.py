"""Known-answer tests pinning the CPU restatement's primitives (CPU only).

Values from SURVEY.md section 4 (probed with g++ 11.4 / glibc 2.35 on this
host) and from this host's libm."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest


def test_wang_known_answers(oracle):
    assert oracle.wang32(0) == 3232319850
    # WangInit(1) (MapperPathTracer.cxx:60-75) = wang^4(1)
    x = 1
    for _ in range(4):
        x = oracle.wang32(x)
    assert x == 3205955024


@pytest.mark.parametrize(
    "seed,vals",
    [
        (0, [0.752583086, 0.716025889, 0.175872773, 0.0962651521]),
        (1, [0.154574186, 0.404735804, 0.186604708, 0.746444583]),
        (639999, [0.23263742, 0.899121642, 0.843598843, 0.552849352]),
    ],
)
def test_randf_known_answers(oracle, seed, vals):
    got, _ = oracle.randf_stream(seed, 4)
    np.testing.assert_allclose(got, vals, rtol=0, atol=5e-9)


def test_randf_reaches_one(oracle):
    """getRandF returns exactly 1.0f for hashes >= 4294967168 (wangXor.h:58)."""
    assert np.float32(4294967168) / np.float32(4294967295.0) == np.float32(1.0)
    # 4294967168 is the midpoint between 2^32-256 and 2^32 and rounds (to even) up
    assert np.float32(4294967167) / np.float32(4294967295.0) < np.float32(1.0)
    assert np.float32(4294967040) / np.float32(4294967295.0) < np.float32(1.0)


def test_randf_is_exact_power_of_two_scaling():
    """float(t)/4294967295.f == float(t) * 2^-32 for every t (the divisor rounds
    to 2^32): the device uses the multiply."""
    rng = np.random.default_rng(0)
    t = rng.integers(0, 2**32, size=200000, dtype=np.uint64).astype(np.uint32)
    t = np.concatenate([t, np.uint32([0, 1, 2**31, 2**32 - 1, 4294967168, 4294967167])])
    f = t.astype(np.float32)
    assert np.array_equal((f / np.float32(4294967295.0)).view(np.uint32), (f * np.float32(2.0**-32)).view(np.uint32))


def _which_threshold(oracle, w):
    L = oracle.lib()
    lo, hi = 0, 1 << 32
    while lo < hi:
        mid = (lo + hi) // 2
        if L.rtpo_which(mid) >= w:
            hi = mid
        else:
            lo = mid + 1
    return lo


def test_which_is_a_two_threshold_step_function(oracle):
    """which = min(3, int(r*3+1)) is monotone in the hash, so the device can
    decide it with two integer compares (rtp_host.cpp which_threshold)."""
    L = oracle.lib()
    t1, t2 = _which_threshold(oracle, 2), _which_threshold(oracle, 3)
    assert 0 < t1 < t2 < 2**32
    for t, w in [(t1 - 1, 1), (t1, 2), (t2 - 1, 2), (t2, 3), (0, 1), (2**32 - 1, 3)]:
        assert L.rtpo_which(t) == w
    rng = np.random.default_rng(5)
    for t in rng.integers(0, 2**32, size=20000, dtype=np.uint64):
        t = int(t)
        assert L.rtpo_which(t) == 1 + (t >= t1) + (t >= t2)


def test_glibc_sincosf_restatement_matches_libm(oracle):
    """The sinf/cosf restatement equals this host's libm bit-for-bit on a dense
    stride through [0, 2*pi] (the exhaustive sweep, stride 1, was run when the
    restatement was written: 1,086,919,938 floats, 0 mismatches)."""
    L = oracle.lib()
    L.rtpo_check_sincos_vs_libm.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_int64)]
    L.rtpo_check_sincos_vs_libm.restype = ctypes.c_int64
    checked = ctypes.c_int64(0)
    bad = L.rtpo_check_sincos_vs_libm(0.0, 6.2831855, 97, ctypes.byref(checked))
    assert checked.value > 10_000_000
    assert bad == 0
    # the region phi can actually reach (<= float(2*pi))
    assert np.float32(2 * np.pi) <= np.float32(6.2831855)


def test_gxx_argument_order_is_encoded(oracle):
    """SphereWorkletGenerateDir calls random(p, getRandF(seed), getRandF(seed),
    ...) (PdfWorklet.h:210); g++ evaluates right to left, so r1 is the second
    draw.  Probe the host compiler and check that the oracle follows it."""
    import os
    import shutil
    import subprocess
    import tempfile

    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    src = r"""
#include <cstdio>
static unsigned s = 0;
float draw() { return (float)(++s); }
struct W { void random(const float& o, float r1, float r2, const float& c, float rad) const {
  std::printf("%g %g\n", r1, r2); } };
int main() { W w; float p = 0, c = 0; w.random(p, draw(), draw(), c, 1.0f); }
"""
    with tempfile.TemporaryDirectory() as d:
        cpp = os.path.join(d, "o.cpp")
        exe = os.path.join(d, "o")
        open(cpp, "w").write(src)
        subprocess.run([gxx, "-O2", "-o", exe, cpp], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["2", "1"], "g++ no longer evaluates right to left; the restatement must follow the compiler"
