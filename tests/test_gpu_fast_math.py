"""The short reciprocal / sqrt sequences the kernels use in place of the IEEE
lowering are bit-identical to it for EVERY float of the range they are used
on (exhaustive, on the device).  Outside [2^-40, 2^40] the kernels fall back
to the IEEE operation (rcp_exact / sqrt_exact / rsqrt_exact)."""
import pytest

pytestmark = pytest.mark.gpu

LO, HI = 2.0**-40, 2.0**40


@pytest.mark.parametrize("kind,name", [(0, "rcp"), (2, "sqrt"), (3, "rsqrt")])
def test_fast_sequence_exact_on_whole_range(device, kind, name):
    bad, first = device.verify_fast_math(kind, LO, HI)
    assert bad == 0, f"{name}: {bad} mismatches, first bit pattern {first:#x}"
    if kind == 0:
        bad, first = device.verify_fast_math(kind, -LO, -HI)
        assert bad == 0, f"{name} (negative): {bad} mismatches, first {first:#x}"


def test_fast_range_boundaries_are_covered(device):
    """The checked range includes every value the guards let through."""
    import numpy as np

    assert np.float32(LO) == np.float32(2.0**-40) and np.float32(HI) == np.float32(2.0**40)


def test_cos_over_pi_product_exact(device):
    """(float)((double)c * (1/pi)) == (float)((double)c / pi) for every float c in [0, 2]."""
    bad, first = device.verify_fast_math(5, 0.0, 2.0)
    assert bad == 0, f"cos_over_pi: {bad} mismatches, first bit pattern {first:#x}"


@pytest.mark.parametrize("kind,name", [(6, "sin"), (7, "cos")])
def test_branch_free_sincos_equals_ports(device, kind, name):
    """rtp_sincosf (the generator's shared sincos) == rtp_sinf / rtp_cosf for
    every float in [0, 2pi] (phi = float(2*pi*r), r in [0, 1])."""
    bad, first = device.verify_fast_math(kind, 0.0, 6.2831855)
    assert bad == 0, f"sincos/{name}: {bad} mismatches, first bit pattern {first:#x}"


def test_markstein_division_exact(device):
    """div_markstein(a, b, rcp_nr1(b)) == a / b (IEEE) for EVERY float divisor b
    with |b| in [2^-20, 2^26] (camera_ray's |rd|: >= ~1, < 2^26) and 32
    numerators per divisor spread over [-b, b] and [-1024 b, 1024 b]
    (rtp_verify_fast_math kind 8; normal quotients)."""
    for lo, hi in ((2.0**-20, 2.0**26), (-(2.0**-20), -(2.0**26))):
        bad, first = device.verify_fast_math(8, lo, hi)
        assert bad == 0, f"markstein: {bad} mismatches, first divisor bit pattern {first:#x}"
