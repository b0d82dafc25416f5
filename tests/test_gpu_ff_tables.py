"""RNG jump tables (rtp_host.cpp, one fused build kernel): the state after 32 /
16 / ... dead depths (chain tables) and after each count of the direct block,
for every 32-bit state.  Checked on random states against an independent
numpy restatement of the dead-depth draw sequence (which draw, then 2 or 3
generator draws, PdfWorklet.h:9-215), itself checked against the oracle's
Wang hash.  Also the table policy of include/rtp.h (rtp_set_ff_tables)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def wang_np(s):
    s = s.astype(np.uint32)
    s = (s ^ np.uint32(61)) ^ (s >> np.uint32(16))
    s = s * np.uint32(9)
    s = s ^ (s >> np.uint32(4))
    s = s * np.uint32(0x27D4EB2D)
    return s ^ (s >> np.uint32(15))


def dead_np(s, t1, t2):
    t = wang_np(s)
    s2 = wang_np(wang_np(t))
    s3 = wang_np(s2)
    return np.where((t >= t1) & (t < t2), s3, s2)


@pytest.fixture(scope="module")
def tables(device):
    """The tables built (policy 'on'); the device's policy restored after."""
    before = device.ff_info()["policy"]
    info = device.set_ff_tables("on")
    yield info
    device.set_ff_tables(before)


@pytest.fixture(scope="module")
def states():
    rng = np.random.default_rng(7)
    edge = np.array([0, 1, 2**31, 2**32 - 1, 0xDEADBEEF], dtype=np.uint32)
    return np.concatenate([edge, rng.integers(0, 2**32, size=1 << 16, dtype=np.uint64).astype(np.uint32)])


def test_numpy_wang_matches_oracle(oracle, states):
    got = wang_np(states[:256])
    assert [int(v) for v in got] == [oracle.wang32(int(s)) for s in states[:256]]


def test_one_dead_step(device, states):
    t1, t2 = json.load(open(os.path.join(GOLD, "kat.json")))["which_thresholds"]
    got = device.eval_primitive(6, states)
    assert np.array_equal(got, dead_np(states, np.uint32(t1), np.uint32(t2)))


@pytest.mark.parametrize("kind,steps", [(4, 16), (5, 32)])
def test_jump_tables(device, tables, states, kind, steps):
    t1, t2 = json.load(open(os.path.join(GOLD, "kat.json")))["which_thresholds"]
    want = states.copy()
    for _ in range(steps):
        want = dead_np(want, np.uint32(t1), np.uint32(t2))
    got = device.eval_primitive(kind, states)
    assert np.array_equal(got, want)


def test_direct_table(device, tables, states):
    t1, t2 = json.load(open(os.path.join(GOLD, "kat.json")))["which_thresholds"]
    r = tables["direct_first"]
    assert tables["direct_count"] > 0 and r > 0
    want = states.copy()
    for _ in range(r):
        want = dead_np(want, np.uint32(t1), np.uint32(t2))
    assert np.array_equal(device.eval_primitive(7, states), want)


def test_policy_on_reports_setup(device, tables):
    i = device.ff_info()
    assert i["policy"] == "on" and i["built"] == 2
    assert i["bytes"] == (i["chain_tables"] + i["direct_count"]) * (4 << 32)
    assert i["chain_tables"] == 4 and i["build_ms"] > 0 and i["alloc_ms"] > 0
    assert 0 < i["auto_samples"] < i["auto_samples_direct"]


def test_bad_policy(device):
    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd._lib import check

    with pytest.raises(rtp.RtpError):
        check(rtp.load().rtp_set_ff_tables(device.handle, 7))
