"""The C++ host interface (include/rtp/rendering.hpp) and the runPath driver
(examples/path_main.cpp, main.cc's path mode) built with g++ over the C ABI.

CPU: the shim's reference error behaviour and helpers (tests/cpp/shim_check),
and the driver failing loudly when no HIP device exists.
GPU: the driver's C1 image (main.cc defaults route: runPath + NormalizeFunctor
+ save) equals the oracle's golden C1 render, float buffer and PNM bytes."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def programs():
    from raytracingtherestofyourlife_amd import build

    exes = build.build_cpp()
    return {os.path.basename(e): e for e in exes}


def _no_hip_device() -> bool:
    return not os.path.exists("/dev/kfd")


def test_shim_check(programs, tmp_path):
    r = subprocess.run([programs["shim_check"], str(tmp_path / "s.pnm")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "OK"


def test_driver_out_of_scope_modes(programs):
    for flag in ("-hemisphere", "-direct"):
        r = subprocess.run([programs["rtp_path"], flag], capture_output=True, text=True, timeout=60)
        assert r.returncode == 2 and "out of scope" in r.stderr


@pytest.mark.skipif(not _no_hip_device(), reason="a HIP device is present")
def test_driver_fails_loudly_without_device(programs, tmp_path):
    r = subprocess.run([programs["rtp_path"], "-x", "8", "-y", "8", "-o", str(tmp_path / "o")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert "no HIP device" in r.stderr
    assert not (tmp_path / "o.pnm").exists()


def _pnm_bytes(rgb: np.ndarray, nx: int, ny: int) -> bytes:
    """save() of main.cc:325-384 restated in numpy (test-side checker)."""
    c = rgb.astype(np.float32)
    bad = np.isnan(c).any(axis=1)
    c = np.where(bad[:, None], np.float32(0), c)
    q = np.trunc(255.99 * c.astype(np.float64)).astype(np.int64)
    lines = [f"P3\n{nx} {ny} 255"] + [f"{a} {b} {d}" for a, b, d in q]
    return ("\n".join(lines) + "\n").encode()


@pytest.mark.gpu
def test_driver_c1_matches_golden(programs, oracle, tmp_path):
    z = np.load(os.path.join(ROOT, "tests", "golden", "c1_full.npz"), allow_pickle=False)
    nx, ny, spp, depth = int(z["nx"]), int(z["ny"]), int(z["spp"]), int(z["depth"])
    assert int(z["variant"]) == 0 and int(z["seed_base"]) == 0
    out = tmp_path / "output"
    raw = tmp_path / "out.f32"
    r = subprocess.run([programs["rtp_path"], "-x", str(nx), "-y", str(ny), "-samplecount", str(spp), "-raydepth",
                        str(depth), "-o", str(out), "-raw", str(raw)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Elapsed time" in r.stdout
    got = np.fromfile(raw, dtype=np.float32).reshape(nx * ny, 4)
    want = np.zeros((nx * ny, 4), dtype=np.float32)
    want[:, :3] = z["rgb"]
    want = oracle.normalize(want, spp)
    assert np.array_equal(got[:, :3].view(np.uint32), want[:, :3].view(np.uint32))
    assert (tmp_path / "output.pnm").read_bytes() == _pnm_bytes(want[:, :3], nx, ny)
