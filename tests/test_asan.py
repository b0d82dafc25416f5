"""Host AddressSanitizer + UBSan over the library's host code (VERDICT r05
item 2, ADVICE r05: rtp_set_scene once read the scene's octant mask from
freed memory).  build.build_asan() compiles every source of librtp with
-Xarch_host -fsanitize=address,undefined (device code unchanged) and links the
test drivers of tests/cpp against those objects.

CPU: the shim's checks (tests/cpp/shim_check.cpp) and the host helpers of the
C ABI run sanitized; rtp_create fails loudly without a device.
GPU: scene replacements Cornell -> C3 sphere BVH (host SAH and device LBVH)
-> Cornell with a render after each, and the octant mask copied back from the
device scene the kernels read."""
from __future__ import annotations

import os
import subprocess

import pytest

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def asan_programs():
    from raytracingtherestofyourlife_amd import build

    return {os.path.basename(e): e for e in build.build_asan()}


def _run(exe, *args, timeout=120):
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout, env=ENV)


def test_shim_check_sanitized(asan_programs, tmp_path):
    r = _run(asan_programs["shim_check"], str(tmp_path / "s.pnm"))
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip() == "OK"
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a HIP device is present (the GPU test covers it)")
def test_scene_entry_points_sanitized_without_device(asan_programs, tmp_path):
    r = _run(asan_programs["asan_scene"], str(tmp_path / "a.pnm"))
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip() == "OK nodev"


@pytest.mark.gpu
def test_scene_replacement_sanitized(asan_programs, tmp_path):
    r = _run(asan_programs["asan_scene"], str(tmp_path / "a.pnm"), timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip() == "OK gpu"
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
