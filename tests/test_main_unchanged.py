"""The reference's own main.cc and CornellBox.cpp, compiled UNCHANGED against
librtp.so (raytracingtherestofyourlife_amd/build.py build_main_unchanged:
both read from the reference tree, their VTK-m and reference includes
resolved by the same-named headers of include/vtkm_compat over
include/rtp/vtkm_compat.hpp; CornellBox.h and pathtracing/vec3.h are the
reference's own) -- north_star's "drops into main.cc unchanged" (SURVEY.md
8(b)).

CPU: they build where the reference is present; the reference's CornellBox,
built by its own code over the shim, equals the library's scene bit for bit
(points, quads, sphere, tables, the point field and the quad cell ids:
tests/cpp/scene_unchanged_check.cpp); without a HIP device main_cc fails
loudly (the mapper's device error, no image).  The scene check tests the
boundary (the reference's scene code through our API builds our scene); it
does not pin the oracle -- a build over VTK-m stand-ins is not a reference
build, and the oracle's parity claims rest on tests/golden alone.
GPU: its path mode writes the oracle's C1 image byte for byte (main.cc's own
NormalizeFunctor through vtkm::cont::Algorithm::Transform and its own save());
its -direct mode writes direct/depth/normals/albedo.pnm equal to the oracle's
quad-mapper renders."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from raytracingtherestofyourlife_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def main_cc():
    exe = build.build_main_unchanged()
    if exe is None:
        exe = build.MAIN_UNCHANGED
        if not os.path.exists(exe):
            pytest.skip("the reference's main.cc is absent and no prebuilt examples/main_cc exists")
    return exe


def test_main_cc_is_built_from_the_reference_file(main_cc):
    if not os.path.exists(build.REFERENCE_MAIN):
        pytest.skip("reference absent (GPU box): the binary was built in the container")
    # the compat headers are ours; the source is the reference's file, unmodified
    compat = os.path.join(ROOT, "include", "vtkm_compat")
    for h in ("MapperPathTracer.h", "View3D.h", "MapperQuad.h", "vtkm/cont/Algorithm.h",
              "vtkm/cont/DataSetBuilderExplicit.h", "pathtracing/SphereExtractor.h", "vtkm/Transform3D.h"):
        assert os.path.exists(os.path.join(compat, h))
    # the reference's own CornellBox.h and sources; no copy of them in the repo
    for f in ("CornellBox.h", "main.cc", "CornellBox.cpp"):
        assert not os.path.exists(os.path.join(compat, f)) and not os.path.exists(os.path.join(ROOT, f))
    assert os.path.getmtime(main_cc) >= os.path.getmtime(build.REFERENCE_MAIN)


def test_reference_cornellbox_equals_the_library_scene(main_cc):
    if not os.path.exists(build.SCENE_CHECK):
        pytest.skip("tests/cpp/scene_unchanged_check was not built (reference absent)")
    r = subprocess.run([build.SCENE_CHECK], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == "OK"


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a HIP device is present")
def test_main_cc_fails_loudly_without_device(main_cc, tmp_path):
    r = subprocess.run([main_cc, "-x", "8", "-y", "8"], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "no HIP device" in r.stderr
    assert not (tmp_path / "output.pnm").exists()


def _pnm_bytes(rgb: np.ndarray, nx: int, ny: int) -> bytes:
    """save() of main.cc:325-384 restated in numpy (test-side checker)."""
    c = rgb.astype(np.float32)
    bad = np.isnan(c).any(axis=1)
    c = np.where(bad[:, None], np.float32(0), c)
    q = np.trunc(255.99 * c.astype(np.float64)).astype(np.int64)
    lines = [f"P3\n{nx} {ny} 255"] + [f"{a} {b} {d}" for a, b, d in q]
    return ("\n".join(lines) + "\n").encode()


@pytest.mark.gpu
def test_main_cc_path_mode_writes_the_c1_golden(main_cc, oracle, tmp_path):
    z = np.load(os.path.join(ROOT, "tests", "golden", "c1_full.npz"), allow_pickle=False)
    nx, ny, spp, depth = int(z["nx"]), int(z["ny"]), int(z["spp"]), int(z["depth"])
    r = subprocess.run([main_cc, "-x", str(nx), "-y", str(ny), "-samplecount", str(spp), "-raydepth", str(depth)],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Elapsed time" in r.stdout
    want = np.zeros((nx * ny, 4), dtype=np.float32)
    want[:, :3] = z["rgb"]
    want = oracle.normalize(want, spp)
    assert (tmp_path / "output.pnm").read_bytes() == _pnm_bytes(want[:, :3], nx, ny)


@pytest.mark.gpu
def test_main_cc_direct_mode_matches_the_oracle(main_cc, oracle, tmp_path):
    import raytracingtherestofyourlife_amd as rtp

    nx, ny = 40, 32
    r = subprocess.run([main_cc, "-x", str(nx), "-y", str(ny), "-direct"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    sc = oracle.cornell_box(0)
    cmap = oracle.sample_color_table()
    cam = oracle.direct_setup(sc, nx, ny)
    for name, aov in (("direct", 1), ("normals", 2), ("albedo", 4)):
        want, depth = oracle.render_direct(sc, cam, aov, cmap=cmap)
        rtp.save_pnm(str(tmp_path / "want.pnm"), want, nx, ny)
        assert (tmp_path / f"{name}.pnm").read_bytes() == (tmp_path / "want.pnm").read_bytes(), name
    rtp.save_depth_pnm(str(tmp_path / "want.pnm"), depth, nx, ny)
    assert (tmp_path / "depth.pnm").read_bytes() == (tmp_path / "want.pnm").read_bytes()


@pytest.mark.gpu
def test_main_cc_hemisphere_views_match_the_oracle(main_cc, oracle, tmp_path):
    """main.cc's -hemisphere mode (generateHemisphere, main.cc:504-561, and
    generate(), :387-429) run unchanged: one output-<phi>-<theta>.pnm per view,
    the camera moved on its sphere by main.cc's own float arithmetic (its
    cos/sin resolve to the float overloads: the binary calls sincosf), the
    canvas reused across views.  Each image is main.cc's save() of the
    oracle's render of that view."""
    from test_cpp_host import _hemisphere_plan_py

    nx, ny, spp, depth = 24, 16, 3, 6
    r = subprocess.run([main_cc, "-hemisphere", "-phicount", "2", "-thetacount", "2", "-x", str(nx), "-y", str(ny),
                        "-samplecount", str(spp), "-raydepth", str(depth)], cwd=tmp_path, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    views = _hemisphere_plan_py(2, 2)
    assert sorted(p.name for p in tmp_path.glob("output-*.pnm")) == sorted(f"output-{n}.pnm" for n, _ in views)
    sc = oracle.cornell_box(0)
    for name, pos_bits in views:
        pos = np.array(pos_bits, dtype=np.uint32).view(np.float32)
        cam = oracle.camera_setup(nx, ny, position=pos)
        want, _, _ = oracle.render_pixels(sc, cam, nx, ny, spp, depth, np.arange(nx * ny, dtype=np.int64))
        want = oracle.normalize(want, spp)
        assert (tmp_path / f"output-{name}.pnm").read_bytes() == _pnm_bytes(want[:, :3], nx, ny), name


@pytest.mark.gpu
def test_main_cc_hemisphere_direct_views_match_the_oracle(main_cc, oracle, tmp_path):
    """-hemisphere -direct: direct-, depth-, normals- and albedo-<phi>-<theta>.pnm
    per view (main.cc:402-421), each the oracle's quad-mapper render of that view."""
    import raytracingtherestofyourlife_amd as rtp
    from test_cpp_host import _hemisphere_plan_py

    nx, ny = 20, 18
    r = subprocess.run([main_cc, "-hemisphere", "-phicount", "2", "-thetacount", "2", "-x", str(nx), "-y", str(ny),
                        "-direct"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    sc = oracle.cornell_box(0)
    cmap = oracle.sample_color_table()
    for name, pos_bits in _hemisphere_plan_py(2, 2):
        pos = np.array(pos_bits, dtype=np.uint32).view(np.float32)
        cam = oracle.direct_setup(sc, nx, ny, position=pos, clip=(1.0, 5.0))  # main.cc:519
        for prefix, aov in (("direct", 1), ("normals", 2), ("albedo", 4)):
            want, dep = oracle.render_direct(sc, cam, aov, cmap=cmap)
            rtp.save_pnm(str(tmp_path / "want.pnm"), want, nx, ny)
            assert (tmp_path / f"{prefix}-{name}.pnm").read_bytes() == (tmp_path / "want.pnm").read_bytes(), (prefix, name)
        rtp.save_depth_pnm(str(tmp_path / "want.pnm"), dep, nx, ny)
        assert (tmp_path / f"depth-{name}.pnm").read_bytes() == (tmp_path / "want.pnm").read_bytes(), name
