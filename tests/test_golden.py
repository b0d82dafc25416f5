"""Committed golden fixtures (tests/golden/, made by tools/make_golden.py from
the oracle).  CPU: the oracle still reproduces them (guards the checker
itself).  GPU: the HIP path reproduces them bit-for-bit."""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import pytest

from _util import assert_render_equal

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RENDERS = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.npz")))


def _load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def test_fixtures_present():
    assert {"c1_full", "c2_subset", "c3_subset", "c4_subset", "glass_subset", "glass2_subset",
            "c5_shard3_subset"} <= set(RENDERS)


def test_kat_json(oracle):
    kat = json.load(open(os.path.join(GOLD, "kat.json")))
    for k, v in kat["wang32"].items():
        assert oracle.wang32(int(k)) == v
    for s, vals in kat["randf"].items():
        got, _ = oracle.randf_stream(int(s), len(vals))
        assert [float(g).hex() for g in np.float32(got)] == vals
    sc = oracle.cornell_box(0)
    assert [float(x).hex() for x in sc.points_np().reshape(-1)] == kat["scene_points_hex"]
    assert sc.quad_ids_np().tolist() == kat["scene_quad_ids"]
    for (nx, ny) in [(800, 800), (200, 200), (1920, 1080)]:
        cam = oracle.camera_setup(nx, ny)
        assert [float(x).hex() for x in cam] == kat[f"camera_{nx}x{ny}_hex"]
    L = oracle.lib()
    for p, v in kat["sinf"].items():
        assert float(np.float32(L.rtpo_sinf(float.fromhex(p)))).hex() == v
    for p, v in kat["cosf"].items():
        assert float(np.float32(L.rtpo_cosf(float.fromhex(p)))).hex() == v


def test_product_scene_matches_kat():
    import raytracingtherestofyourlife_amd as rtp

    kat = json.load(open(os.path.join(GOLD, "kat.json")))
    cb = rtp.CornellBox(0)
    cb.buildDataSet()
    assert [float(x).hex() for x in cb.coord.reshape(-1)] == kat["scene_points_hex"]
    assert cb.ds.cellset.quad_points.tolist() == [r[1:] for r in kat["scene_quad_ids"]]


@pytest.mark.parametrize("name", RENDERS)
def test_oracle_reproduces_fixture(oracle, name):
    g = _load(name)
    sc = oracle.cornell_box(int(g["variant"]))
    nx, ny = int(g["nx"]), int(g["ny"])
    cam = oracle.camera_setup(nx, ny)
    assert np.array_equal(cam.view(np.uint32), g["camera"].view(np.uint32))
    pix = g["pixels"] if name == "c1_full" else g["pixels"][:48]
    sel = np.searchsorted(g["pixels"], pix)
    got = oracle.render_pixels(sc, cam, nx, ny, int(g["spp"]), int(g["depth"]), pix, seed_base=int(g["seed_base"]))
    want = (np.c_[g["rgb"][sel], np.zeros(len(sel), np.float32)], g["final_seed"][sel], g["live"][sel])
    assert_render_equal(got, want, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", RENDERS)
def test_hip_reproduces_fixture(device, name):
    import raytracingtherestofyourlife_amd as rtp

    g = _load(name)
    device.set_cornell_box(int(g["variant"]))
    nx, ny = int(g["nx"]), int(g["ny"])
    got = device.render_pixels(rtp.default_camera(), nx, ny, int(g["spp"]), int(g["depth"]), g["pixels"],
                               seed_base=int(g["seed_base"]))[:3]
    want = (np.c_[g["rgb"], np.zeros(len(g["pixels"]), np.float32)], g["final_seed"], g["live"])
    assert_render_equal(got, want, name)
