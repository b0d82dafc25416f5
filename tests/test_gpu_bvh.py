"""The device LBVH builder (csrc/rtp_bvh_gpu.hip) against
the host binned-SAH builder and the oracle's brute-force closest hit.  The
closest hit is the (t, index) minimum whatever the tree, so renders must be
bit-identical with either builder (rgb, final RNG state, live bounces)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from _util import assert_render_equal, set_scene_from_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rtp():
    import raytracingtherestofyourlife_amd as m

    return m


def _random_sphere_scene(oracle, n, seed):
    """The C3 walls + light (variant 3) with n random spheres: sphere 0 the
    glass light-sphere target at (190,90,190)/555, the rest lambertian or
    glass, radius 3..15 (/555), centres inside the box."""
    sc = oracle.cornell_box(3)
    rng = np.random.default_rng(seed)
    pts = sc.points_np()[: 6 * 4]
    r = rng.uniform(3, 15, n).astype(np.float32)
    c = (r[:, None] + (555 - 2 * r[:, None]) * rng.uniform(0, 1, (n, 3))).astype(np.float32)
    c[0], r[0] = (190, 90, 190), 90
    mat = np.where(rng.uniform(0, 1, n) < 0.8, rng.integers(0, 3, n), 4).astype(np.int32)
    mat[0] = 4
    tex = np.where(mat == 4, 0, mat).astype(np.int32)
    centres = (c.astype(np.float64) / 555.0).astype(np.float32)
    radii = (r.astype(np.float64) / 555.0).astype(np.float32)
    return sc, pts, centres, radii, mat, tex


def _upload(device, sc, pts, centres, radii, mat, tex):
    arr = np.ctypeslib.as_array
    nq = sc.n_quads
    allp = np.concatenate([pts, centres]).astype(np.float32)
    sp = np.arange(len(pts), len(pts) + len(centres), dtype=np.int32)
    device.set_scene(allp, sc.quad_ids_np()[:, 1:], arr(sc.quad_mat)[:nq], arr(sc.quad_tex)[:nq], sp, radii, mat, tex,
                     arr(sc.mat_type)[: sc.n_mat], arr(sc.tex_type)[: sc.n_tex_type], arr(sc.tex)[: sc.n_tex],
                     tuple(sc.light_box_pointids[1:5]), int(sp[0]), sc.ior)


def _render(device, rtp, nx, ny, spp, depth, pixels):
    return device.render_pixels(rtp.default_camera(), nx, ny, spp, depth, pixels)[:3]


def test_gpu_lbvh_matches_oracle_2000_spheres(rtp, oracle, device, monkeypatch):
    """2000 spheres (the oracle's brute-force closest hit): the device-built
    tree renders bit-exact."""
    sc, pts, c, r, mat, tex = _random_sphere_scene(oracle, 2000, 5)
    # the same scene as an oracle Scene (<= RTPO_MAX_SPHERES)
    k0 = 6 * 4
    for i, (ci, ri, mi, ti) in enumerate(zip(c, r, mat, tex)):
        sc.points[k0 + i][:] = [float(v) for v in ci]
        sc.sphere_point[i] = k0 + i
        sc.sphere_radius[i] = float(ri)
        sc.sphere_mat[i] = int(mi)
        sc.sphere_tex[i] = int(ti)
    sc.n_points = k0 + len(c)
    sc.n_spheres = len(c)
    sc.light_sphere_point = k0
    nx = ny = 256
    pix = np.sort(np.random.default_rng(3).choice(nx * ny, 512, replace=False)).astype(np.int64)
    want = oracle.render_pixels(sc, oracle.camera_setup(nx, ny), nx, ny, 8, 50, pix)
    monkeypatch.setenv("RTP_BVH_BUILD", "gpu")
    set_scene_from_oracle(device, sc)
    assert_render_equal(_render(device, rtp, nx, ny, 8, 50, pix), want, "gpu-built BVH, 2000 spheres")


@pytest.mark.parametrize("n", [20000, 200000])
def test_gpu_lbvh_matches_host_sah(rtp, oracle, device, monkeypatch, n):
    """Large scenes: the device LBVH and the host SAH tree render the same bits."""
    scene = _random_sphere_scene(oracle, n, 11)
    nx = ny = 512
    pix = np.sort(np.random.default_rng(4).choice(nx * ny, 2048, replace=False)).astype(np.int64)
    out = {}
    for build in ("host", "gpu"):
        monkeypatch.setenv("RTP_BVH_BUILD", build)
        _upload(device, *scene)
        out[build] = _render(device, rtp, nx, ny, 4, 50, pix)
    assert_render_equal(out["gpu"], out["host"], f"gpu vs host BVH, {n} spheres")


def test_gpu_lbvh_c3_golden(rtp, device, monkeypatch):
    """The C3 golden subset (1000 spheres, 2048^2, 256 spp) with the device-built tree."""
    here = os.path.dirname(os.path.abspath(__file__))
    g = np.load(os.path.join(here, "golden", "c3_subset.npz"), allow_pickle=False)
    monkeypatch.setenv("RTP_BVH_BUILD", "gpu")
    device.set_cornell_box(3)
    # every direction octant walks its own near-to-far copy on the device-built
    # tree too (the mask was once cleared to 0 on this branch, so
    # every ray walked copy 0 -- same bits, slower walks)
    assert device.sphere_walk_oct_mask() == 7
    pix = g["pixels"][:256]
    got = device.render_pixels(rtp.default_camera(), int(g["nx"]), int(g["ny"]), int(g["spp"]), int(g["depth"]), pix)
    want = (np.concatenate([g["rgb"][:256], np.zeros((256, 1), np.float32)], 1), g["final_seed"][:256], g["live"][:256])
    assert_render_equal(got[:3], want, "C3 golden, gpu-built BVH")


def _oracle_scene(oracle, n, seed):
    sc, pts, c, r, mat, tex = _random_sphere_scene(oracle, n, seed)
    k0 = 6 * 4
    for i, (ci, ri, mi, ti) in enumerate(zip(c, r, mat, tex)):
        sc.points[k0 + i][:] = [float(v) for v in ci]
        sc.sphere_point[i] = k0 + i
        sc.sphere_radius[i] = float(ri)
        sc.sphere_mat[i] = int(mi)
        sc.sphere_tex[i] = int(ti)
    sc.n_points = k0 + len(c)
    sc.n_spheres = len(c)
    sc.light_sphere_point = k0
    return sc


def test_lds_walk_matches_oracle_900_spheres(rtp, oracle, device, monkeypatch):
    """900 spheres: the LDS walk's tree (opt-in; leaves <= kLdsWalkLeaf, 8
    octant copies + leaf spheres) fits the block's LDS, so renders take
    rtp_render_pool_lds -- against the oracle's brute-force closest hit,
    bit-exact.  1200 spheres do not fit: those renders walk the global tree."""
    sc = _oracle_scene(oracle, 900, 21)
    nx = ny = 256
    pix = np.sort(np.random.default_rng(8).choice(nx * ny, 512, replace=False)).astype(np.int64)
    want = oracle.render_pixels(sc, oracle.camera_setup(nx, ny), nx, ny, 8, 50, pix)
    monkeypatch.setenv("RTP_BVH_BUILD", "host")
    monkeypatch.setenv("RTP_BVH_LDS", "1")
    set_scene_from_oracle(device, sc)
    assert device.sphere_walk() == "lds"
    assert_render_equal(_render(device, rtp, nx, ny, 8, 50, pix), want, "LDS walk, 900 spheres")
    set_scene_from_oracle(device, _oracle_scene(oracle, 1200, 21))
    assert device.sphere_walk() == "global"
    assert device.sphere_walk_oct_mask() == 7
    device.set_cornell_box(0)
    assert device.sphere_walk() == "scan"
    assert device.sphere_walk_oct_mask() == -1


def test_lds_walk_equals_global_walk_c3(rtp, device, monkeypatch):
    """The C3 scene through the LDS walk (RTP_BVH_LDS=1: its tree fits) and
    the global threaded walk (the default), on a pixel list and through the
    tile-deal instance: the same bits."""
    import torch

    from raytracingtherestofyourlife_amd import shard

    nx = ny = 128
    cam = rtp.default_camera()
    ids = shard.tile_pixels(nx, ny, 1, 3)
    out = {}
    for mode in ("lds", "global"):
        monkeypatch.setenv("RTP_BVH_LDS", "1" if mode == "lds" else "0")
        device.set_cornell_box(3)
        assert device.sphere_walk() == mode
        out[mode] = _render(device, rtp, nx, ny, 8, 50, ids)
        t = torch.zeros((ids.size, 4), dtype=torch.float32, device="cuda")
        device.render_tiles_device(cam, nx, ny, 8, 50, t.data_ptr(), 1, 3, timed=True)
        out[mode + "_tiles"] = (t.cpu().numpy(), None, None)
    monkeypatch.delenv("RTP_BVH_LDS")
    device.set_cornell_box(0)
    assert_render_equal(out["lds"], out["global"], "C3: LDS walk vs global walk")
    assert_render_equal(out["lds_tiles"], out["lds"], "C3: LDS walk, tile-deal instance vs pixel list")
    assert_render_equal(out["global_tiles"], out["global"], "C3: global walk, tile-deal instance vs pixel list")


@pytest.mark.parametrize("walk", ["lds", "global"])
@pytest.mark.parametrize("drop", [0, 1, 3, 8])
def test_dropped_top_nodes_match_oracle(rtp, oracle, device, monkeypatch, drop, walk):
    """Inner nodes above depth `drop` left out of the walks' arrays
    (rtp_host.cpp bvh_flatten, RTP_BVH_DROP): their boxes count as hit, so the
    walk visits more nodes but finds the same (t, index) minimum -- bit-exact
    against the oracle's brute-force closest hit (900 spheres, both walks; 8
    drops most of the tree's inner levels)."""
    sc = _oracle_scene(oracle, 900, 33)
    nx = ny = 128
    pix = np.sort(np.random.default_rng(9).choice(nx * ny, 384, replace=False)).astype(np.int64)
    want = oracle.render_pixels(sc, oracle.camera_setup(nx, ny), nx, ny, 4, 50, pix)
    monkeypatch.setenv("RTP_BVH_BUILD", "host")
    monkeypatch.setenv("RTP_BVH_DROP", str(drop))
    monkeypatch.setenv("RTP_BVH_LDS", "1" if walk == "lds" else "0")
    set_scene_from_oracle(device, sc)
    assert device.sphere_walk() == walk
    assert_render_equal(_render(device, rtp, nx, ny, 4, 50, pix), want,
                        f"sphere BVH ({walk} walk) without its top {drop} levels")
    monkeypatch.delenv("RTP_BVH_DROP")
    monkeypatch.delenv("RTP_BVH_LDS")
    device.set_cornell_box(0)
