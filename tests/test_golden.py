"""Committed golden fixtures (tests/golden/, made by tools/make_golden.py from
the oracle).  CPU: the oracle still reproduces them (guards the checker
itself).  GPU: the HIP path reproduces them bit-for-bit."""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import pytest

from _util import assert_render_equal, load_full_frame, rmse_normalized, same_bits_or_both_nan, sha256_u32

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FULL_FRAMES = ["c2_full"]  # whole frames (byte-plane format, tools/make_golden.py full_frame_fixture)
RENDERS = sorted(n for n in (os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.npz")))
                 if n not in FULL_FRAMES and not n.endswith("_digest")  # (digest fixtures: test_gpu_fullsize)
                 and not n.startswith("c5_reduced"))  # (reduced-frame fixtures: below)
REDUCED = ["c5_reduced", "c5_reduced_small"]


def _load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def test_fixtures_present():
    assert {"c1_full", "c2_subset", "c3_subset", "c4_subset", "glass_subset", "glass2_subset",
            "c5_shard3_subset"} <= set(RENDERS)
    assert all(os.path.exists(os.path.join(GOLD, n + ".npz")) for n in FULL_FRAMES)


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


# ---- the metric's whole frame: C2, 800x800, 1000 spp, depth 50 ----------
# (BASELINE.json metric "... per-pixel RMSE vs ref": main.cc:253-287, 317-321)


def test_c2_full_frame_fixture_is_consistent():
    g = load_full_frame(os.path.join(GOLD, "c2_full.npz"))
    nx, ny = int(g["nx"]), int(g["ny"])
    assert g["rgb"].shape == (nx * ny, 3) and (nx, ny, int(g["spp"]), int(g["depth"])) == (800, 800, 1000, 50)
    assert np.array_equal(np.flatnonzero(np.isnan(g["rgb"]).any(1)), g["nan_pixels"])
    assert g["nan_pixels"].size == 670  # NaN pixels of the reference's C2 frame are data
    # L = live bounces per sample of the whole frame (SURVEY.md 8(d) byte model)
    assert abs(int(g["live_sum"]) / (nx * ny * 1000) - 3.7066) < 1e-4
    # the two committed C2 fixtures agree where they overlap (4096 pixels)
    sub = _load("c2_subset")
    assert same_bits_or_both_nan(g["rgb"][sub["pixels"]], sub["rgb"]).all()


def test_oracle_reproduces_c2_full_frame_rows(oracle):
    """The checker reproduces a spread of the frame's pixels, NaN pixels included."""
    g = load_full_frame(os.path.join(GOLD, "c2_full.npz"))
    rng = np.random.default_rng(5)
    pix = np.sort(np.r_[rng.choice(g["rgb"].shape[0], 24, replace=False), g["nan_pixels"][:8]]).astype(np.int64)
    sc = oracle.cornell_box(0)
    cam = oracle.camera_setup(800, 800)
    assert np.array_equal(cam.view(np.uint32), g["camera"].view(np.uint32))
    rgba, _, _ = oracle.render_pixels(sc, cam, 800, 800, 1000, 50, pix)
    assert same_bits_or_both_nan(rgba[:, :3], g["rgb"][pix]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("path,tables", [("contiguous", "off"), ("contiguous", "on"), ("tiles", "on")])
def test_hip_reproduces_c2_full_frame(device, path, tables):
    """The whole C2 frame on the GPU -- the bench workload -- bit-exact against
    the oracle's frame (NaN-aware), final RNG states and live-bounce counts
    equal (SHA-256 of all 640,000), and the metric's quality gate:
    per-pixel RMSE of the normalised frame < 1e-4 (it is 0).  With the RNG
    jump tables off (every dead depth hashed) and on (include/rtp.h)."""
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard

    g = load_full_frame(os.path.join(GOLD, "c2_full.npz"))
    device.set_cornell_box(0)
    before = device.ff_info()["policy"]
    device.set_ff_tables(tables)
    try:
        _c2_full_frame(device, path, g)
    finally:
        device.set_ff_tables(before)


def _c2_full_frame(device, path, g):
    import torch

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard

    cam = rtp.default_camera()
    n = 800 * 800
    out = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
    if path == "contiguous":
        seeds = torch.zeros(n, dtype=torch.int32, device="cuda")
        live = torch.zeros(n, dtype=torch.int32, device="cuda")
        device.render_device(cam, 800, 800, 1000, 50, out.data_ptr(), seed_ptr=seeds.data_ptr(),
                             live_ptr=live.data_ptr(), timed=True)
        canvas = out.cpu().numpy()
        assert sha256_u32(seeds.cpu().numpy().view(np.uint32)) == bytes(g["seed_sha256"])
        assert sha256_u32(live.cpu().numpy().view(np.uint32)) == bytes(g["live_sha256"])
    else:  # bench.py's instance: the in-kernel 16x16 tile deal, scattered to the canvas
        device.render_tiles_device(cam, 800, 800, 1000, 50, out.data_ptr(), 0, 1, timed=True)
        canvas = np.zeros((n, 4), np.float32)
        canvas[shard.tile_pixels(800, 800, 0, 1)] = out.cpu().numpy()
    ok = same_bits_or_both_nan(canvas[:, :3], g["rgb"]).all(1)
    assert ok.all(), f"{int((~ok).sum())} of {n} pixels differ, first {np.flatnonzero(~ok)[:8].tolist()}"
    assert rmse_normalized(canvas, np.c_[g["rgb"], np.zeros(n, np.float32)], 1000) < 1e-4


def test_c4_full_digest_agrees_with_the_c4_subset():
    """tests/golden/c4_full_digest.npz (tools/make_golden_digest.py: the whole
    C4 frame from the oracle, as digests) and c4_subset16k.npz (16 384 of its
    pixels in full) come from separate oracle runs: the subset's NaN pixels
    are exactly the full frame's NaN pixels among them, and the configs agree."""
    here = os.path.dirname(os.path.abspath(__file__))
    f = os.path.join(here, "golden", "c4_full_digest.npz")
    if not os.path.exists(f):
        pytest.skip("c4_full_digest.npz not generated")
    full = np.load(f, allow_pickle=False)
    sub = np.load(os.path.join(here, "golden", "c4_subset16k.npz"), allow_pickle=False)
    for k in ("nx", "ny", "spp", "depth", "variant"):
        assert int(full[k]) == int(sub[k]), k
    assert np.array_equal(full["camera"], sub["camera"])
    nan_sub = sub["pixels"][np.isnan(sub["rgb"]).any(1)]
    assert np.array_equal(np.intersect1d(full["nan_pixels"], sub["pixels"]), np.sort(nan_sub))
    assert full["rgb_sha256"].size == 32 and full["seed_sha256"].size == 32 and full["live_sha256"].size == 32


@pytest.mark.parametrize("name", ["c5_shard3_full_digest", "c5_shard3_band_digest"])
def test_c5_share_digest_agrees_with_the_2048spp_fixture(name):
    """A C5 rank-share digest (tools/make_golden_digest.py: rank 3 of 8's
    share over the whole canvas or its leading band) and c5_shard3_2048spp.npz
    (1024 of the share's pixels in full, bench.py's shard check) come from
    separate oracle runs: same configuration, and among the fixture's pixels
    inside the digest's range the NaN pixels are the same."""
    f = os.path.join(GOLD, name + ".npz")
    if not os.path.exists(f):
        pytest.skip(f"{name}.npz not generated")
    d = np.load(f, allow_pickle=False)
    sub = _load("c5_shard3_2048spp")
    for k in ("nx", "ny", "spp", "depth", "variant", "seed_base"):
        assert int(d[k]) == int(sub[k]), k
    assert np.array_equal(d["camera"], sub["camera"])
    n = int(d["pixel_count"]) if "pixel_count" in d.files else int(d["nx"]) * int(d["ny"])
    inside = sub["pixels"][sub["pixels"] < n]
    assert inside.size > 0
    nan_sub = sub["pixels"][np.isnan(sub["rgb"]).any(1) & (sub["pixels"] < n)]
    assert np.array_equal(np.intersect1d(d["nan_pixels"], inside), np.sort(nan_sub))
    assert d["nan_pixels"].size == 0 or int(d["nan_pixels"].max()) < n


def test_c5_band_digest_is_the_full_digests_leading_band():
    """The band fixture (the first 1080 rows) and the whole-canvas fixture
    come from the same oracle chunks: their NaN pixels agree on the band."""
    fs = [os.path.join(GOLD, n + ".npz") for n in ("c5_shard3_full_digest", "c5_shard3_band_digest")]
    if not all(os.path.exists(f) for f in fs):
        pytest.skip("C5 share digests not generated")
    full, band = (np.load(f, allow_pickle=False) for f in fs)
    n = int(band["pixel_count"])
    assert n == int(full["nx"]) * int(full["ny"]) // 2
    assert np.array_equal(full["nan_pixels"][full["nan_pixels"] < n], band["nan_pixels"])
    assert int(band["live_sum"]) < int(full["live_sum"])


def _reduced_cases(g):
    from raytracingtherestofyourlife_amd.shard import sample_batches

    npix = int(g["nx"]) * int(g["ny"])
    for n in g["worlds"]:
        for b in sample_batches(int(g["spp"]), int(n), npix):
            yield int(n), b


@pytest.mark.parametrize("name", REDUCED)
def test_reduced_fixture_is_its_shards_summed(name):
    """tools/make_golden_reduced.py: reduced_N is the rank-order float32 sum
    of shards_N, and the shards' final seeds differ per rank (derived streams)."""
    g = _load(name)
    for n in g["worlds"]:
        sh = g[f"shards_{n}"]
        acc = sh[0].copy()
        for x in sh[1:]:
            acc = acc + x
        same = (acc.view(np.uint32) == g[f"reduced_{n}"].view(np.uint32)) | (np.isnan(acc) & np.isnan(g[f"reduced_{n}"]))
        assert same.all()
        assert len({int(s[0]) for s in g[f"final_seed_{n}"]}) == n


@pytest.mark.parametrize("name", REDUCED)
def test_oracle_reproduces_reduced_fixture(oracle, name):
    """A few pixels of every rank's shard re-rendered by the oracle."""
    g = _load(name)
    nx, ny = int(g["nx"]), int(g["ny"])
    sc = oracle.cornell_box(int(g["variant"]))
    cam = oracle.camera_setup(nx, ny)
    k = 4 if nx * ny > 10**6 else 24
    for n, b in _reduced_cases(g):
        if b.rank not in (0, n - 1):
            continue
        got = oracle.render_pixels(sc, cam, nx, ny, b.spp, int(g["depth"]), g["pixels"][:k], seed_base=b.seed_base)
        want = (np.c_[g[f"shards_{n}"][b.rank][:k], np.zeros(k, np.float32)], g[f"final_seed_{n}"][b.rank][:k],
                g[f"live_{n}"][b.rank][:k])
        assert_render_equal(got, want, f"{name} N={n} rank {b.rank}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", REDUCED)
def test_hip_reproduces_reduced_fixture(device, name):
    """Every rank's shard of every world size, all fixture pixels, bit-exact
    (C5: 1024 pixels x 16384 spp per N)."""
    import raytracingtherestofyourlife_amd as rtp

    g = _load(name)
    device.set_cornell_box(int(g["variant"]))
    nx, ny = int(g["nx"]), int(g["ny"])
    m = len(g["pixels"])
    for n, b in _reduced_cases(g):
        got = device.render_pixels(rtp.default_camera(), nx, ny, b.spp, int(g["depth"]), g["pixels"],
                                   seed_base=b.seed_base)[:3]
        want = (np.c_[g[f"shards_{n}"][b.rank], np.zeros(m, np.float32)], g[f"final_seed_{n}"][b.rank],
                g[f"live_{n}"][b.rank])
        assert_render_equal(got, want, f"{name} N={n} rank {b.rank}")
