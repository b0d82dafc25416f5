"""Generate the committed golden fixtures under tests/golden/ from the CPU
oracle (oracle/rtp_oracle.c).  The reference itself cannot be built here (it
needs VTK-m), so these are known-answer vectors of the restatement; see
DESIGN.md "Parity".

    python tools/make_golden.py            # all fixtures (a few minutes, 8 cores)
    python tools/make_golden.py c3_subset  # only the named fixtures
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_ctypes as oc  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def hexf(a):
    return [float(x).hex() for x in np.asarray(a, dtype=np.float32).reshape(-1)]


def subset(n_total, k, seed):
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(n_total, size=k, replace=False)).astype(np.int64)


ONLY = set(sys.argv[1:])


def render_fixture(name, variant, nx, ny, spp, depth, pixels=None, seed_base=0, camera=None):
    if ONLY and name not in ONLY:
        return
    t = time.time()
    sc = oc.cornell_box(variant)
    cam = oc.camera_setup(nx, ny, **(camera or {}))
    if pixels is None:
        pixels = np.arange(nx * ny, dtype=np.int64)
    rgba, seeds, live = oc.render_pixels(sc, cam, nx, ny, spp, depth, pixels, seed_base=seed_base)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), variant=variant, nx=nx, ny=ny, spp=spp, depth=depth,
                        seed_base=seed_base, camera=cam, pixels=pixels, rgb=rgba[:, :3], final_seed=seeds,
                        live=live)
    print(f"{name}: {pixels.size} px x {spp} spp x depth {depth}: {time.time() - t:.1f}s, "
          f"L={live.sum() / (pixels.size * spp):.4f}, nan_px={int(np.isnan(rgba[:, :3]).any(1).sum())}")


def full_frame_fixture(name, variant, nx, ny, spp, depth):
    """A whole frame at full S x D (the metric's own image, main.cc:253-287,
    317-321): the un-normalised rgb sums of every pixel, stored as the four
    byte planes of the float32 bit patterns (deflate packs the exponent planes
    well); the final seeds and live-bounce counts as SHA-256 digests plus
    their sums (16 MB of near-random words otherwise)."""
    if ONLY and name not in ONLY:
        return
    import hashlib

    t = time.time()
    sc = oc.cornell_box(variant)
    cam = oc.camera_setup(nx, ny)
    pixels = np.arange(nx * ny, dtype=np.int64)
    rgba, seeds, live = oc.render_pixels(sc, cam, nx, ny, spp, depth, pixels)
    rgb = np.ascontiguousarray(rgba[:, :3], dtype=np.float32)
    planes = rgb.view(np.uint8).reshape(-1, 4).T.copy()  # [byte][value]
    nan_px = np.flatnonzero(np.isnan(rgb).any(1)).astype(np.int64)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), variant=variant, nx=nx, ny=ny, spp=spp, depth=depth,
                        camera=cam, rgb_planes=planes, nan_pixels=nan_px,
                        seed_sha256=np.frombuffer(hashlib.sha256(seeds.astype("<u4").tobytes()).digest(), np.uint8),
                        live_sha256=np.frombuffer(hashlib.sha256(live.astype("<u4").tobytes()).digest(), np.uint8),
                        seed_sum=np.uint64(seeds.astype(np.uint64).sum()), live_sum=np.uint64(live.astype(np.uint64).sum()))
    print(f"{name}: {nx}x{ny} x {spp} spp x depth {depth}: {time.time() - t:.1f}s, "
          f"L={live.sum() / (pixels.size * spp):.4f}, nan_px={nan_px.size}")


def direct_fixture(name, variant, nx, ny, camera=None, clip=(0.1, 5.0)):
    """-direct mode (main.cc:120-251): colour, normals, albedo and depth of
    one camera, full canvas, from the oracle's restatement."""
    if ONLY and name not in ONLY:
        return
    t = time.time()
    sc = oc.cornell_box(variant)
    cam = oc.direct_setup(sc, nx, ny, clip=clip, **(camera or {}))
    cmap = oc.sample_color_table()
    out = {}
    for key, aov in (("color", oc.AOV_COLOR), ("normals", oc.AOV_NORMALS), ("albedo", oc.AOV_ALBEDO)):
        rgba, depth = oc.render_direct(sc, cam, aov, cmap=cmap)
        out[key] = rgba
    out["depth"] = depth
    d = os.path.join(OUT, "direct")
    os.makedirs(d, exist_ok=True)
    cam_args = {k: np.asarray(v, dtype=np.float32) for k, v in (camera or {}).items()}
    np.savez_compressed(os.path.join(d, name + ".npz"), variant=variant, nx=nx, ny=ny, clip=np.float32(clip),
                        cmap=cmap, subset=np.int32([cam.sub_x0, cam.sub_y0, cam.sub_w, cam.sub_h]),
                        **{"cam_" + k: v for k, v in cam_args.items()}, **out)
    print(f"{name}: {nx}x{ny} direct, subset {cam.sub_x0},{cam.sub_y0} {cam.sub_w}x{cam.sub_h}: "
          f"{time.time() - t:.1f}s, nan depth {int(np.isnan(out['depth']).sum())}")


def main():
    os.makedirs(OUT, exist_ok=True)
    L = oc.lib()
    # --- known answers -------------------------------------------------
    kat = {"wang32": {str(x): oc.wang32(x) for x in (0, 1, 61, 639999, 2**31, 2**32 - 1)}}
    kat["randf"] = {str(s): [float(v).hex() for v in oc.randf_stream(s, 8)[0]] for s in (0, 1, 639999)}
    lo = 0
    thr = []
    for w in (2, 3):
        a, b = 0, 1 << 32
        while a < b:
            m = (a + b) // 2
            if L.rtpo_which(m) >= w:
                b = m
            else:
                a = m + 1
        thr.append(a)
    kat["which_thresholds"] = thr
    sc = oc.cornell_box(0)
    kat["scene_points_hex"] = hexf(sc.points_np())
    kat["scene_quad_ids"] = sc.quad_ids_np().tolist()
    kat["camera_800x800_hex"] = hexf(oc.camera_setup(800, 800))
    kat["camera_200x200_hex"] = hexf(oc.camera_setup(200, 200))
    kat["camera_1920x1080_hex"] = hexf(oc.camera_setup(1920, 1080))
    phis = np.float32([0.0, 0.5, 0.7853982, 1.0, 2.0, 3.1415927, 4.0, 5.5, 6.2831855])
    kat["sinf"] = {float(p).hex(): float(L.rtpo_sinf(float(p))).hex() for p in phis}
    kat["cosf"] = {float(p).hex(): float(L.rtpo_cosf(float(p))).hex() for p in phis}
    if not ONLY or "kat" in ONLY:
        with open(os.path.join(OUT, "kat.json"), "w") as f:
            json.dump(kat, f, indent=1)
    # --- renders ---------------------------------------------------------
    # C1 (BASELINE configs[0]): full image
    render_fixture("c1_full", 0, 200, 200, 10, 10)
    # C2 geometry at full spp/depth on a fixed 4096-pixel subset
    render_fixture("c2_subset", 0, 800, 800, 1000, 50, pixels=subset(800 * 800, 4096, 2))
    # C2, the metric's whole frame (bench.py's workload; ~12 min on 8 cores)
    full_frame_fixture("c2_full", 0, 800, 800, 1000, 50)
    # C4 geometry (1920x1080, 4096 spp, depth 50) on a 256-pixel subset
    render_fixture("c4_subset", 0, 1920, 1080, 4096, 50, pixels=subset(1920 * 1080, 256, 4))
    # dielectric visible: variant 1 (overlapping, NaN-heavy) and variant 2 (clean)
    render_fixture("glass_subset", 1, 256, 256, 64, 50, pixels=subset(256 * 256, 2048, 6))
    render_fixture("glass2_subset", 2, 256, 256, 256, 50, pixels=subset(256 * 256, 2048, 9))
    # sample-batch shard stream: seed_base = k*N for shard k = 3 of C5 geometry
    render_fixture("c5_shard3_subset", 0, 3840, 2160, 16, 50, pixels=subset(3840 * 2160, 512, 8),
                   seed_base=(3 * 3840 * 2160) % (1 << 32))
    # C3 (BASELINE configs[2]): 1000-sphere scene, 2048x2048, 256 spp, depth 50 (assumed)
    render_fixture("c3_subset", 3, 2048, 2048, 256, 50, pixels=subset(2048 * 2048, 1024, 12))
    # round 3: wider config-scale checks (VERDICT r02 "what's weak" #1)
    # C4 at full S x D on 16384 pixels (64x c4_subset)
    render_fixture("c4_subset16k", 0, 1920, 1080, 4096, 50, pixels=subset(1920 * 1080, 16384, 14))
    # one C5 sample-batch shard at its real length: S = 16384 over 8 GPUs = 2048 spp, shard 3
    render_fixture("c5_shard3_2048spp", 0, 3840, 2160, 2048, 50, pixels=subset(3840 * 2160, 1024, 15),
                   seed_base=(3 * 3840 * 2160) % (1 << 32))
    # C3 at full S x D on 4096 pixels (4x c3_subset)
    render_fixture("c3_subset4k", 3, 2048, 2048, 256, 50, pixels=subset(2048 * 2048, 4096, 16))
    # -direct mode (main.cc:120-251, 623-651): the default camera at the
    # reference's default canvas (128x128), a non-square canvas, a hemisphere
    # view (generate(): phi 0.4, theta 1.2566371) and a camera inside the box
    direct_fixture("direct_128", 0, 128, 128)
    direct_fixture("direct_200x120", 0, 200, 120)
    direct_fixture("direct_hemi", 0, 96, 96, camera=dict(position=np.float32([0.19573918, 0.06558621, -1.2823226])))
    direct_fixture("direct_inside", 2, 64, 80, camera=dict(position=np.float32([0.3, 0.7, 0.2]),
                                                            look_at=np.float32([0.8, 0.2, 0.9]),
                                                            view_up=np.float32([0.1, 1.0, 0.0]), fov_y=55.0))


if __name__ == "__main__":
    main()
