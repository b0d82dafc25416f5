"""The oracle's two variants -- scalar per-pixel and the stage-structured SoA
pass sequence of RenderCellsImpl -- must agree bit-for-bit (CPU only)."""
from __future__ import annotations

import numpy as np
import pytest

from _util import assert_render_equal


@pytest.mark.parametrize(
    "variant,nx,ny,spp,depth",
    [(0, 48, 48, 6, 10), (1, 40, 40, 8, 12), (0, 37, 21, 4, 7), (0, 8, 8, 2, 1), (1, 16, 16, 3, 50)],
)
def test_scalar_equals_soa(oracle, variant, nx, ny, spp, depth):
    sc = oracle.cornell_box(variant)
    cam = oracle.camera_setup(nx, ny)
    a = oracle.render_pixels(sc, cam, nx, ny, spp, depth, np.arange(nx * ny))
    b = oracle.render_soa(sc, cam, nx, ny, spp, depth, nthreads=4)
    assert_render_equal(a, b, f"v{variant} {nx}x{ny}")


def test_soa_row_window_equals_full(oracle):
    sc = oracle.cornell_box(0)
    nx, ny = 30, 20
    cam = oracle.camera_setup(nx, ny)
    full = oracle.render_soa(sc, cam, nx, ny, 3, 6, nthreads=2)
    part = oracle.render_soa(sc, cam, nx, ny, 3, 6, row_begin=5, row_end=12, nthreads=2)
    sl = slice(5 * nx, 12 * nx)
    assert_render_equal(part, (full[0][sl], full[1][sl], full[2][sl]), "row window")


def test_pixel_independence(oracle):
    """Any pixel subset renders exactly as in the full image (seed = index)."""
    sc = oracle.cornell_box(0)
    nx, ny = 50, 40
    cam = oracle.camera_setup(nx, ny)
    full = oracle.render_pixels(sc, cam, nx, ny, 4, 8, np.arange(nx * ny))
    pix = np.array([0, 7, 999, 1234, nx * ny - 1], dtype=np.int64)
    sub = oracle.render_pixels(sc, cam, nx, ny, 4, 8, pix)
    assert_render_equal(sub, (full[0][pix], full[1][pix], full[2][pix]), "subset")


def test_dielectric_variant_differs_and_scene_sizes(oracle):
    s0, s1 = oracle.cornell_box(0), oracle.cornell_box(1)
    assert (s0.n_points, s0.n_quads, s0.n_spheres) == (89, 22, 1)
    assert s0.light_sphere_point == 48 and list(s0.light_box_pointids) == [0, 8, 9, 10, 11]
    assert not np.array_equal(s0.points_np()[48], s1.points_np()[48])


def test_normalize_matches_reference_functor(oracle):
    x = np.array([[4.0, np.nan, 0.0, 9.0], [1.0, 2.0, 3.0, 0.0]], dtype=np.float32)
    got = oracle.normalize(x, 4)
    want = np.array([[1.0, 0.0, 0.0, 1.5], [0.5, np.sqrt(0.5), np.sqrt(0.75), 0.0]], dtype=np.float32)
    np.testing.assert_array_equal(got, want)
