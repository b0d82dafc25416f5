"""The closest-hit quad prefilter (rtp_kernels.hip closest_hit)
against the exact scan of every quad, ray by ray (rtp_debug_closest_hit):
the hit (t bits, primitive kind, index) must be identical for every ray.

The rays are built to sit where an approximate test could go wrong: aimed at
quad edges and corners with offsets from 0 to a few hundred ulps, leaving
surfaces (origins on the planes), grazing the planes, parallel to axes (zero
and negative-zero components), unnormalised, non-finite, far outside the
margins' coordinate range -- plus the render's own populations (camera rays,
cosine and light-directed bounces).  The fall-back rate of the ordinary
populations is also bounded, since a prefilter that falls back often would
only cost time."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def scene_quads(variant):
    import raytracingtherestofyourlife_amd as rtp

    cb = rtp.CornellBox(variant)
    ds = cb.buildDataSet()
    P = np.asarray(ds.coords, dtype=np.float32).reshape(-1, 3)
    Q = np.asarray(ds.cellset.quad_points).reshape(-1, 4)
    return P[Q]  # (nq, 4, 3): v00, v10, v11, v01


def stress_rays(verts, n, seed):
    """(n, 6) float32 rays mixing the hard populations described above."""
    rng = np.random.default_rng(seed)
    nq = len(verts)
    k = n // 8
    out = []
    # 1. origins inside the box, aimed at a point on a random quad edge or
    #    corner, then the target nudged by 0..300 ulps along random axes
    o = rng.uniform(0.01, 0.99, (k, 3)).astype(np.float32)
    q = rng.integers(0, nq, k)
    e = rng.integers(0, 4, k)
    s = rng.uniform(0, 1, k)
    s[rng.uniform(0, 1, k) < 0.2] = 0.0  # corners
    a, b = verts[q, e], verts[q, (e + 1) % 4]
    tgt = (a + s[:, None] * (b - a)).astype(np.float32)
    ulps = rng.integers(-300, 301, (k, 3)) * (rng.uniform(0, 1, (k, 3)) < 0.5)
    tgt = (tgt.view(np.int32) + ulps.astype(np.int32)).view(np.float32)
    out.append(np.concatenate([o, (tgt - o).astype(np.float32)], 1))
    # 2. origins ON a quad (the surface a bounce leaves), random directions
    q = rng.integers(0, nq, k)
    u, v = rng.uniform(0, 1, (2, k))
    v00, v10, v01 = verts[q, 0], verts[q, 1], verts[q, 3]
    o = (v00 + u[:, None] * (v10 - v00) + v[:, None] * (v01 - v00)).astype(np.float32)
    d = rng.normal(size=(k, 3)).astype(np.float32)
    out.append(np.concatenate([o, d], 1))
    # 3. grazing: one direction component tiny (down to denormal) or zero / -0
    o = rng.uniform(0.01, 0.99, (k, 3)).astype(np.float32)
    d = rng.normal(size=(k, 3)).astype(np.float32)
    ax = rng.integers(0, 3, k)
    tiny = (10.0 ** rng.uniform(-45, -1, k)).astype(np.float32)
    tiny[rng.uniform(0, 1, k) < 0.2] = 0.0
    sign = np.where(rng.uniform(0, 1, k) < 0.5, -1.0, 1.0).astype(np.float32)
    d[np.arange(k), ax] = sign * tiny
    out.append(np.concatenate([o, d], 1))
    # 4. origins exactly on a quad's plane but anywhere, and axis-parallel rays
    o = rng.uniform(-0.2, 1.2, (k, 3)).astype(np.float32)
    q = rng.integers(0, nq, k)
    ax = rng.integers(0, 3, k)
    o[np.arange(k), ax] = verts[q, 0, ax]
    d = np.zeros((k, 3), np.float32)
    d[np.arange(k), rng.integers(0, 3, k)] = np.where(rng.uniform(0, 1, k) < 0.5, -1.0, 1.0)
    mix = rng.uniform(0, 1, k) < 0.5
    d[mix] = rng.normal(size=(int(mix.sum()), 3)).astype(np.float32)
    out.append(np.concatenate([o, d], 1))
    # 5. unnormalised directions (|d| from 1e-4 to 1e3) and origins outside the box
    o = rng.uniform(-3, 4, (k, 3)).astype(np.float32)
    d = (rng.normal(size=(k, 3)) * (10.0 ** rng.uniform(-4, 3, (k, 1)))).astype(np.float32)
    out.append(np.concatenate([o, d], 1))
    # 6. beyond the margins' range (|o| or |d| > 16) and non-finite components
    o = rng.uniform(-40, 40, (k, 3)).astype(np.float32)
    d = rng.normal(size=(k, 3)).astype(np.float32)
    bad = rng.uniform(0, 1, (k, 6)) < 0.05
    r = np.concatenate([o, d], 1)
    r[bad] = rng.choice(np.array([np.nan, np.inf, -np.inf], np.float32), int(bad.sum()))
    out.append(r)
    # 7. the render's populations: camera-like rays from the eye, and bounces
    #    from random surface points toward the light quad
    eye = np.array([278, 278, -800], np.float32) / np.float32(555)
    tgt = rng.uniform(0, 1, (k, 3)).astype(np.float32)
    out.append(np.concatenate([np.broadcast_to(eye, (k, 3)), tgt - eye], 1).astype(np.float32))
    q = rng.integers(0, nq, k)
    u, v = rng.uniform(0, 1, (2, k))
    o = (verts[q, 0] + u[:, None] * (verts[q, 1] - verts[q, 0]) + v[:, None] * (verts[q, 3] - verts[q, 0]))
    lt = rng.uniform([213, 554, 227], [343, 554, 332], (k, 3)) / 555.0
    out.append(np.concatenate([o, lt - o], 1).astype(np.float32))
    return np.ascontiguousarray(np.concatenate(out, 0), dtype=np.float32)


@pytest.mark.parametrize("variant", [0, 1])
def test_gpu_prefilter_equals_exact_scan(device, variant):
    device.set_cornell_box(variant)
    verts = scene_quads(variant)
    rays = stress_rays(verts, 1 << 21, 100 + variant)
    got = device.debug_closest_hit(rays)
    bad = np.nonzero((got[:, 0:3] != got[:, 3:6]).any(1))[0]
    assert bad.size == 0, f"{bad.size} rays differ, first {rays[bad[:3]].tolist()} -> {got[bad[:3]].tolist()}"
    # the prefilter must actually engage on this scene (axis-plane quads):
    # column 6 is 0 (prefilter decided), 1 (fell back to the exact scan) or
    # 2 (prefilter off for the scene)
    assert (got[:, 6] != 2).all()
    assert (got[:, 6] == 1).mean() < 0.5


def test_gpu_prefilter_fallback_rate(device):
    """Camera and bounce rays fall back to the exact scan rarely."""
    device.set_cornell_box(0)
    verts = scene_quads(0)
    rays = stress_rays(verts, 1 << 20, 7)
    k = len(rays) // 8
    ordinary = np.concatenate([rays[6 * k:], rays[k:2 * k]])
    got = device.debug_closest_hit(ordinary)
    assert (got[:, 0:3] == got[:, 3:6]).all()
    assert (got[:, 6] != 2).all()
    assert (got[:, 6] == 1).mean() < 0.01, (got[:, 6] == 1).mean()


def test_gpu_prefilter_bvh_scene_equals_exact(device):
    """The C3 scene (1000 spheres, BVH kernel variant): quads prefiltered,
    spheres walked after them, same hit as the exact scan."""
    device.set_cornell_box(3)
    verts = scene_quads(3)
    rays = stress_rays(verts, 1 << 19, 3)
    got = device.debug_closest_hit(rays)
    assert (got[:, 0:3] == got[:, 3:6]).all()
    device.set_cornell_box(0)


def test_gpu_prefilter_with_trapezoid_in_axis_plane(device):
    """A scene with a non-parallelogram in an axis plane (a trapezoid in the
    plane z = const).  Its edge masks {1, 2, 3, 1} match no rectangle kind,
    so it is a kind-0 (general) quad, scanned exactly; the prefilter stays
    on for the axis-plane rectangles and every hit equals the exact scan's."""
    import raytracingtherestofyourlife_amd as rtp

    cb = rtp.CornellBox(0)
    ds = cb.buildDataSet()
    P = np.asarray(ds.coords, dtype=np.float32).reshape(-1, 3).copy()
    Q = np.asarray(ds.cellset.quad_points).reshape(-1, 4).copy()
    # quad 12 lies in a z-plane (e01 along x, e03 along y): move its v11
    # along x within the plane, so e21 gains an x component (a trapezoid)
    v11 = int(Q[12, 2])
    P = np.concatenate([P, P[v11:v11 + 1]], 0)
    P[-1, 0] += np.float32(0.05)
    Q[12, 2] = len(P) - 1
    device.set_scene(P, Q, cb.matIdx[0], cb.texIdx[0], ds.cellset.sphere_points, cb.SphereRadii, cb.matIdx[1],
                     cb.texIdx[1], cb.matType, cb.texType, cb.tex, cb.light_quad_points, cb.light_sphere_point,
                     cb.ior)
    try:
        verts = P[Q]
        rays = stress_rays(verts, 1 << 20, 12)
        got = device.debug_closest_hit(rays)
        bad = np.nonzero((got[:, 0:3] != got[:, 3:6]).any(1))[0]
        assert bad.size == 0, f"{bad.size} rays differ, first {rays[bad[:3]].tolist()}"
        assert (got[:, 6] != 2).all(), "prefilter switched off by one non-parallelogram quad"
    finally:
        device.set_cornell_box(0)


# ---------------------------------------------------------------- box cull --
# The rotated box of the reference scene (CornellBox.cpp: the tall box, quads
# 6..11 of the scene, turned -15 degrees about y): four vertical sides
# between y = 0 and 330/555, the bottom at 0, a cap whose corner
# (265, 333, 295)/555 is raised 3 units above the sides' top.
def box_quads(verts):
    ys = verts[:, :, 1]
    sides = [q for q in range(len(verts)) if np.unique(ys[q]).size == 2 and ys[q].min() == 0
             and np.isclose(ys[q].max(), 330 / 555)]
    cap = [q for q in range(len(verts)) if ys[q].min() > 0.5 and np.isclose(ys[q].min(), 330 / 555)]
    return sides, cap[0]


def box_rays(verts, n, seed):
    """Rays where a cull of the box's faces would be closest to wrong: aimed at the
    box's vertical edges, its top rim, the cap's corners and diagonal and the
    gap under the raised cap corner (ulp-nudged), from above, the side and
    inside; leaving its faces; grazing its sides; nearly vertical."""
    rng = np.random.default_rng(seed)
    sides, cap = box_quads(verts)
    C = verts[cap]  # v00 is the raised corner
    k = n // 8
    out = []

    def nudge(p, ulps=400):
        u = rng.integers(-ulps, ulps + 1, p.shape) * (rng.uniform(0, 1, p.shape) < 0.6)
        return (np.asarray(p, np.float32).view(np.int32) + u.astype(np.int32)).view(np.float32)

    def aimed(o, tgt):
        return np.concatenate([o, (nudge(tgt) - o).astype(np.float32)], 1)

    # 1. from anywhere in the room at points on the sides' edges (vertical
    #    edges, top rim at 330, bottom rim) and corners
    q = rng.choice(sides, k)
    e = rng.integers(0, 4, k)
    s = rng.uniform(0, 1, k)
    s[rng.uniform(0, 1, k) < 0.25] = 0.0
    a, b = verts[q, e], verts[q, (e + 1) % 4]
    out.append(aimed(rng.uniform(0.01, 0.99, (k, 3)).astype(np.float32), a + s[:, None] * (b - a)))
    # 2. from above (ceiling, light) at the cap: corners, edges, its diagonal v10-v01
    o = np.c_[rng.uniform(0.05, 0.95, k), rng.uniform(0.62, 0.999, k), rng.uniform(0.05, 0.95, k)].astype(np.float32)
    j = rng.integers(0, 4, k)
    s = rng.uniform(0, 1, k)
    s[rng.uniform(0, 1, k) < 0.3] = 0.0
    diag = rng.uniform(0, 1, k) < 0.3
    a = np.where(diag[:, None], C[1], C[j])
    b = np.where(diag[:, None], C[3], C[(j + 1) % 4])
    out.append(aimed(o, a + s[:, None] * (b - a)))
    # 3. into the gap under the raised corner: points on the two sides meeting
    #    at it, between y = 330 and 333 (and just outside the footprint)
    tgt = C[0][None, :] + rng.uniform(0, 1, (k, 1)) * (C[rng.choice([1, 3], k)] - C[0][None, :])
    tgt[:, 1] = rng.uniform(329.5, 333.5, k) / 555.0
    o = rng.uniform(0.01, 0.99, (k, 3)).astype(np.float32)
    out.append(aimed(o, tgt.astype(np.float32)))
    # 4. origins inside the box (under the cap), random directions
    lo, hi = verts[sides].reshape(-1, 3).min(0), verts[sides].reshape(-1, 3).max(0)
    o = rng.uniform(lo, hi, (k, 3)).astype(np.float32)
    out.append(np.concatenate([o, rng.normal(size=(k, 3)).astype(np.float32)], 1))
    # 5. leaving a side or the cap (origins on the face), cosine-like outward
    #    and grazing directions
    q = rng.choice(sides + [cap], k)
    u, v = rng.uniform(0, 1, (2, k))
    v00, v10, v01 = verts[q, 0], verts[q, 1], verts[q, 3]
    o = (v00 + u[:, None] * (v10 - v00) + v[:, None] * (v01 - v00)).astype(np.float32)
    nrm = np.cross(v10 - v00, v01 - v00)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    t = rng.normal(size=(k, 3))
    t -= (t * nrm).sum(1, keepdims=True) * nrm
    h = (10.0 ** rng.uniform(-7, 0, (k, 1))) * np.where(rng.uniform(0, 1, (k, 1)) < 0.5, 1, -1)
    out.append(np.concatenate([o, (t + h * nrm).astype(np.float32)], 1))
    # 6. grazing the sides: directions within 1e-7..1e-1 rad of a side's
    #    plane, passing near it
    q = rng.choice(sides, k)
    u, v = rng.uniform(-0.1, 1.1, (2, k))
    v00, v10, v01 = verts[q, 0], verts[q, 1], verts[q, 3]
    p = v00 + u[:, None] * (v10 - v00) + v[:, None] * (v01 - v00)
    nrm = np.cross(v10 - v00, v01 - v00)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    t = rng.normal(size=(k, 3))
    t -= (t * nrm).sum(1, keepdims=True) * nrm
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    ang = (10.0 ** rng.uniform(-7, -1, (k, 1))) * np.where(rng.uniform(0, 1, (k, 1)) < 0.5, 1, -1)
    d = t + ang * nrm
    o = p - rng.uniform(0.05, 0.6, (k, 1)) * d
    out.append(np.concatenate([o, d], 1).astype(np.float32))
    # 7. nearly vertical rays over the footprint and its rim (tiny x, z)
    o = np.c_[rng.uniform(lo[0] - 0.02, hi[0] + 0.02, k), rng.uniform(0.62, 0.99, k),
              rng.uniform(lo[2] - 0.02, hi[2] + 0.02, k)].astype(np.float32)
    d = np.c_[rng.normal(size=k) * 10.0 ** rng.uniform(-8, -1, k), -np.ones(k),
              rng.normal(size=k) * 10.0 ** rng.uniform(-8, -1, k)].astype(np.float32)
    out.append(np.concatenate([o, d], 1))
    # 8. the render's populations near the box: camera rays at it, bounces from
    #    the floor and walls toward random points on it
    eye = np.array([278, 278, -800], np.float32) / np.float32(555)
    q = rng.choice(sides + [cap], k)
    u, v = rng.uniform(0, 1, (2, k))
    tgt = verts[q, 0] + u[:, None] * (verts[q, 1] - verts[q, 0]) + v[:, None] * (verts[q, 3] - verts[q, 0])
    half = k // 2
    o = np.c_[rng.uniform(0, 1, k), np.zeros(k), rng.uniform(0, 1, k)].astype(np.float32)
    o[:half] = eye
    out.append(np.concatenate([o, (tgt - o).astype(np.float32)], 1))
    return np.ascontiguousarray(np.concatenate(out, 0), dtype=np.float32)


@pytest.mark.parametrize("variant", [0, 2])
def test_gpu_prefilter_box_rays_equal_exact_scan(device, variant):
    """The rotated box's hard rays (box_rays) through the prefiltered closest
    hit and the exact scan: the same hit, ray by ray.  (Round 6 also ran them
    against a per-lane cull of the box's faces: exact, not faster; DESIGN.md
    4.1, profiles/r06_box_cull.txt.)"""
    device.set_cornell_box(variant)
    verts = scene_quads(variant)
    rays = box_rays(verts, 1 << 21, 200 + variant)
    got = device.debug_closest_hit(rays)
    bad = np.nonzero((got[:, 0:3] != got[:, 3:6]).any(1))[0]
    assert bad.size == 0, f"{bad.size} rays differ, first {rays[bad[:3]].tolist()} -> {got[bad[:3]].tolist()}"
    assert (got[:, 6] != 2).all()
    device.set_cornell_box(0)
