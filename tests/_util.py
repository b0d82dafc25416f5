"""Shared helpers for the parity tests."""
from __future__ import annotations

import numpy as np


def same_bits_or_both_nan(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Elementwise: identical float32 bit patterns, or both NaN (the NaN payload
    differs between x86 SSE and CDNA and carries no information here)."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def assert_render_equal(got, want, what=""):
    """got/want: (rgba, seeds, live).  rgb sums bit-exact (NaN-aware), the
    final RNG state and the live-bounce count exact."""
    g_rgba, g_seed, g_live = got
    w_rgba, w_seed, w_live = want
    ok = same_bits_or_both_nan(g_rgba[:, :3], w_rgba[:, :3]).all(axis=1)
    bad = np.flatnonzero(~ok)
    assert bad.size == 0, (
        f"{what}: {bad.size} pixels differ, first {bad[:8].tolist()}: got {g_rgba[bad[:4]].tolist()} "
        f"want {w_rgba[bad[:4]].tolist()}"
    )
    if g_seed is not None and w_seed is not None:
        sb = np.flatnonzero(np.asarray(g_seed) != np.asarray(w_seed))
        assert sb.size == 0, f"{what}: final RNG state differs at {sb[:8].tolist()}"
    if g_live is not None and w_live is not None:
        lb = np.flatnonzero(np.asarray(g_live) != np.asarray(w_live))
        assert lb.size == 0, f"{what}: live-bounce count differs at {lb[:8].tolist()}"


def rmse_normalized(a_sum: np.ndarray, b_sum: np.ndarray, spp: int) -> float:
    """Per-pixel RMSE of the NormalizeFunctor outputs (main.cc:253-287)."""

    def norm(x):
        x = np.array(x[:, :3], dtype=np.float32)
        x[np.isnan(x)] = 0
        return np.sqrt(x / np.float32(spp))

    d = norm(a_sum).astype(np.float64) - norm(b_sum).astype(np.float64)
    return float(np.sqrt(np.mean(d * d)))


def load_full_frame(path: str) -> dict:
    """A whole-frame fixture (tools/make_golden.py full_frame_fixture): the
    rgb sums float32 [N, 3] rebuilt from their four byte planes, the NaN
    pixel list and the digests of the final seeds and live-bounce counts."""
    z = np.load(path, allow_pickle=False)
    g = {k: z[k] for k in z.files}
    planes = g.pop("rgb_planes")
    g["rgb"] = np.ascontiguousarray(planes.T).view(np.float32).reshape(-1, 3)
    return g


def sha256_u32(a) -> bytes:
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u4").tobytes()).digest()


def set_scene_from_oracle(device, sc) -> None:
    """Upload an oracle Scene (e.g. an edited cornell_box) through rtp_set_scene."""
    nq, ns = sc.n_quads, sc.n_spheres
    arr = np.ctypeslib.as_array
    device.set_scene(sc.points_np(), sc.quad_ids_np()[:, 1:], arr(sc.quad_mat)[:nq], arr(sc.quad_tex)[:nq],
                     arr(sc.sphere_point)[:ns], arr(sc.sphere_radius)[:ns], arr(sc.sphere_mat)[:ns],
                     arr(sc.sphere_tex)[:ns], arr(sc.mat_type)[: sc.n_mat], arr(sc.tex_type)[: sc.n_tex_type],
                     arr(sc.tex)[: sc.n_tex], tuple(sc.light_box_pointids[1:5]), sc.light_sphere_point, sc.ior)


def sample_shard_consistency(single: np.ndarray, shards: list, spp: int) -> dict:
    """Monte Carlo consistency of a sample-sharded image with the single-stream
    image of the same frame (SURVEY.md 8(e) C5 "statistical vs the unsharded
    reference"; shard.sample_batches).  single: the float32 [n, 4] sums of spp
    samples per pixel on the reference's stream (seed_base 0); shards: G
    arrays, each the sums of spp/G samples on its derived stream (seed_base
    k*n).  The two images are two independent estimates of each pixel's mean
    radiance, so their per-pixel difference D = (single - sum(shards)) / spp
    has mean 0 and variance 2 sigma^2 / spp, with sigma^2 the per-sample
    variance.  sigma^2 / (spp/G) is estimated per pixel from the spread of
    the G shard means (ddof 1), so Var(D) ~ 2 s^2 / G.  Pixels that are NaN in
    either image (a non-finite attenuation: the sum stays NaN, MapperPathTracer
    .cxx:350; NormalizeFunctor zeroes it) are counted, not compared.
    Returns: n (pixels compared), z_total (sum D / sqrt(sum Var D): ~N(0,1)),
    ratio (sum D^2 / sum Var D: ~1), outliers (fraction with |D| > 5 sd),
    norm_ratio (the same ratio after NormalizeFunctor, delta method:
    Var(sqrt m) ~ Var(m) / (4 m)), nan_single / nan_sharded."""
    G = len(shards)
    x = np.asarray(single, np.float64)[:, :3]
    ys = np.stack([np.asarray(s, np.float64)[:, :3] for s in shards])  # [G, n, 3]
    nan = np.isnan(x).any(1) | np.isnan(ys).any((0, 2))
    keep = ~nan
    x, ys = x[keep], ys[:, keep]
    mx = x / spp
    my = ys.sum(0) / spp
    means = ys / (spp / G)  # per-shard means
    var_d = 2.0 * means.var(0, ddof=1) / G  # [n, 3]
    d = mx - my
    live = var_d > 0
    z = np.zeros_like(d)
    z[live] = d[live] / np.sqrt(var_d[live])
    m = np.maximum(0.5 * (mx + my), 1e-12)
    nx_, ny_ = np.sqrt(mx), np.sqrt(my)
    return {
        "n": int(keep.sum()),
        "z_total": float(d[live].sum() / np.sqrt(var_d[live].sum())),
        "ratio": float((d[live] ** 2).sum() / var_d[live].sum()),
        "outliers": float((np.abs(z) > 5).mean()),
        "zero_var_nonzero_d": int(((~live) & (d != 0)).sum()),
        "norm_ratio": float(((nx_ - ny_)[live] ** 2).sum() / (var_d[live] / (4 * m[live])).sum()),
        "nan_single": int(np.isnan(np.asarray(single)[:, :3]).any(1).sum()),
        "nan_sharded": int(np.isnan(np.stack([np.asarray(s)[:, :3] for s in shards])).any((0, 2)).sum()),
    }


def assert_shards_consistent(st: dict, what: str = "") -> None:
    """Bounds for sample_shard_consistency (generous: the radiance per sample
    is heavy-tailed -- rare light hits of 15 -- and the variance is estimated
    from G shard means).  Measured on the oracle at 64x36: an unbiased
    sharded image gives z_total -0.3..-1.7, ratio 1.2-1.5, norm_ratio 1.07-1.09;
    the same image scaled by 1.02 gives z_total -5.5..-7.0, rendered at depth
    2 instead of 50 z_total 26-42 and norm_ratio 17-35."""
    assert st["n"] > 0, what
    assert abs(st["z_total"]) < 4, f"{what}: frame-mean difference is {st['z_total']:.2f} standard errors: {st}"
    assert 0.5 < st["ratio"] < 2.0, f"{what}: squared differences / expected = {st['ratio']:.3f}: {st}"
    assert 0.3 < st["norm_ratio"] < 3.0, f"{what}: normalised squared differences / expected: {st}"
    # (single-stream pixels that caught a rare light hit their 8 shards missed:
    # 2-3% of channels on an unbiased 64x36x256 frame, 27% at the wrong depth)
    assert st["outliers"] < 0.08, f"{what}: {st['outliers']:.4f} of pixel channels beyond 5 sd: {st}"
    a, b = st["nan_single"], st["nan_sharded"]
    assert abs(a - b) <= 5 * np.sqrt(a + b) + 3, f"{what}: NaN pixel counts {a} vs {b}"
