"""A whole-frame DIGEST fixture from the CPU oracle (test infrastructure):
every pixel of a frame at full S x D, rendered in row chunks (resumable: each
chunk's result is kept under --work until the frame is assembled), reduced
to SHA-256 digests -- of the float32 rgb sums with every NaN written as one
canonical pattern (NaN payloads differ between x86 and CDNA and carry no
information), of the final seeds and of the live-bounce counts -- plus the
NaN pixel list and float64 channel sums for diagnosis.  A render is bit-exact
against the oracle iff its digests match.

    python tools/make_golden_digest.py c4_full_digest 0 1920 1080 4096 50 [--threads 8]
    python tools/make_golden_digest.py c5_shard3_full_digest 0 3840 2160 2048 50 --seed-base 24883200

A second process can share the work: --reverse-from C renders chunks C-1
down to 0 (both skip chunks already kept).  --assemble-first K writes the
digest of the first K chunks only (pixels [0, bounds[K]): a leading band of
the frame, its pixel_count recorded) once those exist.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_ctypes as oc  # noqa: E402


def canonical_rgb_bytes(rgb: np.ndarray) -> bytes:
    a = np.ascontiguousarray(rgb, dtype=np.float32).copy()
    bits = a.view(np.uint32)
    bits[np.isnan(a)] = 0x7FC00000
    return bits.astype("<u4").tobytes()


def digest_fields(rgb: np.ndarray, seeds: np.ndarray, live: np.ndarray) -> dict:
    rgb = np.asarray(rgb, np.float32)
    return {"rgb_sha256": np.frombuffer(hashlib.sha256(canonical_rgb_bytes(rgb)).digest(), np.uint8),
            "seed_sha256": np.frombuffer(hashlib.sha256(np.asarray(seeds).astype("<u4").tobytes()).digest(), np.uint8),
            "live_sha256": np.frombuffer(hashlib.sha256(np.asarray(live).astype("<u4").tobytes()).digest(), np.uint8),
            "nan_pixels": np.flatnonzero(np.isnan(rgb).any(1)).astype(np.int64),
            "rgb_sum": np.nansum(rgb.astype(np.float64), axis=0),
            "seed_sum": np.uint64(np.asarray(seeds).astype(np.uint64).sum()),
            "live_sum": np.uint64(np.asarray(live).astype(np.uint64).sum())}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("variant", type=int)
    ap.add_argument("nx", type=int)
    ap.add_argument("ny", type=int)
    ap.add_argument("spp", type=int)
    ap.add_argument("depth", type=int)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--seed-base", type=int, default=0, help="seed = pixel + seed_base (a sample-batch shard)")
    ap.add_argument("--chunks", type=int, default=60)
    ap.add_argument("--work", default="/tmp/rtp_golden_work")
    ap.add_argument("--reverse-from", type=int, default=None, help="render chunks C-1 .. 0 (a helper process)")
    ap.add_argument("--assemble-first", type=int, default=None, help="assemble the first K chunks only")
    a = ap.parse_args()
    work = os.path.join(a.work, a.name)
    os.makedirs(work, exist_ok=True)
    # the chunk cache is valid only for the configuration that wrote it: a
    # manifest records it, and a different one under the same name is refused
    config = {"variant": a.variant, "nx": a.nx, "ny": a.ny, "spp": a.spp, "depth": a.depth,
              "seed_base": a.seed_base, "chunks": a.chunks}
    manifest = os.path.join(work, "manifest.json")
    if os.path.exists(manifest):
        with open(manifest) as f:
            old = json.load(f)
        if old != config:
            raise SystemExit(f"{work} holds chunks of another configuration ({old}); remove it or use another --work")
    else:
        if any(fn.startswith("chunk") for fn in os.listdir(work)):
            raise SystemExit(f"{work} holds chunks without a manifest; remove them or use another --work")
        with open(manifest, "w") as f:
            json.dump(config, f)
    sc = oc.cornell_box(a.variant)
    cam = oc.camera_setup(a.nx, a.ny)
    n = a.nx * a.ny
    bounds = np.linspace(0, n, a.chunks + 1).astype(np.int64)
    t0 = time.time()
    order = range(a.chunks) if a.reverse_from is None else range(a.reverse_from - 1, -1, -1)
    if a.assemble_first is not None:
        order = []
    for c in order:
        f = os.path.join(work, f"chunk{c:04d}.npz")
        if os.path.exists(f):
            continue
        pix = np.arange(bounds[c], bounds[c + 1], dtype=np.int64)
        rgba, seeds, live = oc.render_pixels(sc, cam, a.nx, a.ny, a.spp, a.depth, pix, seed_base=a.seed_base,
                                             nthreads=a.threads)
        np.savez(f + ".tmp.npz", rgb=rgba[:, :3], seeds=seeds, live=live, begin=bounds[c], end=bounds[c + 1])
        os.replace(f + ".tmp.npz", f)
        print(f"chunk {c + 1}/{a.chunks} ({pix.size} px): {time.time() - t0:.0f}s", flush=True)
    k = a.chunks if a.assemble_first is None else a.assemble_first
    missing = [c for c in range(k) if not os.path.exists(os.path.join(work, f"chunk{c:04d}.npz"))]
    if missing:
        raise SystemExit(f"{len(missing)} chunks still missing (first {missing[:4]})")
    parts = [np.load(os.path.join(work, f"chunk{c:04d}.npz")) for c in range(k)]
    for c, p in enumerate(parts):
        if (int(p["begin"]), int(p["end"])) != (int(bounds[c]), int(bounds[c + 1])) or len(p["rgb"]) != bounds[c + 1] - bounds[c]:
            raise SystemExit(f"chunk {c} does not cover pixels [{bounds[c]}, {bounds[c + 1]})")
    rgb = np.concatenate([p["rgb"] for p in parts])
    seeds = np.concatenate([p["seeds"] for p in parts])
    live = np.concatenate([p["live"] for p in parts])
    assert len(rgb) == len(seeds) == len(live) == bounds[k]
    out = os.path.join(ROOT, "tests", "golden", a.name + ".npz")
    np.savez_compressed(out, variant=a.variant, nx=a.nx, ny=a.ny, spp=a.spp, depth=a.depth, camera=cam,
                        seed_base=a.seed_base, pixel_begin=0, pixel_count=int(bounds[k]),
                        **digest_fields(rgb, seeds, live))
    print(f"{a.name}: {a.nx}x{a.ny} ({int(bounds[k])} px) x {a.spp} spp x depth {a.depth}: "
          f"L={live.sum() / (int(bounds[k]) * a.spp):.4f}, "
          f"nan_px={int(np.isnan(rgb).any(1).sum())} -> {out}")


if __name__ == "__main__":
    main()
