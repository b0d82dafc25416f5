"""Oracle fixtures of the sample-batch shard's REDUCED frame (VERDICT r05
"next" 1): for each world size N, every rank's shard -- spp/N samples of each
fixture pixel on its derived stream seed = pixel + k*nx*ny
(shard.sample_batches; MapperPathTracer.cxx:265-267 seeds, :278 the sample
loop, :350 cols += s) -- and their float32 sum in rank order.  bench.py's N > 1
line checks its shards bit for bit and its reduced frame against these.

    python tools/make_golden_reduced.py          # both fixtures (~1 min, 8 cores)
    python tools/make_golden_reduced.py small    # only the small-canvas one

tests/golden/c5_reduced.npz: C5 (3840x2160, 16384 spp, depth 50) on the 1024
  pixels of c5_shard3_2048spp (its rank-3-of-8 shard doubles as a cross-check),
  N = 2, 4, 8.
tests/golden/c5_reduced_small.npz: 96x64, 512 spp, depth 20, the whole frame,
  N = 2 and 4 (the one-GPU rehearsals of tests/test_gpu_bench_c5.py).
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_ctypes as oc  # noqa: E402

from raytracingtherestofyourlife_amd.shard import sample_batches  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def reduced_fixture(name, nx, ny, spp, depth, pixels, worlds, variant=0):
    t = time.time()
    sc = oc.cornell_box(variant)
    cam = oc.camera_setup(nx, ny)
    out = {}
    for n in worlds:
        shards, seeds, lives = [], [], []
        for b in sample_batches(spp, n, nx * ny):
            rgba, fs, lv = oc.render_pixels(sc, cam, nx, ny, b.spp, depth, pixels, seed_base=b.seed_base)
            shards.append(np.ascontiguousarray(rgba[:, :3], np.float32))
            seeds.append(fs)
            lives.append(lv)
        red = shards[0].copy()
        for s in shards[1:]:
            red = (red + s).astype(np.float32)  # rank order, one float32 add per rank
        out[f"shards_{n}"] = np.stack(shards)
        out[f"final_seed_{n}"] = np.stack(seeds)
        out[f"live_{n}"] = np.stack(lives)
        out[f"reduced_{n}"] = red
        print(f"{name} N={n}: {pixels.size} px x {spp} spp, nan_px={int(np.isnan(red).any(1).sum())}, "
              f"{time.time() - t:.1f}s", flush=True)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), variant=variant, nx=nx, ny=ny, spp=spp, depth=depth,
                        camera=cam, pixels=pixels, worlds=np.int32(worlds), **out)


def main():
    only = set(sys.argv[1:])
    if not only or "small" in only:
        reduced_fixture("c5_reduced_small", 96, 64, 512, 20, np.arange(96 * 64, dtype=np.int64), (2, 4))
    if not only or "full" in only:
        z = np.load(os.path.join(OUT, "c5_shard3_2048spp.npz"), allow_pickle=False)
        reduced_fixture("c5_reduced", 3840, 2160, 16384, 50, np.asarray(z["pixels"], np.int64), (2, 4, 8))


if __name__ == "__main__":
    main()
