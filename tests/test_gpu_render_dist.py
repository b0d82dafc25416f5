"""The multi-GPU render driver (raytracingtherestofyourlife_amd.render_dist)
rehearsed on one GPU: torch.distributed.run with 2 and 3 ranks sharing device
0, gloo (host-side) reduce.  Rank 0 checks the reduced canvas against a
one-process render of the same plan (tiles: bit-exact; sample batches: the
shard renders summed)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("shard,ranks", [("tiles", 2), ("samples", 2), ("tiles", 3), ("samples", 3)])
def test_render_dist_rehearsal(shard, ranks, tmp_path):
    env = dict(os.environ, RTP_FF_TABLES="1", MASTER_ADDR="127.0.0.1")
    port = str(29600 + ranks * 10 + (shard == "samples"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", port, "-m", "raytracingtherestofyourlife_amd.render_dist",
           "--nx", "96", "--ny", "64", "--spp", "12", "--depth", "20", "--shard", shard, "--backend", "gloo",
           "--share-gpu", "--check", "--out", str(tmp_path / "img.pnm")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["check"] is True and lines[0]["n_gpus"] == ranks
    assert (tmp_path / "img.pnm").read_text().startswith("P3\n96 64 255\n")
