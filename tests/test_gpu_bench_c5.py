"""bench.py's C5 path (--workload c5, the sample-batch shard) rehearsed on
one GPU: torch.distributed.run with 2 ranks sharing device 0, gloo reduce, a
small canvas.  Rank k renders spp/2 samples of every pixel on its derived
stream (seed_base k*nx*ny); rank 0 then renders the whole frame alone (the
same-workload one-GPU anchor) and checks the reduced canvas: it equals the
sum of the gathered shards exactly (two ranks: one float add per pixel, NaN
pixels in the same places) and agrees with the single-stream image
statistically (shard.sample_shard_ttest)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_c5_sample_shard_rehearsal():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29671", "bench.py", "--gpus", "2",
           "--dist-backend", "gloo", "--share-gpu", "--workload", "c5", "--nx", "96", "--ny", "64",
           "--spp", "512", "--depth", "20", "--steps", "2", "--warmup", "1", "--ff-tables", "off", "--check"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["config"]["spp_per_gpu"] == 256
    assert "sample batches" in line["config"]["shard"]
    chk = line["check_reduced_canvas"]
    assert chk["pixels"] == 96 * 64
    assert chk["reduced_equals_sum_of_shards_max_rel"] == 0.0 and chk["nan_pattern_equal"]
    assert chk["consistent"] is True, chk
    assert line["one_gpu_same_workload"]["kernel_ms"] > 0
    assert line["speedup_vs_one_gpu_same_workload"] > 0
