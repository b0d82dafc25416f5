"""bench.py's C5 path (--workload c5, the sample-batch shard) rehearsed on
one GPU: `bench.py --gpus N` started WITHOUT torch.distributed.run (bench.py
launches its N ranks itself), the ranks sharing device 0, gloo reduce, a small
canvas.  Rank k renders spp/N samples of every pixel on its derived stream
(seed_base k*nx*ny).  The line's parity comes from the oracle's reduced-frame
fixture of that N (tests/golden/c5_reduced_small.npz,
tools/make_golden_reduced.py): every rank's shard bit-exact, the reduced frame
bit-exact (two ranks: one float add; more: the sum in the reduce's fixed
association, shard.tree_reduce_'s pairwise tree) and rmse 0 at N = 2.  Rank 0 then renders the whole frame alone
on an unused stream (the same-workload one-GPU anchor) and checks the reduced
canvas statistically against it (shard.sample_shard_ttest)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--dist-backend", "gloo", "--share-gpu", "--workload", "c5",
           "--nx", "96", "--ny", "64", "--spp", "512", "--depth", "20", "--steps", "2", "--warmup", "1",
           "--ff-tables", "off", "--check"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


def test_bench_c5_sample_shard_rehearsal():
    line = _run(2)
    assert line["n_gpus"] == 2 and line["config"]["spp_per_gpu"] == 256
    assert "sample batches" in line["config"]["shard"]
    par = line["reduced_frame_parity"]
    assert par["fixture"] == "c5_reduced_small.npz" and par["pixels"] == 96 * 64
    assert par["shards_bit_exact"] and par["reduced_bit_exact_rank_order"], par
    assert line["bit_exact"] is True and line["rmse"] == 0.0
    chk = line["check_reduced_canvas"]
    assert chk["pixels"] == 96 * 64
    assert chk["reduced_equals_sum_of_shards_max_rel"] == 0.0 and chk["nan_pattern_equal"]
    assert chk["consistent"] is True, chk
    assert line["one_gpu_same_workload"]["kernel_ms"] > 0
    sp = line["speedup_vs_one_gpu_same_workload"]
    assert sp["kernel"] > 0 and sp["wall"] > 0


def test_bench_c5_four_ranks_reduced_parity():
    line = _run(4)
    assert line["n_gpus"] == 4 and line["config"]["spp_per_gpu"] == 128
    par = line["reduced_frame_parity"]
    assert par["ranks"] == 4 and par["shards_bit_exact"], par
    assert par["bit_exact"] is True and line["bit_exact"] is True, json.dumps(par)
    assert par["reduced_bit_exact_tree"] is True  # ((s0 + s1) + (s2 + s3)), every pixel
    assert line["rmse"] < 1e-6
    chk = line["check_reduced_canvas"]
    assert chk["reduced_equals_sum_of_shards_max_rel"] == 0.0 and chk["nan_pattern_equal"]
