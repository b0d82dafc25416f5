"""The RCCL (torch.distributed "nccl") path of the multi-GPU bench, run on a
one-GPU box: torch.distributed.run with ONE rank and --force-collective, so
init_process_group("nccl", device_id=...), the asynchronous dist.reduce of
the float4 canvas on two alternating canvases (shard.OverlappedCanvasReduce)
and its wait() all execute, as on every rank of an N-GPU run.  The reduced
canvas must equal a one-process render bit for bit (a 1-rank sum is the
identity), and RCCL must report itself initialised (NCCL_DEBUG=INFO)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_rccl_reduce_path_on_one_rank():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", NCCL_DEBUG="INFO")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", "29655", "bench.py", "--gpus", "1",
           "--force-collective", "--dist-backend", "nccl", "--workload", "c2", "--nx", "64", "--ny", "64",
           "--spp", "8", "--depth", "10", "--steps", "3", "--warmup", "1", "--cpu-budget", "0",
           "--cpu-budget-mt", "0", "--ff-tables", "off", "--check"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["config"]["dist_backend"] == "nccl"
    assert "RCCL" in line["config"]["shard"]
    assert line["check_reduced_canvas_equals_single_render"] is True
    log = r.stdout + r.stderr
    assert "NCCL INFO" in log, log[-2000:]


def test_bench_rccl_sample_shard_path_on_one_rank():
    """bench.py's C5 path (--workload c5) through RCCL on one rank: the
    all_gather of the shard-check codes and of the shards' check pixels, the
    whole-canvas copy into the overlapped reduce, rank 0's same-workload
    one-GPU render and the reduced-canvas checks (one rank: the reduce is the
    identity, so the reduced canvas equals the shard exactly)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", "29657", "bench.py", "--gpus", "1",
           "--force-collective", "--dist-backend", "nccl", "--workload", "c5", "--nx", "96", "--ny", "64",
           "--spp", "64", "--depth", "20", "--steps", "2", "--warmup", "1", "--ff-tables", "off", "--check"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["config"]["dist_backend"] == "nccl" and "sample batches" in line["config"]["shard"]
    chk = line["check_reduced_canvas"]
    assert chk["reduced_equals_sum_of_shards_max_rel"] == 0.0 and chk["nan_pattern_equal"]
    assert chk["consistent"] is True
    sp = line["speedup_vs_one_gpu_same_workload"]
    assert sp["kernel"] > 0 and sp["wall"] > 0
    # no committed reduced-frame fixture for this N = 1 configuration: said so
    assert line["reduced_frame_parity"].startswith("not checked")
