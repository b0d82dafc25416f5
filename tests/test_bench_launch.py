"""bench.py's multi-GPU launch and its N > 1 parity helpers, on CPU.

`bench.py --gpus N` without torch.distributed.run launches its N ranks as a
child (never a one-GPU line for --gpus N); the reduced-frame parity of the
N > 1 line against the oracle's fixtures (tools/make_golden_reduced.py)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_cmd_is_one_process_per_gpu():
    cmd = bench.launch_cmd(["--gpus", "8", "--steps", "3"], 8, 29500)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")


def _env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}


def test_world_size_mismatch_fails():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=dict(_env(), WORLD_SIZE="3"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr
    assert not any(l.startswith("{") for l in r.stdout.splitlines())


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a HIP device is present")
def test_gpus_n_without_launcher_starts_ranks_and_never_reports_one_gpu():
    """No GPU here: the N ranks bench.py starts fail, and so does bench.py --
    with their exit code, and without a JSON line."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--share-gpu"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not any(l.startswith("{") for l in r.stdout.splitlines())
    assert "torch.distributed" in r.stderr or "ChildFailedError" in r.stderr or "rank" in r.stderr.lower()


def test_find_reduced_fixture():
    for n in (2, 4, 8):
        f = bench.find_reduced_fixture(3840, 2160, 16384, 50, n)
        assert f["name"] == "c5_reduced.npz" and f["shards"].shape == (n, 1024, 3)
    f = bench.find_reduced_fixture(96, 64, 512, 20, 2)
    assert f["name"] == "c5_reduced_small.npz" and f["pixels"].size == 96 * 64
    assert bench.find_reduced_fixture(96, 64, 512, 20, 8) is None
    assert bench.find_reduced_fixture(3840, 2160, 16384, 49, 8) is None


def test_fixture_shards_match_the_shard3_fixture():
    """The N = 8 fixture's rank 3 is the older c5_shard3_2048spp fixture."""
    f = bench.find_reduced_fixture(3840, 2160, 16384, 50, 8)
    z = np.load(os.path.join(ROOT, "tests", "golden", "c5_shard3_2048spp.npz"), allow_pickle=False)
    assert np.array_equal(f["pixels"], z["pixels"])
    assert bench._same_bits(f["shards"][3], np.asarray(z["rgb"], np.float32)).all()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_reduced_frame_parity(n):
    f = bench.find_reduced_fixture(3840, 2160, 16384, 50, n)
    shards = [np.c_[s, np.zeros(len(s), np.float32)] for s in f["shards"]]
    sums = bench.association_sums(f["shards"])
    tree = sums["pairwise_tree" if n > 2 else "rank_order"]  # the reduce's own association (shard.tree_reduce_)
    for name, red in sums.items():
        p = bench.reduced_frame_parity(f, shards, red, 16384)
        assert p["shards_bit_exact"], (name, p)
        assert p["reduced_association"][name] == 1024 and p["reduced_pixels_matching_an_association"] == 1024
        # bit_exact: the reduce's association only (another one passes where it happens to agree)
        same = bool(bench._same_bits(red, tree).all())
        assert p["bit_exact"] == same and p["reduced_bit_exact_tree"] == same, (name, p)
        assert p["rmse"] < (1e-6 if n > 2 else 1e-30)
    assert bench.reduced_frame_parity(f, shards, tree, 16384)["bit_exact"]
    if n == 8:  # RCCL-style rank-order chains are not the reduce's bits
        assert not bench.reduced_frame_parity(f, shards, sums["rank_order"], 16384)["bit_exact"]
    assert bench.reduced_frame_parity(f, shards, f["reduced"], 16384)["rmse"] == 0.0
    # one ulp off in one shard's pixel: the shard check and the line's bit_exact fail
    bad = [s.copy() for s in shards]
    k = int(np.flatnonzero(np.isfinite(bad[-1][:, 0]) & (bad[-1][:, 0] > 0))[0])
    bad[-1][k, 0] = np.nextafter(bad[-1][k, 0], np.float32(np.inf))
    p = bench.reduced_frame_parity(f, bad, f["reduced"], 16384)
    assert not p["shards_bit_exact"] and p["shard_bit_exact_per_rank"] == [True] * (n - 1) + [False]
    assert not p["bit_exact"]
    # a reduced frame that matches no association
    red = f["reduced"].copy()
    red[k, 1] = red[k, 1] * np.float32(1.01) + np.float32(1.0)
    p = bench.reduced_frame_parity(f, shards, red, 16384)
    assert p["reduced_pixels_matching_an_association"] == 1023 and not p["bit_exact"] and p["rmse"] > 0


def test_association_sums_orders():
    s = np.random.default_rng(1).standard_normal((4, 64, 3)).astype(np.float32) * np.float32(1e3)
    sums = bench.association_sums(s)
    assert np.array_equal(sums["rank_order"], ((s[0] + s[1]) + s[2]) + s[3])
    assert np.array_equal(sums["ring_fwd_from_1"], ((s[1] + s[2]) + s[3]) + s[0])
    assert np.array_equal(sums["ring_rev_from_2"], ((s[2] + s[1]) + s[0]) + s[3])
    assert np.array_equal(sums["pairwise_tree"], (s[0] + s[1]) + (s[2] + s[3]))
    assert len(sums) == 9  # 2 directions x 4 starts + the tree (distinct on random data)
    assert set(bench.association_sums(s[:2])) == {"rank_order"}  # one add: the same either way


def test_load_golden_frame_skips_non_frame_fixtures():
    """`bench.py --workload c5` on one GPU: the workload's fixture is the N > 1
    reduced-frame file, which holds no frame; the N = 1 line then reports no
    frame quality instead of failing (the r06x run that found it)."""
    assert bench.load_golden_frame(os.path.join(ROOT, "tests", "golden", "c5_reduced.npz")) is None
    g = bench.load_golden_frame(os.path.join(ROOT, "tests", "golden", "c4_subset16k.npz"))
    assert g is not None and g["pixels"] is not None and (g["nx"], g["ny"]) == (1920, 1080)
