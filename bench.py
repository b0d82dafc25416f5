"""Benchmark of the path-tracing hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload auto|c2|c4|c5] [--scaling strong|weak]

One step = one full render of the workload's frame.  On one GPU (no process
group) the frame goes through the library's default contiguous launch
(rtp_render_device over [0, nx*ny), like main.cc's render; --n1-launch tiles:
the tile-deal instance the ranks of a tile-sharded run use).
  c2: Cornell Box 800x800, 1000 spp, depth 50 (BASELINE.json configs[1]), the
      metric's own image: the N = 1 workload (--workload auto).
  c4: Cornell Box 1920x1080, 4096 spp, depth 50 (BASELINE.json configs[3]),
      image-tile shard over the ranks.
  c5: Cornell Box 3840x2160, 16384 spp, depth 50 (BASELINE.json configs[4]),
      sample-batch shard: the N > 1 workload (--workload auto).  Rank k renders
      spp/N samples of EVERY pixel on its derived stream (seed = pixel + k*nx*ny,
      shard.sample_batches), so no rank carries a whole pixel's sample chain
      (the chain floor that caps the tile shards).
N > 1 (launched by torch.distributed.run, one process per GPU):
  --scaling strong (default): THE frame, split over the ranks (c2/c4: 16x16
      tiles dealt round-robin; c5: sample batches); the float4
      framebuffer is summed to rank 0 with ONE reduce per step, a pairwise tree
      of RCCL point-to-point transfers over xGMI in a fixed association
      (shard.tree_reduce_: the same bits on any node), overlapped with the next
      step's render (two canvases, alternating).
  --scaling weak: every rank renders a full nx x ny band of an nx x ny*N
      canvas (per-GPU work fixed).
  After the timed region rank 0 renders the same workload's whole frame alone
  (--anchor, default on): `one_gpu_same_workload` and
  `speedup_vs_one_gpu_same_workload` compare like with like (the driver's
  N-GPU / 1-GPU ratio divides C5's rate by C2's).  The N = 1 line carries
  `scaling_anchors`: one-GPU kernel times of C4's whole frame and of one C5
  rank share, measured in the same run.

Rank 0 prints one JSON line.  `value` = all ranks' samples / max-over-ranks
wall time of the K timed steps (steady state: the renderer's context, scene
and RNG jump tables are set up before the timed region -- `setup` and
`first_render_ms` report what that costs, and `one_shot` what a fresh process
rendering once, like main.cc, would see).  `rmse` / `bit_exact` compare the
last timed frame (normalised, NormalizeFunctor) with the oracle's committed
C2 frame (tests/golden/c2_full.npz); at N > 1 the C5 line takes them from
`reduced_frame_parity`: every rank's shard and the reduced frame at 1024
pixels against the oracle's reduced-frame fixture of that N
(tests/golden/c5_reduced.npz, N = 2/4/8; bit-exact shards, the reduced frame
bit-exact against the shards' sum in the reduce's fixed association), plus the
statistical check of the reduced frame against an independent single-stream
image.  `bench.py --gpus N` without torch.distributed.run starts it (one
process per GPU) as a child and relays rank 0's line.  `roofline` prices the render kernel
with the SoA byte model of SURVEY.md 8(d) (56 + 88*L bytes per sample) against
the 8 TB/s HBM peak; `roofline_valu` gives the VALU-issue bound (the one that
binds) from the committed PMC summary; `cpu_baseline` times
the oracle's stage-structured restatement on a bounded sample of the same
workload on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec (whole node), Cornell Box 800×800×1000spp; per-pixel RMSE vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
TILE = 16
# BASELINE.json configs: the bench workloads and their committed oracle fixtures
WORKLOADS = {
    "c2": {"nx": 800, "ny": 800, "spp": 1000, "depth": 50, "golden": "c2_full.npz",
           "name": "C2: Cornell Box 800x800, 1000 spp, depth 50"},
    "c4": {"nx": 1920, "ny": 1080, "spp": 4096, "depth": 50, "golden": "c4_subset16k.npz",
           "name": "C4: Cornell Box 1920x1080, 4096 spp, depth 50 (BASELINE configs[3], image-tile shard)"},
    "c5": {"nx": 3840, "ny": 2160, "spp": 16384, "depth": 50, "golden": "c5_reduced.npz",
           "name": "C5: Cornell Box 3840x2160, 16384 spp, depth 50 (BASELINE configs[4], sample-batch shard)"},
}
SHARD = {"c2": "tiles", "c4": "tiles", "c5": "samples"}
# pixels of the C5 frame compared with the single-stream image (statistical check)
C5_CHECK_PIXELS = 65536


def cpu_baseline(budget_s: float, nx: int, ny: int, depth: int, nthreads: int = 1) -> dict:
    """Oracle stage-structured SoA pass sequence (the reference's cost model:
    every stage over every ray, no compaction), on the C2 camera: a band of
    rows at 1 spp sized to ~budget_s, widened to the full frame and then to
    more samples per pixel when one frame is cheaper than the budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as oc

    oc.build()
    sc = oc.cornell_box(0)
    cam = oc.camera_setup(nx, ny)
    mid = ny // 2
    rows = 8
    t = time.perf_counter()
    oc.render_soa(sc, cam, nx, ny, 1, depth, row_begin=mid - rows // 2, row_end=mid + rows // 2, nthreads=nthreads)
    probe = time.perf_counter() - t
    want_rows = rows * budget_s / max(probe, 1e-3)
    spp = max(1, int(want_rows / ny)) if want_rows > ny else 1
    rows = int(max(8, min(ny, want_rows)))
    r0 = max(0, mid - rows // 2)
    r1 = min(ny, r0 + rows)
    t = time.perf_counter()
    oc.render_soa(sc, cam, nx, ny, spp, depth, row_begin=r0, row_end=r1, nthreads=nthreads)
    dt = time.perf_counter() - t
    samples = (r1 - r0) * nx * spp
    return {
        "value": samples / dt / 1e6,
        "unit": "Msamples/s",
        "cores": nthreads,
        "kind": "port",
        "sample": f"C2 scene+camera {nx}x{ny}, rows {r0}-{r1} ({(r1 - r0) * nx} pixels) x {spp} spp, depth {depth}: "
                  f"{samples} samples in {dt:.1f}s, stage-structured SoA oracle, {nthreads} thread(s)",
    }


def host_threads() -> int:
    """CPU share of this process (affinity), capped at 16 (the GPU box's share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def load_traffic(path: str, cfg: dict):
    """Per-launch HBM bytes measured by rocprofv3 --pmc for this config (or None)."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if all(t.get(k) == v for k, v in cfg.items()):
        return t.get("hbm_bytes_per_launch")
    return None


def load_golden_frame(path: str, any_seed: bool = False):
    """The oracle's committed fixture of the workload: tests/golden/c2_full.npz
    (tools/make_golden.py full_frame_fixture, every pixel: un-normalised rgb
    sums [N, 3]) or a pixel-subset fixture (c4_subset16k.npz: `pixels` and
    their sums), with its config; None if absent."""
    try:
        z = np.load(path, allow_pickle=False)
    except OSError:
        return None
    if "rgb_planes" not in z.files and "rgb" not in z.files:
        return None  # not a frame fixture (c5_reduced.npz: the N > 1 shards, reduced_frame_parity)
    if "rgb_planes" in z.files:
        rgb, pixels = np.ascontiguousarray(z["rgb_planes"].T).view(np.float32).reshape(-1, 3), None
    else:
        rgb, pixels = np.asarray(z["rgb"], np.float32), np.asarray(z["pixels"], np.int64)
        if int(z["seed_base"]) != 0 and not any_seed:
            return None
    return {"rgb": rgb, "pixels": pixels, "nx": int(z["nx"]), "ny": int(z["ny"]), "spp": int(z["spp"]),
            "depth": int(z["depth"]), "seed_base": int(z["seed_base"]) if "seed_base" in z.files else 0}


def frame_quality(canvas: np.ndarray, gold: dict, spp: int) -> dict:
    """Per-pixel RMSE of the normalised frames (NormalizeFunctor, main.cc:253-287,
    before quantisation) and bitwise equality of the sums (NaN-aware), over
    every pixel the fixture holds (the whole frame, or its pixel subset)."""
    import raytracingtherestofyourlife_amd as rtp

    a = np.ascontiguousarray(canvas if gold["pixels"] is None else canvas[gold["pixels"]], dtype=np.float32).copy()
    b = np.c_[gold["rgb"], np.zeros(len(gold["rgb"]), np.float32)].astype(np.float32)
    same = (a[:, :3].view(np.uint32) == b[:, :3].view(np.uint32)) | (np.isnan(a[:, :3]) & np.isnan(b[:, :3]))
    rtp.normalize(a, spp)
    rtp.normalize(b, spp)
    d = a[:, :3].astype(np.float64) - b[:, :3].astype(np.float64)
    return {"rmse": float(np.sqrt(np.mean(d * d))), "bit_exact": bool(same.all()),
            "pixels_checked": int(len(b)), "pixels_differing": int((~same.all(1)).sum()),
            "nan_pixels_ref": int(np.isnan(gold["rgb"]).any(1).sum())}


def launch_cmd(argv: list, gpus: int, port: int) -> list:
    """`bench.py --gpus N` started without torch.distributed.run (WORLD_SIZE
    unset): the one-process-per-GPU launch of the driver's contract, as a
    fresh child process started before this process touches the GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def self_launch(argv: list, gpus: int) -> int:
    """Run launch_cmd as a child (stdout inherited: rank 0's JSON line is this
    process's line) and return its exit code."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(launch_cmd(argv, gpus, port), env=env).returncode


REDUCED_FIXTURES = ("c5_reduced.npz", "c5_reduced_small.npz")


def find_reduced_fixture(nx: int, ny: int, spp: int, depth: int, world: int, explicit: str | None = None):
    """The oracle's reduced-frame fixture (tools/make_golden_reduced.py) of
    this sample-shard configuration and world size: every rank's shard at the
    fixture pixels (shards_N [N, n, 3]) and their float32 sum in rank order
    (reduced_N); None if no committed fixture matches."""
    cands = [explicit] if explicit else [os.path.join(ROOT, "tests", "golden", f) for f in REDUCED_FIXTURES]
    for path in cands:
        try:
            z = np.load(path, allow_pickle=False)
        except (OSError, ValueError):
            continue
        if f"shards_{world}" not in z.files:
            continue
        if (int(z["nx"]), int(z["ny"]), int(z["spp"]), int(z["depth"])) != (nx, ny, spp, depth):
            continue
        return {"name": os.path.basename(path), "pixels": np.asarray(z["pixels"], np.int64),
                "shards": np.asarray(z[f"shards_{world}"], np.float32),
                "reduced": np.asarray(z[f"reduced_{world}"], np.float32)}
    return None


def _same_bits(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def association_sums(shards: np.ndarray) -> dict:
    """float32 sums of the N shards in several associations: the pairwise
    tree (shard.tree_reduce_'s, the one bench.py's reduce uses) and, for
    diagnosis, a chain along the ring of ranks from any start k in either
    direction (((s_k + s_k+1) + ...) + s_k-1: what a ring reduce in rank
    order would give).  "rank_order" is the forward chain from rank 0."""
    s = [np.asarray(x, np.float32) for x in shards]
    n = len(s)
    if n <= 2:  # one add: the same either way
        return {"rank_order": s[0] + s[1] if n == 2 else s[0].copy()}
    out = {}
    for direction in (1, -1):
        for k in range(n):
            order = [(k + direction * i) % n for i in range(n)]
            acc = s[order[0]].copy()
            for r in order[1:]:
                acc = acc + s[r]
            name = "rank_order" if (direction, k) == (1, 0) else f"ring_{'fwd' if direction > 0 else 'rev'}_from_{k}"
            out[name] = acc
    from raytracingtherestofyourlife_amd import shard

    out["pairwise_tree"] = shard.tree_sum(s)
    return out


def reduced_frame_parity(fix: dict, shards_got: list, reduced_got: np.ndarray, spp: int) -> dict:
    """The N > 1 line's parity against the oracle:
    every rank's shard at the fixture pixels bit for bit against the oracle's
    shard, and the reduced frame bit for bit against the oracle's shards
    summed in float32 in the reduce's own association (shard.tree_reduce_:
    the pairwise tree; two ranks: one add, so exactly the fixture's
    rank-order sum), plus the per-pixel RMSE of the normalised frames
    (NormalizeFunctor, main.cc:253-287) against the fixture's rank-order sum.
    The other associations are reported for diagnosis.  shards_got: N arrays
    [n, >=3]; reduced_got [n, >=3]."""
    import raytracingtherestofyourlife_amd as rtp

    want = fix["shards"]
    n = want.shape[1]
    shard_ok = [bool(_same_bits(np.ascontiguousarray(g[:, :3], np.float32), w).all())
                for g, w in zip(shards_got, want)]
    red = np.ascontiguousarray(reduced_got[:, :3], np.float32)
    sums = association_sums(want)
    per = {k: _same_bits(red, v).all(1) for k, v in sums.items()}
    own = per["pairwise_tree" if "pairwise_tree" in per else "rank_order"]  # shard.tree_reduce_'s association
    any_match = np.logical_or.reduce(list(per.values()))
    a = np.c_[red, np.zeros(n, np.float32)].astype(np.float32)
    b = np.c_[fix["reduced"], np.zeros(n, np.float32)].astype(np.float32)
    rtp.normalize(a, spp)
    rtp.normalize(b, spp)
    d = a[:, :3].astype(np.float64) - b[:, :3].astype(np.float64)
    fin = np.isfinite(red) & np.isfinite(fix["reduced"])
    rel = np.abs(red[fin].astype(np.float64) - fix["reduced"][fin]) / np.maximum(np.abs(fix["reduced"][fin]), 1e-30)
    return {"fixture": fix["name"], "pixels": int(n), "ranks": len(want),
            "shards_bit_exact": all(shard_ok) and len(shard_ok) == len(want),
            "shard_bit_exact_per_rank": shard_ok,
            "reduced_bit_exact_tree": bool(own.all()),
            "reduced_bit_exact_rank_order": bool(per["rank_order"].all()),
            "reduced_association": {k: int(v.sum()) for k, v in per.items()},
            "reduced_pixels_matching_an_association": int(any_match.sum()),
            "reduced_max_rel_vs_rank_order": float(rel.max()) if rel.size else 0.0,
            "rmse": float(np.sqrt(np.mean(d * d))),
            "bit_exact": bool(all(shard_ok) and own.all())}


def load_valu(path: str, cfg: dict, kernel_ms: float):
    """VALU-issue bound of the render kernel from a committed PMC summary
    (tools/pmc_valu.sh): wave64 VALU instructions per launch against the
    SIMDs' issue capacity at 2 cycles per wave64 instruction
    (MI355X_MICROARCH.md, per-instruction constants: v_fma_f32 2 cyc on
    SIMD-32), over the cycles the chip ran (GRBM_GUI_ACTIVE / 8 XCDs).  The
    live HIP-event kernel time rescales the PMC run's cycles to this run."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if not all(t.get(k) == v for k, v in cfg.items()):
        return None
    cap = t["simds"] * t["gpu_cycles_per_launch"] / t["cycles_per_wave64_valu"]
    frac = t["valu_insts_per_launch"] / cap
    lanes = t.get("lanes_per_instr")
    return {"bound": "valu-issue", "achieved": t["valu_insts_per_launch"] / (kernel_ms / 1e3) / 1e12,
            "peak": t["simds"] * t["clock_ghz"] * 1e9 / t["cycles_per_wave64_valu"] / 1e12,
            "unit": "T wave64-VALU instr/s", "frac": round(frac, 4),
            "lanes_per_instr": lanes,
            # issue slots x the fraction of their 64 lanes doing work: the
            # lane-weighted VALU utilisation
            "lane_frac": None if lanes is None else round(frac * lanes / 64.0, 4),
            "source": t.get("source")}


def timed_ms(fn) -> float:
    """Kernel time of one render (rtp_stats.kernel_ms: HIP events on the
    launch's stream, synchronised)."""
    return float(fn().kernel_ms)


def scaling_anchors(dev, cam, stream) -> dict:
    """One-GPU kernel times of the multi-GPU workloads, on this GPU in this
    run: C4's whole frame through the tile instance its ranks use, and one
    rank's share of the C5 frame at N = 8 (2048 of 16384 spp on its derived
    stream), so that an N-GPU line of either workload can be read against
    the same workload on one GPU."""
    import torch

    out = {}
    c4 = WORKLOADS["c4"]
    n_tiles = -(-c4["nx"] // TILE) * -(-c4["ny"] // TILE)
    buf = torch.empty((TILE * TILE * n_tiles, 4), dtype=torch.float32, device="cuda")
    ms = timed_ms(lambda: dev.render_tiles_device(cam, c4["nx"], c4["ny"], c4["spp"], c4["depth"], buf.data_ptr(), 0, 1,
                                                  stream=stream, timed=True))
    smp = c4["nx"] * c4["ny"] * c4["spp"]
    out["c4_whole_frame"] = {"config": "1920x1080, 4096 spp, depth 50", "kernel_ms": round(ms, 2),
                             "msamples_per_s": round(smp / ms / 1e3, 1),
                             "launch": "tile instance, rank 0 of 1 (the instance every rank of a C4 run launches)"}
    del buf
    c5 = WORKLOADS["c5"]
    npix = c5["nx"] * c5["ny"]
    from raytracingtherestofyourlife_amd import shard

    b = shard.sample_batches(c5["spp"], 8, npix)[0]
    buf = torch.empty((npix, 4), dtype=torch.float32, device="cuda")
    ms = timed_ms(lambda: dev.render_device(cam, c5["nx"], c5["ny"], b.spp, c5["depth"], buf.data_ptr(),
                                            seed_base=b.seed_base, stream=stream, timed=True))
    out["c5_share_of_8"] = {"config": f"3840x2160, {b.spp} of 16384 spp (rank 0 of 8), depth 50",
                            "kernel_ms": round(ms, 2), "msamples_per_s": round(npix * b.spp / ms / 1e3, 1),
                            "one_gpu_frame_ms_est": round(8 * ms, 1),
                            "launch": "contiguous pixels, work stealing (the instance every rank of a C5 run launches)"}
    del buf
    torch.cuda.synchronize()
    return out


class Heartbeat:
    """Rank 0 prints `bench: <phase> (<s> s)` to stderr every `period` seconds
    (stdout keeps its one JSON line): a C5 run at N = 2 renders for minutes
    between its start and its line, and a silent process looks hung."""

    def __init__(self, enabled: bool, period: float = 30.0):
        self.phase = "setup"
        self.period = period
        self.t0 = time.perf_counter()
        self._stop = threading.Event()
        if enabled:
            threading.Thread(target=self._run, daemon=True).start()

    def _run(self):
        while not self._stop.wait(self.period):
            print(f"bench: {self.phase} ({time.perf_counter() - self.t0:.0f} s)", file=sys.stderr, flush=True)

    def stop(self):
        self._stop.set()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the one frame split over the ranks (tiles or sample batches); weak: a band per rank")
    ap.add_argument("--workload", default="auto", choices=["auto", "c2", "c4", "c5"],
                    help="auto: c2 on one GPU (the metric's frame), c5 on N > 1 (the sample-batch shard "
                         "configuration)")
    ap.add_argument("--nx", type=int, default=None, help="override the workload's width")
    ap.add_argument("--ny", type=int, default=None, help="rows of the frame (weak: per GPU, canvas nx x ny*N)")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--ff-tables", default="on", choices=["on", "auto", "off"],
                    help="RNG jump-table policy (include/rtp.h rtp_set_ff_tables); on: a long-lived renderer, "
                         "tables built during setup (reported in `setup`)")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work (0: skip)")
    ap.add_argument("--cpu-budget-mt", type=float, default=6.0, help="seconds of all-cores CPU baseline (0: skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL over xGMI, production); gloo: host-side reduce, for rehearsing N>1 on one GPU")
    ap.add_argument("--share-gpu", action="store_true", help="every rank uses device 0 (rehearsal on a 1-GPU box)")
    ap.add_argument("--check", action="store_true",
                    help="rank 0 verifies the reduced canvas against its own one-GPU render of the frame "
                         "(implied by --anchor on a process group)")
    ap.add_argument("--anchor", default="on", choices=["on", "off"],
                    help="process group: rank 0 renders the same workload's whole frame alone after the timed "
                         "region (one_gpu_same_workload, speedup_vs_one_gpu_same_workload, the checks)")
    ap.add_argument("--scaling-anchors", default="auto", choices=["auto", "on", "off"],
                    help="N = 1: time C4's whole frame and one C5 rank share on this GPU (auto: on for the "
                         "default c2 workload at its own size)")
    ap.add_argument("--force-collective", action="store_true",
                    help="create the process group and run the per-step reduce even on one rank (torchrun "
                         "--nproc-per-node 1: exercises the RCCL path on a one-GPU box)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_c2.json"))
    ap.add_argument("--valu-json", default=os.path.join(ROOT, "profiles", "valu_c2.json"))
    ap.add_argument("--golden", default=None, help="whole-frame fixture (c2), pixel-subset fixture (c4) or a "
                                                   "sample-shard fixture (c5)")
    ap.add_argument("--n1-launch", default="contig", choices=["contig", "tiles"],
                    help="one GPU, no process group: contig = the whole frame through the library's default launch "
                         "(rtp_render_device over [0, nx*ny), like main.cc's render); tiles = the tile-deal instance "
                         "the ranks of an N-GPU run use (rank 0 of 1)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: torch.distributed.run as a fresh child, before
        # anything here touches the GPU; never a one-GPU line for --gpus N
        raise SystemExit(self_launch(sys.argv[1:], args.gpus))

    import torch
    import torch.distributed as dist

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    workload = args.workload if args.workload != "auto" else ("c2" if world == 1 else "c5")
    W = WORKLOADS[workload]
    sized = all(getattr(args, k) is None for k in ("nx", "ny", "spp", "depth"))
    for k in ("nx", "ny", "spp", "depth"):
        if getattr(args, k) is None:
            setattr(args, k, W[k])
    golden_given = args.golden is not None
    if args.golden is None:
        args.golden = os.path.join(ROOT, "tests", "golden", W["golden"])
    beat = Heartbeat(rank == 0)
    gpu = 0 if args.share_gpu else local
    torch.cuda.set_device(gpu)
    if world > 1 or args.force_collective:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    grouped = dist.is_initialized()

    strong = args.scaling == "strong"
    nx, ny = args.nx, args.ny * (1 if strong else world)
    # one GPU without a process group renders the frame in pixel order through
    # the default contiguous launch (--n1-launch contig); ranks of a group
    # render their tiles (c2, c4, weak bands) or their sample batch (c5)
    contig = world == 1 and not (args.force_collective) and args.n1_launch == "contig"
    mode = "contig" if contig else (SHARD[workload] if strong else "tiles")
    samples = mode == "samples"
    spp_mine, seed_base = args.spp, 0
    if samples:
        b = shard.sample_batches(args.spp, world, nx * ny)[rank]
        spp_mine, seed_base = b.spp, b.seed_base
    ids_np = np.arange(nx * ny, dtype=np.int64) if mode in ("contig", "samples") else shard.tile_pixels(nx, ny, rank,
                                                                                                         world)
    npix = ids_np.size
    # setup, timed: the context, the scene, the RNG jump tables (policy), then
    # the first render -- what a fresh process pays before its first frame.
    # The HIP runtime's own first-use initialisation (~120 ms on the first
    # host-to-device copy of the process, r03j tools/scene_cost.py) is process
    # start, like the imports: one small copy takes it before the timer.
    torch.ones(1).cuda()
    torch.cuda.synchronize()
    t_setup = time.perf_counter()
    dev = rtp.Device(gpu)
    t_ctx = time.perf_counter()
    dev.set_cornell_box(0)
    t_scene = time.perf_counter()
    ff = dev.set_ff_tables(args.ff_tables)
    t_ff = time.perf_counter()
    cam = rtp.default_camera()
    ids = None if mode in ("contig", "samples") else torch.from_numpy(ids_np).cuda()
    out = torch.empty((npix, 4), dtype=torch.float32, device="cuda")
    canvas = torch.zeros((nx * ny, 4), dtype=torch.float32, device="cuda")
    live = torch.zeros(npix, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    # RCCL: the reduce of step k runs on the collective stream while step k+1
    # renders (shard.OverlappedCanvasReduce); gloo reduces host tensors.
    red = shard.OverlappedCanvasReduce(canvas, dist, overlap=(args.dist_backend == "nccl"),
                                       host_copy=(args.dist_backend != "nccl"), force=args.force_collective)

    # the rank's tiles: computed in the kernel (rtp_render_tiles_device; C4's
    # 1/8 share 263 vs 276 ms through the pixel list, profiles/r04y_*), which
    # renders clipped edge tiles whole (C4's 1080 rows: 0.7% more work, not
    # counted as samples): the entries inside the canvas are scattered
    # (shard.tile_entries).  RTP_BENCH_LIST=1: the explicit pixel list.
    tiled = mode == "tiles" and os.environ.get("RTP_BENCH_LIST") != "1"
    if tiled:
        ent_np, pix_np = shard.tile_entries(nx, ny, rank, world)
        assert np.array_equal(pix_np, ids_np)
        n_tiles = len(range(rank, -(-nx // TILE) * -(-ny // TILE), world))
        tile_out = torch.empty((TILE * TILE * n_tiles, 4), dtype=torch.float32, device="cuda")
        whole = ent_np.size == tile_out.shape[0]
        ent = None if whole else torch.from_numpy(ent_np).cuda()

    def gather_canvas():
        if tiled:
            return red.step(ids, tile_out if whole else tile_out.index_select(0, ent))
        return red.step(ids, out)

    def drain():
        red.drain()

    def render():
        if tiled:
            dev.render_tiles_device(cam, nx, ny, args.spp, args.depth, tile_out.data_ptr(), rank, world,
                                    stream=stream.cuda_stream)
        else:  # contiguous pixels (the whole frame, or a sample batch of it), or the pixel list
            dev.render_device(cam, nx, ny, spp_mine, args.depth, out.data_ptr(), pixel_count=npix,
                              pixel_ids_ptr=0 if ids is None else ids.data_ptr(), seed_base=seed_base,
                              stream=stream.cuda_stream)

    def step(count_live: bool = False):
        if count_live:  # (the list / contiguous path carries the per-pixel live-bounce counters)
            dev.render_device(cam, nx, ny, spp_mine, args.depth, out.data_ptr(), pixel_count=npix,
                              pixel_ids_ptr=0 if ids is None else ids.data_ptr(), seed_base=seed_base,
                              stream=stream.cuda_stream, live_ptr=live.data_ptr())
            return red.step(ids, out)
        render()
        return gather_canvas()

    # (the first frame after setup is timed on one GPU only: at N > 1 a C5
    # frame takes seconds, and the warmup renders it anyway)
    beat.phase = "first render and warmup"
    t_first = time.perf_counter()
    if world == 1:
        render()
    torch.cuda.synchronize()
    t_first_done = time.perf_counter()
    for i in range(args.warmup):  # the first also counts live bounces (for the byte model)
        step(count_live=(i == 0))
    if args.warmup == 0:
        step(count_live=True)
    drain()
    torch.cuda.synchronize()
    live_total = int(live.to(torch.int64).sum().item())

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    beat.phase = f"{args.steps} timed steps"
    t0 = time.perf_counter()
    for k in range(args.steps):
        # kernel duration bracketed on the stream the kernel is launched on
        ev[k][0].record(stream)
        render()
        ev[k][1].record(stream)
        canvas = gather_canvas()
    drain()
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if args.steps else float("nan")

    # ---- after the timed region: checks and the same-workload one-GPU anchor ----
    beat.phase = "checks and the one-GPU anchor"
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    quality = None
    parity = None
    gathered = None
    if samples:
        # (a) every rank's shard at the pixels of the oracle's reduced-frame
        # fixture of this world size (tools/make_golden_reduced.py), gathered
        # to rank 0 with the reduced frame there (reduced_frame_parity)
        fix = find_reduced_fixture(nx, ny, args.spp, args.depth, world,
                                   args.golden if golden_given else None)
        if fix is not None:
            mine = out.index_select(0, torch.from_numpy(fix["pixels"]).cuda()).to(coll_dev)
            if grouped and world > 1:
                parts = [torch.empty_like(mine) for _ in range(world)]
                dist.all_gather(parts, mine)
            else:
                parts = [mine]
            if rank == 0:
                red_px = canvas.index_select(0, torch.from_numpy(fix["pixels"]).cuda()).cpu().numpy()
                parity = reduced_frame_parity(fix, [q.cpu().numpy() for q in parts], red_px, args.spp)
        # (b) every rank's shard at a fixed pixel sample, gathered to rank 0
        # for the statistical comparison with the single-stream image
        chk = np.sort(np.random.default_rng(5).choice(nx * ny, min(C5_CHECK_PIXELS, nx * ny), replace=False))
        mine = out.index_select(0, torch.from_numpy(chk).cuda()).to(coll_dev)
        if grouped and world > 1:
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            gathered = [q.cpu().numpy() for q in parts]
        else:
            gathered = [mine.cpu().numpy()]

    one_gpu = None
    check = None
    want_anchor = grouped and args.anchor == "on"
    if rank == 0 and (want_anchor or args.check):
        # rank 0 renders the same workload's whole frame alone: the one-GPU
        # time of this workload (the others wait at the barrier below)
        # sample batches: the anchor renders on a stream no rank uses
        # (seed_base N*nx*ny), so the statistical check compares two
        # independent estimates (rank 0's batch IS the first spp/N samples of
        # the seed_base-0 stream)
        anchor_seed = (world * nx * ny) & 0xFFFFFFFF if samples else 0
        full = torch.empty((nx * ny, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        t_one = time.perf_counter()
        st = dev.render_device(cam, nx, ny, args.spp, args.depth, full.data_ptr(), seed_base=anchor_seed,
                               stream=stream.cuda_stream, timed=True)
        torch.cuda.synchronize()
        one_wall_ms = (time.perf_counter() - t_one) * 1e3
        one_ms = float(st.kernel_ms)
        one_gpu = {"kernel_ms": round(one_ms, 2), "wall_ms": round(one_wall_ms, 2),
                   "msamples_per_s": round(nx * ny * args.spp / one_ms / 1e3, 1),
                   "launch": "rank 0's GPU alone, the whole frame through the default contiguous launch"
                             + (f" on a stream no rank uses (seed_base {anchor_seed}; same pixels, samples and "
                                f"scene as the sharded frame)" if samples else "")}
        red_np = canvas[:, :3].cpu().numpy()
        if samples:
            single = full.index_select(0, torch.from_numpy(chk).cuda()).cpu().numpy()
            # the shards summed in float32 in the reduce's association (shard.tree_sum): exact
            summed = shard.tree_sum([q[:, :3] for q in gathered]).astype(np.float64)
            red_chk = red_np[chk].astype(np.float64)
            # the reduced frame against the single-stream image (shard.sample_shard_ttest: block means of the
            # per-pixel difference, Student-t); both estimate the same radiance
            stats = shard.sample_shard_ttest(single, red_chk, args.spp)
            fin = np.isfinite(summed) & np.isfinite(red_chk)
            rel = float(np.max(np.abs(red_chk[fin] - summed[fin]) / np.maximum(np.abs(summed[fin]), 1e-30))) \
                if fin.any() else 0.0
            check = {"pixels": int(chk.size),
                     "reduced_equals_sum_of_shards_max_rel": rel,
                     "nan_pattern_equal": bool(np.array_equal(np.isnan(red_chk), np.isnan(summed))),
                     "statistics_vs_single_stream": stats,
                     "consistent": shard.ttest_consistent(stats)}
        else:
            # the reduced canvas must equal one process rendering every pixel (bit-exact, NaN-aware)
            b_np = full[:, :3].cpu().numpy()
            same = (red_np.view(np.uint32) == b_np.view(np.uint32)) | (np.isnan(red_np) & np.isnan(b_np))
            check = bool(same.all())
        del full
    if grouped:
        dist.barrier()

    # a one-shot render on the library's default policy (AUTO: no jump tables
    # for a single C2 frame), as main.cc's rtp_render would run it: the whole
    # frame, tables switched off (one process: N = 1 only).  It runs through
    # the OTHER kernel instance than the timed renders (the tile deal when the
    # timed launch is contiguous, the contiguous launch when it is the tile
    # deal; the two render at rates within ~1%, r04q), so the rocprof
    # statistics of the timed instance stay the timed renders'.
    beat.phase = "one-shot render and scaling anchors"
    off_ms = float("nan")
    if world == 1:
        dev.set_ff_tables("off")
        full_off = torch.empty((nx * ny, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        t_off = time.perf_counter()
        if contig and nx % TILE == 0 and ny % TILE == 0:
            dev.render_tiles_device(cam, nx, ny, args.spp, args.depth, full_off.data_ptr(), 0, 1,
                                    stream=stream.cuda_stream)
        else:
            dev.render_device(cam, nx, ny, args.spp, args.depth, full_off.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize()
        off_ms = (time.perf_counter() - t_off) * 1e3
        del full_off
        dev.set_ff_tables(args.ff_tables)
    anchors = None
    if world == 1 and not grouped and (args.scaling_anchors == "on" or (
            args.scaling_anchors == "auto" and workload == "c2" and sized)):
        anchors = scaling_anchors(dev, cam, stream.cuda_stream)
    if rank == 0 and not samples:
        gold = load_golden_frame(args.golden)
        if gold and (gold["nx"], gold["ny"], gold["spp"], gold["depth"]) == (nx, ny, args.spp, args.depth):
            quality = frame_quality(canvas.cpu().numpy(), gold, args.spp)
    kernel_ms_max = kernel_ms
    if grouped:
        t = torch.tensor([elapsed, live_total, kernel_ms], dtype=torch.float64, device=coll_dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = t.clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0].item())
        kernel_ms_max = float(mx[2].item())
        live_all = float(tot[1].item())
    else:
        live_all = float(live_total)

    samples_rank = npix * spp_mine
    samples_all = nx * ny * args.spp
    value = samples_all * args.steps / elapsed / 1e6
    L = live_all / samples_all
    bytes_per_sample = 56.0 + 88.0 * L
    achieved = samples_rank * bytes_per_sample / (kernel_ms / 1e3) / 1e9
    cfg = {"nx": nx, "ny": args.ny, "spp": args.spp, "depth": args.depth}
    traffic = load_traffic(args.traffic_json, cfg) if world == 1 else None
    valu = load_valu(args.valu_json, cfg, kernel_ms) if world == 1 else None
    setup = {
        "context_ms": round((t_ctx - t_setup) * 1e3, 2),
        "scene_ms": round((t_scene - t_ctx) * 1e3, 2),
        "ff_tables_ms": round((t_ff - t_scene) * 1e3, 2),
        "ff_tables": {k: ff[k] for k in ("policy", "built", "chain_tables", "direct_first", "direct_count")}
                     | {"gib": round(ff["bytes"] / 2**30, 1), "alloc_ms": round(ff["alloc_ms"], 1),
                        "build_ms": round(ff["build_ms"], 1),
                        "render_ms_without": round(off_ms, 2) if world == 1 else None,
                        "per_rank": (f"every rank builds its own tables on its own GPU before its first frame "
                                     f"({round(ff['bytes'] / 2**30, 1)} GiB of each GPU's HBM; this line: rank 0's "
                                     f"setup)") if grouped else None},
    }
    first_ms = (t_first_done - t_first) * 1e3
    setup_base_ms = (t_scene - t_setup) * 1e3  # context + scene
    e2e_s = t_first_done - t_setup

    beat.phase = "CPU baseline"
    if rank == 0:
        cpu = cpu_mt = None
        if world == 1 and args.cpu_budget > 0:
            cpu = cpu_baseline(args.cpu_budget, args.nx, args.ny, args.depth)
        if world == 1 and args.cpu_budget_mt > 0:
            cpu_mt = cpu_baseline(args.cpu_budget_mt, args.nx, args.ny, args.depth, nthreads=host_threads())
        backend = "RCCL" if args.dist_backend == "nccl" else "gloo"
        if contig:
            shard_desc = "one GPU: the whole frame in pixel order (the default contiguous launch)"
        elif world == 1 and not grouped:
            shard_desc = "one GPU: the whole frame"
        elif samples:
            shard_desc = (f"sample batches: rank k renders spp/{world} samples of every pixel on the derived stream "
                          f"seed = pixel + k*{nx * ny} (shard.sample_batches), 1 {backend} reduce/step")
        else:
            shard_desc = (f"{TILE}x{TILE} tiles round-robin over {world} rank(s), 1 {backend} reduce/step"
                          + (" (pixel of each tile entry computed in-kernel)" if tiled else " (pixel list)"))
        ms_step = elapsed / max(args.steps, 1) * 1e3
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32 (f64 mixture/pdf islands)",
            "data": "synthetic: the reference's deterministic Cornell Box scene and camera (main.cc:616-622), "
                    "seed = pixel index" + (" + k*nx*ny on rank k (sample batches)" if samples else ""),
            "config": {
                "workload": W["name"] + ("" if strong or world == 1 else f" per GPU (canvas {nx}x{ny})"),
                "nx": nx, "ny": ny, "spp": args.spp, "depth": args.depth,
                "pixels_per_gpu": npix,
                "spp_per_gpu": spp_mine,
                "shard": shard_desc,
                "live_bounces_per_sample": round(L, 6),
                "dist_backend": args.dist_backend if grouped else None,
            },
            "rmse": quality["rmse"] if quality is not None else (
                parity["rmse"] if parity is not None else None),
            "bit_exact": quality["bit_exact"] if quality is not None else (
                parity["bit_exact"] if parity is not None else None),
            "quality": quality,
            "setup": setup,
            "first_render_ms": round(first_ms, 2) if world == 1 else None,
            "one_shot": None if world > 1 else {
                "note": "a fresh process rendering this frame once, like main.cc (its timer, :584-585, 661-663; "
                        "process start, imports and the HIP runtime's first-use initialisation excluded): "
                        "context + scene + jump-table policy + one render (its render through the other kernel "
                        "instance than the timed one: within ~1%)",
                "default_policy": {"policy": "auto (no tables for one frame)",
                                   "end_to_end_ms": round(setup_base_ms + off_ms, 1),
                                   "render_ms": round(off_ms, 1),
                                   "msamples_per_s": round(samples_all / ((setup_base_ms + off_ms) / 1e3) / 1e6, 1)},
                "bench_policy": {"policy": args.ff_tables, "end_to_end_ms": round(e2e_s * 1e3, 1),
                                 "msamples_per_s": round(samples_all / e2e_s / 1e6, 1)},
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic,
                "kernel_ms": round(kernel_ms, 3),
                "bytes_per_sample_model": round(bytes_per_sample, 3),
            },
            "roofline_valu": valu,
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_mt,
        }
        if anchors is not None:
            line["scaling_anchors"] = anchors
        if one_gpu is not None:
            line["one_gpu_same_workload"] = one_gpu
            # like for like: kernel time against the max-over-ranks kernel
            # time of a step, wall time against ms_per_step
            line["speedup_vs_one_gpu_same_workload"] = {
                "kernel": round(one_gpu["kernel_ms"] / kernel_ms_max, 3),
                "wall": round(one_gpu["wall_ms"] / ms_step, 3),
                "kernel_ms_max_over_ranks": round(kernel_ms_max, 3)}
        if samples:
            line["reduced_frame_parity"] = parity if parity is not None else (
                f"not checked: no committed reduced-frame fixture for {nx}x{ny}, {args.spp} spp, depth "
                f"{args.depth} at N = {world} (tools/make_golden_reduced.py)")
        if check is not None:
            line["check_reduced_canvas" + ("" if samples else "_equals_single_render")] = check
        beat.stop()
        print(json.dumps(line), flush=True)
    beat.stop()
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
