"""Benchmark of the path-tracing hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload auto|c2|c4] [--scaling strong|weak]

One step = one full render of the workload's frame.  On one GPU (no process
group) the frame goes through the library's default contiguous launch
(rtp_render_device over [0, nx*ny), like main.cc's render; --n1-launch tiles:
the tile-deal instance the ranks of an N-GPU run use).
  c2: Cornell Box 800x800, 1000 spp, depth 50 (BASELINE.json configs[1]), the
      metric's own image: the N = 1 workload (--workload auto).
  c4: Cornell Box 1920x1080, 4096 spp, depth 50 (BASELINE.json configs[3]),
      the configuration BASELINE.json names for the 2/4/8-GPU image-tile
      shard: the N > 1 workload (--workload auto).  On one GPU it renders at
      the same rate as C2 (5591 vs 5646 Msamples/s, r03z2), so the driver's
      N-GPU / 1-GPU ratio compares like with like.
N > 1 (launched by torch.distributed.run, one process per GPU):
  --scaling strong (default): THE frame, its 16x16 tiles dealt to the ranks
      round-robin; each rank renders 1/N of the pixels, and
      the float4 framebuffer is summed to rank 0 with ONE reduce per step
      (RCCL over xGMI), overlapped with the next step's render (two canvases,
      alternating; exact: every pixel is non-zero on one rank).
  --scaling weak: every rank renders a full nx x ny band of an nx x ny*N
      canvas (per-GPU work fixed).

Rank 0 prints one JSON line.  `value` = all ranks' samples / max-over-ranks
wall time of the K timed steps (steady state: the renderer's context, scene
and RNG jump tables are set up before the timed region -- `setup` and
`first_render_ms` report what that costs, and `one_shot` what a fresh process
rendering once, like main.cc, would see).  `rmse` / `bit_exact` compare the
last timed frame (normalised, NormalizeFunctor) with the oracle's committed
C2 frame (tests/golden/c2_full.npz).  `roofline` prices the render kernel with
the SoA byte model of SURVEY.md 8(d) (56 + 88*L bytes per sample) against the
8 TB/s HBM peak; `roofline_valu` gives the VALU-issue bound from the
committed PMC summary; `cpu_baseline` times the oracle's stage-structured
restatement on a bounded sample of the same workload on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
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
}


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


def load_golden_frame(path: str):
    """The oracle's committed fixture of the workload: tests/golden/c2_full.npz
    (tools/make_golden.py full_frame_fixture, every pixel: un-normalised rgb
    sums [N, 3]) or a pixel-subset fixture (c4_subset16k.npz: `pixels` and
    their sums), with its config; None if absent."""
    try:
        z = np.load(path, allow_pickle=False)
    except OSError:
        return None
    if "rgb_planes" in z.files:
        rgb, pixels = np.ascontiguousarray(z["rgb_planes"].T).view(np.float32).reshape(-1, 3), None
    else:
        rgb, pixels = np.asarray(z["rgb"], np.float32), np.asarray(z["pixels"], np.int64)
        if int(z["seed_base"]) != 0:
            return None
    return {"rgb": rgb, "pixels": pixels, "nx": int(z["nx"]), "ny": int(z["ny"]), "spp": int(z["spp"]),
            "depth": int(z["depth"])}


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
    return {"bound": "valu-issue", "achieved": t["valu_insts_per_launch"] / (kernel_ms / 1e3) / 1e12,
            "peak": t["simds"] * t["clock_ghz"] * 1e9 / t["cycles_per_wave64_valu"] / 1e12,
            "unit": "T wave64-VALU instr/s", "frac": round(frac, 4),
            "lanes_per_instr": t.get("lanes_per_instr"), "source": t.get("source")}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the one 800x800 frame dealt over the ranks; weak: an 800x800 band per rank")
    ap.add_argument("--workload", default="auto", choices=["auto", "c2", "c4"],
                    help="auto: c2 on one GPU (the metric's frame), c4 on N > 1 (the tile-shard configuration)")
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
    ap.add_argument("--check", action="store_true", help="rank 0 verifies the reduced canvas against a 1-process render")
    ap.add_argument("--force-collective", action="store_true",
                    help="create the process group and run the per-step reduce even on one rank (torchrun "
                         "--nproc-per-node 1: exercises the RCCL path on a one-GPU box)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_c2.json"))
    ap.add_argument("--valu-json", default=os.path.join(ROOT, "profiles", "valu_c2.json"))
    ap.add_argument("--golden", default=None, help="whole-frame fixture (c2) or pixel-subset fixture (c4)")
    ap.add_argument("--n1-launch", default="contig", choices=["contig", "tiles"],
                    help="one GPU, no process group: contig = the whole frame through the library's default launch "
                         "(rtp_render_device over [0, nx*ny), like main.cc's render); tiles = the tile-deal instance "
                         "the ranks of an N-GPU run use (rank 0 of 1)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import raytracingtherestofyourlife_amd as rtp
    from raytracingtherestofyourlife_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    workload = args.workload if args.workload != "auto" else ("c2" if world == 1 else "c4")
    W = WORKLOADS[workload]
    for k in ("nx", "ny", "spp", "depth"):
        if getattr(args, k) is None:
            setattr(args, k, W[k])
    if args.golden is None:
        args.golden = os.path.join(ROOT, "tests", "golden", W["golden"])
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
    # render their tiles
    contig = world == 1 and not (args.force_collective) and args.n1_launch == "contig"
    ids_np = np.arange(nx * ny, dtype=np.int64) if contig else shard.tile_pixels(nx, ny, rank, world)
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
    ids = torch.from_numpy(ids_np).cuda()
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
    tiled = (not contig) and os.environ.get("RTP_BENCH_LIST") != "1"
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
        if contig:
            dev.render_device(cam, nx, ny, args.spp, args.depth, out.data_ptr(), pixel_count=npix,
                              stream=stream.cuda_stream)
        elif tiled:
            dev.render_tiles_device(cam, nx, ny, args.spp, args.depth, tile_out.data_ptr(), rank, world,
                                    stream=stream.cuda_stream)
        else:
            dev.render_device(cam, nx, ny, args.spp, args.depth, out.data_ptr(), pixel_count=npix,
                              pixel_ids_ptr=ids.data_ptr(), stream=stream.cuda_stream)

    def step(count_live: bool = False):
        if count_live:  # (the list path carries the per-pixel live-bounce counters)
            dev.render_device(cam, nx, ny, args.spp, args.depth, out.data_ptr(), pixel_count=npix,
                              pixel_ids_ptr=0 if contig else ids.data_ptr(), stream=stream.cuda_stream,
                              live_ptr=live.data_ptr())
            return red.step(ids, out)
        render()
        return gather_canvas()

    t_first = time.perf_counter()
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
    check = None
    if args.check and rank == 0:
        # the reduced canvas must equal one process rendering every pixel (bit-exact, NaN-aware)
        full = torch.empty((nx * ny, 4), dtype=torch.float32, device="cuda")
        dev.render_device(cam, nx, ny, args.spp, args.depth, full.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize()
        a, b = canvas[:, :3].cpu().numpy(), full[:, :3].cpu().numpy()
        same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
        check = bool(same.all())
    # a one-shot render on the library's default policy (AUTO: no jump tables
    # for a single C2 frame), as main.cc's rtp_render would run it: the whole
    # frame, tables switched off (one process: N = 1 only).  It runs through
    # the OTHER kernel instance than the timed renders (the tile deal when the
    # timed launch is contiguous, the contiguous launch when it is the tile
    # deal; the two render at rates within ~1%, r04q), so the rocprof
    # statistics of the timed instance stay the timed renders'.
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
    quality = None
    if rank == 0:
        gold = load_golden_frame(args.golden)
        if gold and (gold["nx"], gold["ny"], gold["spp"], gold["depth"]) == (nx, ny, args.spp, args.depth):
            quality = frame_quality(canvas.cpu().numpy(), gold, args.spp)
    if grouped:
        t = torch.tensor([elapsed, live_total], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = t.clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0].item())
        live_all = float(tot[1].item())
    else:
        live_all = float(live_total)

    samples_rank = npix * args.spp
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
                        "render_ms_without": round(off_ms, 2) if world == 1 else None},
    }
    first_ms = (t_first_done - t_first) * 1e3
    setup_base_ms = (t_scene - t_setup) * 1e3  # context + scene
    e2e_s = t_first_done - t_setup

    if rank == 0:
        cpu = cpu_mt = None
        if world == 1 and args.cpu_budget > 0:
            cpu = cpu_baseline(args.cpu_budget, args.nx, args.ny, args.depth)
        if world == 1 and args.cpu_budget_mt > 0:
            cpu_mt = cpu_baseline(args.cpu_budget_mt, args.nx, args.ny, args.depth, nthreads=host_threads())
        if contig:
            shard_desc = "one GPU: the whole frame in pixel order (the default contiguous launch)"
        elif world == 1 and not grouped:
            shard_desc = "one GPU: the whole frame"
        else:
            shard_desc = (f"{TILE}x{TILE} tiles round-robin over {world} rank(s), 1 "
                          + ("RCCL" if args.dist_backend == "nccl" else "gloo") + " reduce/step")
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(args.steps, 1) * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32 (f64 mixture/pdf islands)",
            "data": "synthetic: the reference's deterministic Cornell Box scene and camera (main.cc:616-622), "
                    "seed = pixel index",
            "config": {
                "workload": W["name"] + ("" if strong or world == 1 else f" per GPU (canvas {nx}x{ny})"),
                "nx": nx, "ny": ny, "spp": args.spp, "depth": args.depth,
                "pixels_per_gpu": npix,
                "shard": shard_desc + ("" if contig else " (pixel of each tile entry computed in-kernel)" if tiled
                                       else " (pixel list)"),
                "live_bounces_per_sample": round(L, 6),
                "dist_backend": args.dist_backend if grouped else None,
            },
            "rmse": None if quality is None else quality["rmse"],
            "bit_exact": None if quality is None else quality["bit_exact"],
            "quality": quality,
            "setup": setup,
            "first_render_ms": round(first_ms, 2),
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
        if check is not None:
            line["check_reduced_canvas_equals_single_render"] = check
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
