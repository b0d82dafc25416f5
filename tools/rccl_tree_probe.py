"""Probe: shard.OverlappedCanvasReduce's tree over RCCL (nccl backend), one
rank per GPU (on an N-GPU node; RCCL refuses ranks that share a device:
"Duplicate GPU detected", profiles/r06q_tree_reduce_tests.txt).  Each rank's canvas holds
values spread over many binades; rank 0 compares the reduced canvas with
shard.tree_sum of all ranks' canvases bit for bit and prints one JSON line.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_tree_probe.py
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raytracingtherestofyourlife_amd import shard  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
gpu = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(gpu)
dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
n = 1 << 20


def part(r, step):
    g = np.random.default_rng(1000 * step + r)
    return (g.standard_normal((n, 4)) * 10.0 ** g.integers(-3, 4, (n, 4))).astype(np.float32)


canvas = torch.zeros((n, 4), dtype=torch.float32, device="cuda")
red = shard.OverlappedCanvasReduce(canvas, dist, overlap=True)
last = None
for step in range(4):
    last = red.step(None, torch.from_numpy(part(rank, step)).cuda())
red.drain()
torch.cuda.synchronize()
if rank == 0:
    got = last.cpu().numpy()
    want = shard.tree_sum([part(r, 3) for r in range(world)])
    print(json.dumps({"probe": "rccl tree reduce", "world": world, "elements": int(got.size),
                      "bit_exact": bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))}), flush=True)
dist.barrier()
dist.destroy_process_group()
