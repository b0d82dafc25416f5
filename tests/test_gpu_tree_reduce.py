"""shard.OverlappedCanvasReduce's device path (the one RCCL ranks run: the
tree's transfers and adds on a communication stream, an event the render
stream waits on before a canvas is reused) with real device asynchrony on
one GPU.  RCCL refuses two ranks on one device (profiles/
r06q_tree_reduce_tests.txt), so the ranks here are objects in one process
and the transfers go through an in-process hub with RCCL's stream
semantics: a send reads its buffer on the sender's current stream, a recv
makes the receiver's current stream wait for it.  Each step's partials come
from kernels still in flight on the render stream when the step is issued;
the steps are issued back to back, and rank 0's canvases of the last two
(one per slot of the double buffer) must hold their step's tree sum
(shard.tree_sum) bit for bit."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _Hub:
    def __init__(self):
        self.box = {}
        self.keep = []


class _RankView:
    """The slice of torch.distributed that OverlappedCanvasReduce and
    tree_reduce_ call, for one rank of the hub."""

    def __init__(self, hub, rank, world):
        self.hub, self.rank, self.world = hub, rank, world

    def is_initialized(self):
        return True

    def get_world_size(self):
        return self.world

    def get_rank(self):
        return self.rank

    def send(self, t, dst):
        import torch

        buf = t.clone()  # read on the sender's current stream (the transfer)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.hub.box.setdefault((self.rank, dst), []).append((buf, ev))

    def recv(self, t, src):
        import torch

        buf, ev = self.hub.box[(src, self.rank)].pop(0)
        torch.cuda.current_stream().wait_event(ev)
        t.copy_(buf)
        self.hub.keep.append(buf)  # (allocated on the sender's stream: kept until the test ends)


@pytest.mark.parametrize("world", [2, 4])
def test_overlapped_tree_reduce_on_device(world):
    import torch

    from raytracingtherestofyourlife_amd import shard

    n = 1 << 21
    hub = _Hub()
    reds = [shard.OverlappedCanvasReduce(torch.zeros((n, 4), dtype=torch.float32, device="cuda"),
                                         _RankView(hub, r, world), overlap=True) for r in range(world)]
    assert all(r.overlap and r.stream is not None for r in reds)
    g = torch.Generator(device="cuda")
    steps, hist = 6, []
    for step in range(steps):  # issued back to back: no host wait between steps
        parts = []
        for r in range(world):
            g.manual_seed(100 * step + r)
            # several kernels per partial, still running when the reduce is issued
            x = torch.randn((n, 4), device="cuda", generator=g)
            x = x * torch.pow(10.0, torch.randint(-3, 4, (n, 4), device="cuda", generator=g).float())
            parts.append(x)
        outs = [None] * world
        for r in reversed(range(world)):  # senders first (higher ranks), as their receivers expect
            outs[r] = reds[r].step(None, parts[r])
        hist.append((parts, outs[0]))
    for red in reds:
        red.drain()
    torch.cuda.synchronize()
    # the last two steps' canvases (one per slot of the double buffer): each
    # slot was reused twice under the tree reduces still running on it
    for parts, canvas in hist[-2:]:
        want = shard.tree_sum([p.cpu().numpy() for p in parts])
        got = canvas.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert hist[-1][1].data_ptr() != hist[-2][1].data_ptr()
    assert not any(hub.box.values())
