"""The dp headline's root share (rank 0 sheds the images its gather ingest costs it) never changes the
root's stream-lane or micro-batch count (round-4 ADVICE item 2): at 8 GPUs x 32
images the cost model sheds the root to 30, which split 1 lane against its peers' 2 and made
ScatterComputeGather raise before the first step. The lane split is pure arithmetic
(:func:`anx.models.alexnet_blocks.split_lanes`), so the shapes the driver's 8-GPU run uses are checked
here on CPU ranks over gloo with a fake two-lane model (the real lanes exist only on GPUs)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from anx.models.alexnet_blocks import LANE_MIN, split_lanes  # noqa: E402
from anx.parallel import cost  # noqa: E402
from anx.parallel.pipeline import micro_splits, root_batch_for  # noqa: E402


def test_split_lanes():
    assert split_lanes(1, 2) == [0, 1]
    assert split_lanes(2 * LANE_MIN - 1, 2) == [0, 2 * LANE_MIN - 1]
    assert split_lanes(2 * LANE_MIN, 2) == [0, LANE_MIN, 2 * LANE_MIN]
    assert split_lanes(128, 2) == [0, 64, 128]
    assert split_lanes(100, 3) == [0, 33, 66, 100]
    assert split_lanes(64, 1) == [0, 64]


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("batch", [1, 2, 16, 31, 32, 33, 40, 48, 64, 128, 256])
@pytest.mark.parametrize("lanes", [1, 2, 3])
@pytest.mark.parametrize("micro", [1, 2, 4])
def test_root_share_keeps_lanes_and_micro(world, batch, lanes, micro):
    bounds = lambda n: split_lanes(n, lanes)
    modelled = cost.dp_root_batch(world, batch)
    rb, note = root_batch_for(modelled, batch, micro, bounds)
    assert 1 <= rb <= batch
    assert len(bounds(rb)) == len(bounds(batch))
    assert len(micro_splits(rb, micro)) == len(micro_splits(batch, micro))
    assert (note is None) == (rb == modelled)
    assert rb >= modelled  # only ever raised: the shed the model prices is the most the root gives up


def test_root_share_the_crashing_shapes():
    """The shapes the verdict named: 8 ranks, 2 lanes, 32 and 40 images (30 and 38 before), and 1 image."""
    two = lambda n: split_lanes(n, 2)
    modelled = cost.dp_root_batch(8, 32)
    assert len(two(modelled)) - 1 == 1  # 30: what used to reach set_root_batch
    rb, note = root_batch_for(modelled, 32, 1, two)
    assert rb == 2 * LANE_MIN and note and len(two(rb)) - 1 == 2
    for batch in (40, 64, 128):  # shed shares that already keep two lanes pass through unchanged
        modelled = cost.dp_root_batch(8, batch)
        assert root_batch_for(modelled, batch, 1, two) == (modelled, None)
    assert root_batch_for(cost.dp_root_batch(8, 1), 1, 1, two) == (1, None)


class _FakeLanes:
    """Stands in for AlexNetBlocks(lanes=2) on CPU: forward_async splits like the GPU model and calls the
    pipeline's per-lane hooks, y = 2 x + 1."""

    def __init__(self, lanes=2):
        self.lanes = lanes

    def lane_bounds(self, n):
        return split_lanes(n, self.lanes)

    def __call__(self, x, out=None):
        out.copy_(2 * x + 1)
        return out

    def forward_async(self, x, y, on_lane=None, pre_lane=None):
        b = self.lane_bounds(x.shape[0])
        for i, (lo, hi) in enumerate(zip(b[:-1], b[1:])):
            if pre_lane is not None:
                pre_lane(i, lo, hi)
            y[lo:hi].copy_(2 * x[lo:hi] + 1)
            if on_lane is not None:
                on_lane(i, lo, hi)
        return y

    def join(self):
        pass


def _worker(rank, world, port, batch, q):
    sys.path.insert(0, ROOT)
    from anx.parallel import cost as c
    from anx.parallel.pipeline import PipelineConfig, ScatterComputeGather, root_batch_for as rbf
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        m = _FakeLanes(2)
        rb, _ = rbf(c.dp_root_batch(world, batch), batch, 1, m.lane_bounds)  # bench.py's path
        pipe = ScatterComputeGather(m, PipelineConfig(batch, micro=1, scatter=False, gather=True, prefetch=True,
                                                      async_lanes=True, root_batch=rb), (1, 1, 4), (1, 1, 4), "cpu")
        assert pipe.async_lanes and pipe.root_batch == rb
        for k in range(3):
            for xb in pipe._xb:
                xb.copy_(torch.arange(xb.numel(), dtype=torch.float32).view_as(xb) + 1000 * rank + k)
            pipe.step()
        pipe.drain()
        if rank == 0:
            ok = True
            for r in range(world):
                n = rb if r == 0 else batch
                x = torch.arange(n * 4, dtype=torch.float32).view(n, 1, 1, 4) + 1000 * r + 2
                ok &= torch.equal(pipe.y_global[r, :n], 2 * x + 1)
            q.put((rb, bool(ok)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batch", [32, 40, 1])
def test_root_share_pipeline_8_ranks_gloo(batch):
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    rb, ok = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok
    assert len(split_lanes(rb, 2)) == len(split_lanes(batch, 2))
