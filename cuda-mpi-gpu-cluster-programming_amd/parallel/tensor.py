"""P7 tensor (filter) parallelism for AlexNet Blocks 1-2.

The reference only discusses "filter decomposition" (README.md:638,643). Here it is a working
strategy:

* Block 1 (Conv1 + ReLU + Pool1) is replicated on every rank. It is 19% of the FLOPs, and its
  output feeds every Conv2 filter.
* Conv2's K = 256 filters are split into contiguous shards, one per rank. A rank computes Conv2
  + ReLU + Pool2 for its filters only.
* LRN mixes channels c-2 .. c+2, so it needs a channel halo: each rank sends its first and last
  size//2 channels to its neighbours over torch.distributed P2P (RCCL over xGMI on GPUs).
* The shards are all-gathered along channels.

The result is bitwise equal to a single device running the same ops:

* Conv2 outputs are per-filter independent with a fixed k order.
* The zero channels at the global edges add exactly 0 to the LRN sums.

On MI355X this trades the row decomposition's spatial halos for a channel halo of
2 × N × 13 × 13 × 2 floats. The Conv2 weights (2.4 MB) are also split across ranks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops
from ..config import BLOCK1, BLOCK2, BlockSpec
from .comm import _p2p, world
from .plan import Rows


def filter_ranges(K: int, world_size: int) -> list[Rows]:
    """Contiguous filter shards, sizes differing by at most one (the first K % ws get one more)."""
    base, extra = divmod(K, world_size)
    out, lo = [], 0
    for r in range(world_size):
        hi = lo + base + (1 if r < extra else 0)
        out.append(Rows(lo, hi))
        lo = hi
    return out


def block1(x: torch.Tensor, w: dict, b1: BlockSpec = BLOCK1) -> torch.Tensor:
    """Conv1 + ReLU + Pool1 on every rank (replicated)."""
    c = b1.conv
    y = ops.conv2d(x, w["w1"], w["b1"], c.S, c.P, c.groups, relu=True)
    return ops.maxpool(y, b1.pool.F, b1.pool.S)


def shard_pool2(p1: torch.Tensor, w: dict, k: Rows, b2: BlockSpec = BLOCK2) -> torch.Tensor:
    """Conv2 filters [k.lo, k.hi) + ReLU + Pool2 -> [N, 13, 13, k.size]."""
    c = b2.conv
    if c.groups != 1:
        raise ValueError("filter parallelism shards ungrouped Conv2 only")
    w2 = w["w2"][k.lo:k.hi].contiguous()
    bias = w["b2"][k.lo:k.hi].contiguous()
    y = ops.conv2d(p1, w2, bias, c.S, c.P, 1, relu=True)
    return ops.maxpool(y, b2.pool.F, b2.pool.S)


def shard_lrn(p2: torch.Tensor, left: torch.Tensor, right: torch.Tensor, b2: BlockSpec = BLOCK2) -> torch.Tensor:
    """LRN of a channel shard given its h = size//2 halo channels on each side (zeros at the edges)."""
    h = b2.lrn.N // 2
    ext = torch.cat([left, p2, right], dim=3).contiguous()
    l = b2.lrn
    y = ops.lrn(ext, l.N, l.alpha, l.beta, l.k, l.mode)
    return y[..., h:h + p2.shape[3]].contiguous()


def filter_parallel_forward(x: torch.Tensor, w: dict, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2,
                            gather: str = "all", comm_device=None) -> torch.Tensor | None:
    """x: the full input [N,227,227,3] on every rank. Returns [N,13,13,K] on every rank
    (gather="all") or on rank 0 only (gather="root"; None elsewhere). ``comm_device`` stages the
    halo and gather traffic (e.g. "cpu" for the V4-style host-staged path over gloo); default: the
    compute device (RCCL for GPU tensors)."""
    rank, ws = world()
    K, h = b2.conv.K, b2.lrn.N // 2
    ranges = filter_ranges(K, ws)
    if min(r.size for r in ranges) < h:
        raise ValueError(f"filter parallelism needs >= {h} filters per rank (K={K}, world={ws})")
    k = ranges[rank]
    p2 = shard_pool2(block1(x, w, b1), w, k, b2)
    N, Ho, Wo, Ks = p2.shape
    cdev = torch.device(comm_device) if comm_device is not None else p2.device
    zeros = lambda: torch.zeros((N, Ho, Wo, h), device=cdev, dtype=p2.dtype)  # noqa: E731
    left, right = zeros(), zeros()
    if ws > 1:  # channel halo: my first h -> rank-1, my last h -> rank+1
        ops_ = []
        if rank > 0:
            ops_ += [dist.P2POp(dist.isend, p2[..., :h].to(cdev).contiguous(), rank - 1),
                     dist.P2POp(dist.irecv, left, rank - 1)]
        if rank < ws - 1:
            ops_ += [dist.P2POp(dist.isend, p2[..., Ks - h:].to(cdev).contiguous(), rank + 1),
                     dist.P2POp(dist.irecv, right, rank + 1)]
        _p2p(ops_)
    y = shard_lrn(p2, left.to(p2.device), right.to(p2.device), b2)
    if ws == 1:
        return y
    kmax = max(r.size for r in ranges)
    pad = torch.zeros((N, Ho, Wo, kmax), device=cdev, dtype=y.dtype)
    pad[..., :Ks] = y
    if gather == "root":
        bufs = [torch.empty_like(pad) for _ in range(ws)] if rank == 0 else None
        dist.gather(pad, bufs, dst=0)
        if rank != 0:
            return None
    else:
        bufs = [torch.empty_like(pad) for _ in range(ws)]
        dist.all_gather(bufs, pad)
    return torch.cat([b[..., :r.size] for b, r in zip(bufs, ranges)], dim=3).contiguous()


def simulate(x: torch.Tensor, w: dict, world_size: int, b1: BlockSpec = BLOCK1, b2: BlockSpec = BLOCK2):
    """All shards of a ``world_size``-way filter split in one process (halos passed in memory): the
    single-GPU rehearsal of :func:`filter_parallel_forward` used by the GPU tests."""
    K, h = b2.conv.K, b2.lrn.N // 2
    ranges = filter_ranges(K, world_size)
    p1 = block1(x, w, b1)
    p2s = [shard_pool2(p1, w, k, b2) for k in ranges]
    N, Ho, Wo, _ = p2s[0].shape
    z = torch.zeros((N, Ho, Wo, h), device=x.device)
    ys = []
    for r, p2 in enumerate(p2s):
        left = p2s[r - 1][..., -h:] if r > 0 else z
        right = p2s[r + 1][..., :h] if r < world_size - 1 else z
        ys.append(shard_lrn(p2, left.contiguous(), right.contiguous(), b2))
    return torch.cat(ys, dim=3).contiguous()
