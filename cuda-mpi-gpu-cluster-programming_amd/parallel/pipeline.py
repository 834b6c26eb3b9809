"""Batch-parallel scatter -> compute -> gather pipeline over torch.distributed (RCCL on GPUs,
gloo on CPU ranks).

This is the reference's V4/V5 program shape — rank 0 owns the input, ``MPI_Scatterv`` rows out,
compute, ``MPI_Gatherv`` back (final_project/v4_mpi_cuda/src/main_mpi_cuda.cpp:52-130) — at
batch scale and MI355X-first:

* the decomposition axis is the batch (images are independent; no halo traffic at all), the
  row/halo decomposition of single images lives in :mod:`anx.parallel.strategies`;
* collectives are RCCL scatter/gather (grouped point-to-point from/to the root, one direct xGMI
  link per peer) issued asynchronously on RCCL's stream, split into micro-batches so the scatter
  of micro-batch i+1 and the gather of i-1 overlap the compute of i on the compute stream;
* buffers are allocated once and reused every step (the reference re-mallocs per call, D5).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


def micro_splits(B: int, M: int) -> list[tuple[int, int]]:
    M = max(1, min(M, B)) if B > 0 else 1
    sizes = [B // M + (1 if i < B % M else 0) for i in range(M)]
    out, lo = [], 0
    for s in sizes:
        out.append((lo, lo + s))
        lo += s
    return out


@dataclass
class PipelineConfig:
    batch_per_rank: int
    micro: int = 4
    scatter: bool = True   # rank 0 owns the global batch and scatters it
    gather: bool = True    # outputs are gathered to rank 0


class ScatterComputeGather:
    """One step: ``x_global[world, B, ...]`` (rank 0) -> per-rank ``model`` -> ``y_global`` (rank 0).

    ``model(x, out=y)`` must run asynchronously on the current stream (AlexNetBlocks does).
    """

    def __init__(self, model, cfg: PipelineConfig, in_shape, out_shape, device, group=None):
        self.model, self.cfg, self.device, self.group = model, cfg, torch.device(device), group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        B = cfg.batch_per_rank
        self.splits = micro_splits(B, cfg.micro if self.world > 1 else 1)
        self.x = torch.empty((B, *in_shape), device=self.device)
        self.y = torch.empty((B, *out_shape), device=self.device)
        # single rank: no scatter/gather buffers at all (the V3 shape: compute on resident data)
        root = self.rank == 0 and self.world > 1
        self.x_global = torch.empty((self.world, B, *in_shape), device=self.device) if root and cfg.scatter else None
        self.y_global = torch.empty((self.world, B, *out_shape), device=self.device) if root and cfg.gather else None

    def step(self) -> None:
        if self.world == 1:
            if self.x_global is not None:
                self.x.copy_(self.x_global[0])
            self.model(self.x, out=self.y)
            if self.y_global is not None:
                self.y_global[0].copy_(self.y)
            return
        root = self.rank == 0
        sw = []
        if self.cfg.scatter:
            for lo, hi in self.splits:
                src = [self.x_global[r, lo:hi] for r in range(self.world)] if root else None
                sw.append(dist.scatter(self.x[lo:hi], src, src=0, group=self.group, async_op=True))
        gw = []
        for i, (lo, hi) in enumerate(self.splits):
            if sw:
                sw[i].wait()
            self.model(self.x[lo:hi], out=self.y[lo:hi])
            if self.cfg.gather:
                dst = [self.y_global[r, lo:hi] for r in range(self.world)] if root else None
                gw.append(dist.gather(self.y[lo:hi], dst, dst=0, group=self.group, async_op=True))
        for w in gw:
            w.wait()
